"""Windows of small systems (n <= 2560, the one-workgroup bound): one workgroup per system in ONE
launch (LSPCG_BATCH_SMALL=1) vs the lockstep phases (=0) vs one solve at a time; K = 8 and 64
systems of Poisson-2D / Kuhn grids (1.0 k - 2.4 k unknowns), ext_spai with a spai-like L, rtol 1e-8."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from tests import _cases  # noqa: E402
from learningsparsepreconditioner4gpu_amd import problems as P  # noqa: E402
from learningsparsepreconditioner4gpu_amd.linalg import (BatchedConjugateGradient,  # noqa: E402
                                                         PreconditionedConjugateGradient)


def systems(K):
    out = []
    for k in range(K):
        if k % 2:
            out.append(P.kuhn_laplacian(10 + k % 4, 1e-2))
        else:
            nx = 32 + (k * 5) % 17
            out.append(P.poisson2d_grid(nx, 2400 // nx)[0])
    return out


def best_of(f, reps=3):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    return best, r


def main():
    eps, rtol = 3e-3, 1e-8
    for K in (8, 64):
        As = systems(K)
        Ls = [_cases.spai_like(A, seed=k) for k, A in enumerate(As)]
        bs = [torch.from_numpy(A @ np.ones(A.shape[0])).cuda() for A in As]
        xs = [torch.zeros_like(b) for b in bs]
        rec = {"systems": K, "n_max": max(A.shape[0] for A in As), "n_min": min(A.shape[0] for A in As)}
        for mode in ("1", "0"):
            os.environ["LSPCG_BATCH_SMALL"] = mode
            B = BatchedConjugateGradient(As, Ls, eps)
            B.solve(bs, xs, rtol)

            def run():
                for x in xs:
                    x.zero_()
                return B.solve(bs, xs, rtol)[0]

            t, res = best_of(run)
            rec[f"batch_small{mode}_ms"] = t * 1e3
            rec["iters_total"] = sum(r[0] for r in res)
            rec["iters_max"] = max(r[0] for r in res)
        solvers = []
        for A, L in zip(As, Ls):
            s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
            s.set_spai(L, eps)
            solvers.append(s)

        def seq():
            its = []
            for s, b, x in zip(solvers, bs, xs):
                x.zero_()
                its.append(s.solve(b, x, rtol)[0])
            return its

        seq()
        t, its = best_of(seq)
        rec["sequential_ms"] = t * 1e3
        rec["iters_equal"] = its == [r[0] for r in res]
        rec["us_per_iter_per_system_small1"] = rec["batch_small1_ms"] * 1e3 / rec["iters_total"]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
