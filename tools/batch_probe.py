"""Concurrent independent solves on one GPU: the heat_batch8 systems (C5, the reference's real
sizes) and 8 copies of poisson256 solved one after another vs from K host threads at once (each
solver owns a non-blocking stream; ctypes drops the GIL inside lspcg_solver_solve).  Prints the
whole-batch wall time and the effective us per iteration per system."""
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def main():
    sys.path.insert(0, ".")
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    sets = {"heat_batch8": synthetic_dataset("heat_batch8")}
    A_raw, mask, feats, bs, e2n = P.workload("poisson256")
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    sets["poisson256x8"] = [s] * 8
    for name, samples in sets.items():
        jobs = []
        for s in samples:
            ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], seed=0)
            d = s.to("cuda")
            L, _ = ws.inference_step(d)
            A = ws.system_matrix(d)
            b = A.matvec(d.mask.reshape(-1).to(torch.float64))
            solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
            solver.set_spai(L, ws.epsilon)
            x = torch.zeros_like(b)
            solver.solve(b, x, rtol=1e-6)  # graphs built, caches warm
            jobs.append((solver, b, x, A, L))
        torch.cuda.synchronize()

        def run(j):
            solver, b, x = j[0], j[1], j[2]
            x.zero_()
            it, conv, _ = solver.solve(b, x, rtol=1e-6)
            return it

        for K in (1, 2, 4, 8):
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if K == 1:
                    its = [run(j) for j in jobs]
                else:
                    with ThreadPoolExecutor(K) as ex:
                        its = list(ex.map(run, jobs))
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None or dt < best else best
            tot = sum(its)
            rec = {"set": name, "threads": K, "systems": len(jobs), "iters_total": tot, "wall_ms": best * 1e3,
                   "us_per_iter_per_system": best * 1e6 / tot, "max_iters": max(its)}
            print(json.dumps(rec), flush=True)
        # the same systems as ONE lockstep batch (linalg.BatchedConjugateGradient)
        from learningsparsepreconditioner4gpu_amd.linalg import BatchedConjugateGradient

        import os

        for rtol, red in ((1e-6, "auto"), (1e-8, "auto"), (1e-8, "0"), (1e-8, "1")):
            if red == "auto":
                os.environ.pop("LSPCG_BATCH_REDUCE", None)
            else:
                os.environ["LSPCG_BATCH_REDUCE"] = red
            B = BatchedConjugateGradient([j[3] for j in jobs], [j[4] for j in jobs], ws.epsilon)
            bs = [j[1] for j in jobs]
            xs = [torch.zeros_like(b) for b in bs]
            B.solve(bs, xs, rtol=rtol)  # graphs built
            best, its = None, None
            for _ in range(3):
                for x in xs:
                    x.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res, _ = B.solve(bs, xs, rtol=rtol)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None or dt < best else best
                its = [r[0] for r in res]
            ref = []
            for j in jobs:
                x = torch.zeros_like(j[1])
                ref.append(j[0].solve(j[1], x, rtol=rtol)[0])
            tot = sum(its)
            rec = {"set": name, "mode": "batch", "reduce": red, "rtol": rtol, "systems": len(jobs), "iters_total": tot,
                   "wall_ms": best * 1e3, "us_per_iter_per_system": best * 1e6 / tot, "max_iters": max(its),
                   "us_per_lockstep_iter": best * 1e6 / max(its), "iters_equal_single": its == ref}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
