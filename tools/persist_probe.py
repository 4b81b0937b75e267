"""µs per PCG iteration of the persistent one-launch solve (k_pcg_persist) against the 5-launch
split schedule, on the mid-size systems the reference actually solves (C5 heat batch, 900 -
30 k unknowns; C2 Poisson 65 k) and a few larger ones.  For each system and variant: a fresh
solver (the environment is read at creation), one warm-up solve, then the median of 5 solves;
us_per_iter = solve time / iterations.  Also checks that every variant returns the split
schedule's iteration count and iterate bit for bit.

    python tools/persist_probe.py [--workloads heat_batch8,poisson256,kuhn41] > out.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

VARIANTS = {
    "split": {"LSPCG_PERSIST_N": "0"},
    "persist256": {"LSPCG_PERSIST_N": "100000000", "LSPCG_PERSIST_WG": "256"},
    "persist128": {"LSPCG_PERSIST_N": "100000000", "LSPCG_PERSIST_WG": "128"},
    "persist64": {"LSPCG_PERSIST_N": "100000000", "LSPCG_PERSIST_WG": "64"},
}


def systems(names):
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset

    for name in names:
        if name == "heat_batch8":
            for i, s in enumerate(synthetic_dataset("heat_batch8")):
                yield f"heat{i}", s
        else:
            A_raw, mask, feats, bs, e2n = P.workload(name)
            yield name, make_sample(A_raw, mask, node_features=feats, block_size=bs,
                                    use_edge_features_as_node_feature=e2n)


def main():
    sys.path.insert(0, ".")
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="heat_batch8,poisson256,kuhn41,kuhn61")
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    os.environ["LSPCG_SMALL_N"] = "0"
    for name, s in systems(args.workloads.split(",")):
        ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1],
                                      block_size=s.block_size, seed=0)
        d = s.to("cuda")
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d)
        b = A.matvec(d.mask.reshape(-1).to(torch.float64))
        rec = {"system": name, "n": A.n, "nnz": A.nnz}
        ref = None
        for v, env in VARIANTS.items():
            os.environ.update(env)
            solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
            solver.set_spai(L, ws.epsilon, block_size=L.block_size)
            x = torch.zeros_like(b)
            solver.solve(b, x, rtol=args.rtol)
            ts = []
            for _ in range(args.reps):
                x.zero_()
                it, conv, t = solver.solve(b, x, rtol=args.rtol)
                ts.append(t)
            xs = x.cpu().numpy()
            if ref is None:
                ref = (it, xs)
            same = it == ref[0] and np.array_equal(xs, ref[1])
            ms = float(np.median(ts)) * 1e3
            rec[v] = {"iters": it, "solve_ms": ms, "us_per_iter": ms * 1e3 / max(it, 1), "same_bits_as_split": bool(same)}
            del solver
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
