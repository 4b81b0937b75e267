"""Measurement only (GPU box): the one-workgroup solve (k_pcg_small) against the 5-kernel schedule on
the systems inside its n bound -- C5's heat and Delaunay datasets and Kuhn grids -- one JSON line per
system: n, nnz(A), nnz(L), iterations and the steady per-iteration time of both paths (best of 3
full solves after a warm-up; LSPCG_SMALL_N=0 selects the 5-kernel schedule at solver creation).

    python tools/small_cut_probe.py [heat_batch8 delaunay_batch8 kuhn ...]
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def systems(name):
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    if name == "kuhn":
        samples = []
        for k in (8, 10, 12, 13):
            A_raw, mask, feats, bs, e2n = P.workload(f"kuhn{k}")
            samples.append(make_sample(A_raw, mask, node_features=feats, block_size=bs,
                                       use_edge_features_as_node_feature=e2n))
    else:
        samples = synthetic_dataset(name)
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=samples[0].edge_attr.shape[1],
                                  seed=0)
    for smp in samples:
        d = smp.to("cuda")
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d)
        b = A.matvec(d.mask.reshape(-1).to(torch.float64))
        yield A, L, b, ws.epsilon


def per_iter(A, L, b, eps, small_n):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    os.environ["LSPCG_SMALL_N"] = str(small_n)
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
    s.set_spai(L, eps)
    x = torch.zeros_like(b)
    s.solve(b, x, rtol=1e-8)
    best, it = None, 0
    for _ in range(3):
        x.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it, conv, _ = s.solve(b, x, rtol=1e-8)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    return int(it), best * 1e6 / max(int(it), 1)


def main():
    for name in sys.argv[1:] or ["heat_batch8", "delaunay_batch8", "kuhn"]:
        for A, L, b, eps in systems(name):
            if A.shape[0] > 2560:
                continue
            it1, us1 = per_iter(A, L, b, eps, 3072)
            it0, us0 = per_iter(A, L, b, eps, 0)
            print(json.dumps({"set": name, "n": int(A.shape[0]), "nnz_A": int(A.nnz), "nnz_L": int(L.nnz),
                              "iters": [it1, it0], "us_small": us1, "us_5kernel": us0}), flush=True)
    os.environ.pop("LSPCG_SMALL_N", None)


if __name__ == "__main__":
    main()
