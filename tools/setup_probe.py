"""Per-sample costs of a new L on the same solver (measurement only, GPU box): set_spai time and the
first solve after it (graph capture for every chunk size, allocations) vs a repeated solve.

    python tools/setup_probe.py [workload] [samples]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.data import make_sample
from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "kuhn101"
    samples = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    A_raw, mask, feats, bs, e2n = P.workload(wl)
    smp = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    d = smp.to("cuda")
    A = None
    s = None
    rows = []
    for k in range(samples):
        ws = SimpleInferenceWorkspace(node_features=smp.x.shape[1], edge_features=smp.edge_attr.shape[1],
                                      block_size=bs, epsilon=3e-3, seed=k)  # a new L per sample
        L, _ = ws.inference_step(d)
        if A is None:
            A = ws.system_matrix(d)
            b = A.matvec(d.mask.reshape(-1).to(torch.float64))
            s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev = s.set_spai(L, 3e-3, block_size=bs)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = []
        for r in range(3):
            x = torch.zeros_like(b)
            t2 = time.perf_counter()
            it, conv, sec = s.solve(b, x, rtol=1e-8)
            torch.cuda.synchronize()
            res.append({"iters": it, "solve_ms": sec * 1e3, "wall_ms": (time.perf_counter() - t2) * 1e3})
        rows.append({"sample": k, "set_spai_ms": (t1 - t0) * 1e3, "device_ms": dev * 1e3, "solves": res})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
