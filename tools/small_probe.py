"""Per-iteration time of the one-workgroup solve (k_pcg_small) vs the multi-kernel schedule on a
small heat system: solves with rtol = 0 and max_iter = K; the slope over K is the iteration
time, the intercept the per-solve fixed cost.

    python tools/small_probe.py [system index in heat_batch8]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    idx = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    s = synthetic_dataset("heat_batch8")[idx]
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], seed=0)
    d = s.to("cuda")
    L, _ = ws.inference_step(d)
    A = ws.system_matrix(d)
    b = A.matvec(d.mask.reshape(-1).to(torch.float64))
    for small in ("0", "4096"):
        os.environ["LSPCG_SMALL_N"] = small
        solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
        solver.set_spai(L, ws.epsilon)
        rec = {"n": A.n, "small_n": small}
        for K in (1, 50, 200, 400, 1, 50, 200, 400):
            x = torch.zeros_like(b)
            it, conv, t = solver.solve(b, x, rtol=0.0, max_iter=K)
            torch.cuda.synchronize()
            rec[f"K{K}"] = round(t * 1e3, 4)
        ks = np.array([1, 50, 200, 400], dtype=float)
        ts = np.array([rec[f"K{k}"] for k in (1, 50, 200, 400)])
        slope, icpt = np.polyfit(ks, ts, 1)
        rec["us_per_iter"] = slope * 1e3
        rec["fixed_ms"] = icpt
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
