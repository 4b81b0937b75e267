"""Reorder analysis timing on the bench's irregular systems (measurement only, GPU box):
DeviceMatrix.rcm() alone, solver creation and set_spai with LSPCG_REORDER=1 / 0.

    LSPCG_REORDER_PROFILE=1 python tools/rcm_probe.py [kuhn101rand]
"""
import json
import os
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
    wl = sys.argv[1] if len(sys.argv) > 1 else "kuhn101rand"
    A_raw, mask, feats, bs, e2n = P.workload(wl)
    smp = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=smp.x.shape[1], edge_features=smp.edge_attr.shape[1], block_size=bs,
                                  epsilon=3e-3, seed=0)
    d = smp.to("cuda")
    L, _ = ws.inference_step(d)
    A = ws.system_matrix(d)
    torch.cuda.synchronize()
    out = {"workload": wl, "n": A.n}
    for r in range(3):
        t0 = time.perf_counter()
        perm, before, after = A.rcm()
        torch.cuda.synchronize()
        out.setdefault("rcm_ms", []).append((time.perf_counter() - t0) * 1e3)
    for mode in ("1", "0", "1"):
        os.environ["LSPCG_REORDER"] = mode
        t0 = time.perf_counter()
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
        t1 = time.perf_counter()
        s.set_spai(L, 3e-3, block_size=bs)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out.setdefault(f"reorder{mode}", []).append({"create_ms": (t1 - t0) * 1e3, "set_spai_ms": (t2 - t1) * 1e3})
        del s
    print(json.dumps(out))


if __name__ == "__main__":
    main()
