"""Solver setup split (measurement only, GPU box): PreconditionedConjugateGradient(A) creation and
set_spai, host clock around each with the device drained, three solvers per workload.

    LSPCG_REORDER_PROFILE=1 python tools/create_probe.py delaunay27k [kuhn41 ...]
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
    for wl in sys.argv[1:] or ["delaunay27k"]:
        A_raw, mask, feats, bs, e2n = P.workload(wl)
        smp = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
        d = smp.to("cuda")
        ws = SimpleInferenceWorkspace(node_features=smp.x.shape[1], edge_features=smp.edge_attr.shape[1],
                                      block_size=bs, seed=0)
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d)
        rows = []
        for r in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            s.set_spai(L, 3e-3, block_size=bs)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append({"create_ms": (t1 - t0) * 1e3, "set_spai_ms": (t2 - t1) * 1e3, "views": s.views["A"]["columns"],
                         "reorder": s.reorder_info["applied"]})
            del s
        print(json.dumps({wl: rows}), flush=True)


if __name__ == "__main__":
    main()
