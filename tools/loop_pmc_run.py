"""A short PCG loop on a named workload for PMC passes (tools/pmc_run.sh ... -- FETCH_SIZE WRITE_SIZE;
tools/loop_traffic.py then reads the per-dispatch counters): the bench's GNN-L ext_spai solver,
3 solves of at most `iters` iterations each.  Prints one JSON line with the config fields
loop_traffic.py reads.

    python tools/loop_pmc_run.py delaunay1m [iters]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.data import make_sample
from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "delaunay1m"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    A_raw, mask, feats, bs, e2n = P.workload(wl)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs,
                                  seed=0)
    d = s.to("cuda")
    L, _ = ws.inference_step(d)
    A = ws.system_matrix(d)
    b = A.matvec(d.mask.reshape(-1).to(torch.float64))
    sol = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
    sol.set_spai(L, ws.epsilon, block_size=bs)
    x = torch.zeros_like(b)
    for _ in range(3):
        x.zero_()
        it, conv, t = sol.solve(b, x, rtol=1e-8, max_iter=iters)
    torch.cuda.synchronize()
    print(json.dumps({"config": {"workload": f"{wl}: ext_spai loop, {iters} iterations x 3", "n": A.n,
                                 "nnz_A": A.nnz}, "views": sol.views, "iters": it}), flush=True)


if __name__ == "__main__":
    main()
