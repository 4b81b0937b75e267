"""BSR 3x3 SpMV on the C4 elasticity stand-in: staged block kernel vs the BSELL-64 copy, cold
(Infinity Cache evicted) and warm, against SURVEY 8(d)'s BSR bytes.  Run once per
LSPCG_BSELL_QB setting (read once per process)."""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, ".")
from bench import FLUSH_BYTES, HBM_PEAK_GBS, bsr3_bytes  # noqa: E402
from learningsparsepreconditioner4gpu_amd import problems as P  # noqa: E402
from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix, assemble  # noqa: E402

A, mask, _ = P.elasticity_box()
g = P.to_block_graph(A, 3)
Ad = assemble(torch.from_numpy(g.edge_index).cuda(), torch.from_numpy(g.block_values).cuda(), A.shape[0],
              torch.from_numpy(mask.reshape(-1)).cuda(), block_output=True)
n = Ad.n
x = torch.randn(n, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
alg = bsr3_bytes(n // 3, Ad.nnzb)
staged = Ad.spmv_timed(x, y, 30, flush_bytes=FLUSH_BYTES)
kind = Ad.prepare_spmv()
cold = Ad.spmv_timed(x, y, 30, flush_bytes=FLUSH_BYTES)
warm = Ad.spmv_timed(x, y, 90)
print(json.dumps({"qb": os.environ.get("LSPCG_BSELL_QB", "2"), "n": n, "nnzb": Ad.nnzb, "alg_bytes": alg, "kind": kind,
                  "staged_cold_us": staged * 1e3, "bsell_cold_us": cold * 1e3, "bsell_warm_us": warm * 1e3,
                  "frac_cold": alg / (cold * 1e-3) / 1e9 / HBM_PEAK_GBS}), flush=True)
