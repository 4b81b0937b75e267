"""PCG A/B probe on the bench system (GPU box): CSR-staged vs SELL iteration views.

Builds the bench workload once (kuhn101, GNN-inferred L), then for each variant creates a
solver (env switches are read at solver creation), solves `reps` times and reports the
iteration count, time per iteration and whether x and the residual history are bit-identical
to the first variant.  Also times the standalone SELL SpMV of A against the CSR kernel.

    python tools/pcg_probe.py [workload] [reps]
"""
import ctypes as C
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from learningsparsepreconditioner4gpu_amd import _lib
from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.data import make_sample
from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

wl = sys.argv[1] if len(sys.argv) > 1 else "kuhn101"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
A_raw, mask, feats, bs, e2n = P.workload(wl)
s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs, seed=0)
ds = s.to("cuda")
L, _ = ws.inference_step(ds)
A = ws.system_matrix(ds)
gt = ds.mask.reshape(-1).to(torch.float64)
b = A.matvec(gt)
print(f"{wl}: n={A.n} nnz={A.nnz}", flush=True)

VARIANTS = [("csr", {"LSPCG_NO_SELL": "1"}),
            ("ticket16", {"LSPCG_NO_SELL": "0", "LSPCG_SPLIT_REDUCE": "0"}),
            ("split16", {"LSPCG_NO_SELL": "0", "LSPCG_SPLIT_REDUCE": "1"})]
if os.environ.get("PROBE_VARIANTS") == "cap":
    VARIANTS = [("ticket16", {"LSPCG_NO_SELL": "0", "LSPCG_SPLIT_REDUCE": "0"}),
                ("split16", {"LSPCG_NO_SELL": "0", "LSPCG_SPLIT_REDUCE": "1"})]
ref = None
for name, env in VARIANTS:
    os.environ.update(env)
    for k, v in env.items():
        if v == "":
            os.environ.pop(k, None)
    solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
    solver.set_spai(L, 3e-3, block_size=L.block_size)
    ts = []
    for _ in range(reps):
        x = torch.zeros_like(b)
        it, conv, sec, hist = solver.solve(b, x, rtol=1e-8, max_iter=int(os.environ.get("PROBE_MAXIT", "0")),
                                           return_history=True)
        ts.append(sec)
    t = float(np.median(ts))
    same = ""
    if ref is None:
        ref = (x.clone(), hist.copy(), it)
    else:
        same = f" x_bitexact={torch.equal(x, ref[0])} hist_bitexact={np.array_equal(hist, ref[1])} iters_equal={it == ref[2]}"
    print(f"{name:6s}: iters={it} conv={conv} solve {t*1e3:.3f} ms  {t/it*1e6:.2f} us/iter  {it/t:.0f} it/s{same}", flush=True)
    del solver

if os.environ.get("PROBE_VARIANTS") == "cap":
    sys.exit(0)
lib = _lib.load()
x = torch.randn(A.n, dtype=torch.float64, device="cuda")
y0 = torch.empty_like(x)
y1 = torch.empty_like(x)
alg = 12 * A.nnz + 4 * (A.n + 1) + 16 * A.n
for label, flush in (("cold", 512 << 20), ("warm", 0)):
    r = 30 if flush else 90
    ms0 = A.spmv_timed(x, y0, r, flush_bytes=flush)
    out = [f"csr {ms0*1e3:.1f} us ({alg/ms0/1e6:.0f} GB/s)"]
    for compact in (0, 2, 1, 3, 7):
        ms = C.c_double()
        _lib.check(lib.lspcg_spmv_sell_timed(A.ctx.handle, A.handle, compact, C.c_void_p(x.data_ptr()),
                                             C.c_void_p(y1.data_ptr()), r, flush, C.byref(ms)))
        out.append(f"sell{['', '-f32val', '-c16', '-f32val-c16', '', '', '', '-f32val-c16-pairgather'][compact]} {ms.value*1e3:.1f} us ({alg/ms.value/1e6:.0f} GB/s) "
                   f"bitexact={torch.equal(y0, y1)}")
    print(f"SpMV {label}: " + " | ".join(out), flush=True)
    rd = []
    for nbytes in (alg, 115 << 20):
        ms = C.c_double()
        _lib.check(lib.lspcg_read_timed(A.ctx.handle, int(nbytes), r, flush, C.byref(ms)))
        rd.append(f"read {nbytes/1e6:.0f} MB {ms.value*1e3:.1f} us ({nbytes/ms.value/1e6:.0f} GB/s)")
    print(f"stream {label}: " + " | ".join(rd), flush=True)
