"""SpMV probe on the bench matrix: bit-exactness vs scipy + cold/warm timing (GPU box)."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, torch
from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

n = int(sys.argv[1]) if len(sys.argv) > 1 else 101
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
A = P.kuhn_laplacian(n)
for dt, name in [(np.float64, "f64"), (np.float32, "f32")]:
    Ad = DeviceMatrix.from_scipy(A, dtype=dt)
    x = np.random.default_rng(0).normal(size=A.shape[0]).astype(dt)
    xt = torch.from_numpy(x).cuda()
    y = Ad.matvec(xt)
    ok = np.array_equal(y.cpu().numpy(), A.astype(dt) @ x)
    es = 8 if dt == np.float64 else 4
    alg = (es + 4) * A.nnz + 4 * (A.shape[0] + 1) + 2 * es * A.shape[0]
    cold = Ad.spmv_timed(xt, y, reps, 512 << 20)
    warm = Ad.spmv_timed(xt, y, reps * 3)
    print(f"{name} n={A.shape[0]} nnz={A.nnz} bitexact={ok} cold {cold*1e3:.1f} us {alg/cold/1e6:.0f} GB/s "
          f"warm {warm*1e3:.1f} us {alg/warm/1e6:.0f} GB/s", flush=True)

# ---- launch-configuration A/B (fp64), interleaved rounds in one process
import ctypes as C
from learningsparsepreconditioner4gpu_amd import _lib
lib = _lib.load()
Ad = DeviceMatrix.from_scipy(A, dtype=np.float64)
x = torch.randn(A.shape[0], dtype=torch.float64, device="cuda"); y = torch.empty_like(x)
nv = lib.lspcg_spmv_variant_timed(Ad.ctx.handle, Ad.handle, -1, None, None, 1, 0, None)
alg = 12 * A.nnz + 4 * (A.shape[0] + 1) + 16 * A.shape[0]
res = {v: ([], []) for v in range(nv)}
for rnd in range(3):
    for v in range(nv):
        ms = C.c_double()
        _lib.check(lib.lspcg_spmv_variant_timed(Ad.ctx.handle, Ad.handle, v, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 10, 512 << 20, C.byref(ms)))
        res[v][0].append(ms.value)
        _lib.check(lib.lspcg_spmv_variant_timed(Ad.ctx.handle, Ad.handle, v, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 30, 0, C.byref(ms)))
        res[v][1].append(ms.value)
for v in range(nv):
    c, w = np.median(res[v][0]), np.median(res[v][1])
    print(f"variant {v}: cold {c*1e3:.1f} us {alg/c/1e6:.0f} GB/s  warm {w*1e3:.1f} us {alg/w/1e6:.0f} GB/s", flush=True)
