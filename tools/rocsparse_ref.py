"""Known-good reference point (measurement only, never in the product): rocSPARSE dcsrmv
(adaptive, with analysis) on the same Kuhn matrix, cold and warm, HIP events."""
import ctypes as C, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, torch
from learningsparsepreconditioner4gpu_amd import problems as P

n = int(sys.argv[1]) if len(sys.argv) > 1 else 101
reps = 30
A = P.kuhn_laplacian(n)
rs = C.CDLL("/opt/rocm/lib/librocsparse.so")
h, descr, info = C.c_void_p(), C.c_void_p(), C.c_void_p()
assert rs.rocsparse_create_handle(C.byref(h)) == 0
assert rs.rocsparse_create_mat_descr(C.byref(descr)) == 0
assert rs.rocsparse_create_mat_info(C.byref(info)) == 0
m = A.shape[0]; nnz = A.nnz
val = torch.from_numpy(A.data).cuda(); ptr = torch.from_numpy(A.indptr.astype(np.int32)).cuda()
col = torch.from_numpy(A.indices.astype(np.int32)).cuda()
x = torch.randn(m, dtype=torch.float64, device="cuda"); y = torch.empty_like(x)
vp = lambda t: C.c_void_p(t.data_ptr())
assert rs.rocsparse_dcsrmv_analysis(h, 111, m, m, nnz, descr, vp(val), vp(ptr), vp(col), info) == 0
alpha, beta = C.c_double(1.0), C.c_double(0.0)
def run():
    assert rs.rocsparse_dcsrmv(h, 111, m, m, nnz, C.byref(alpha), descr, vp(val), vp(ptr), vp(col), info, vp(x), C.byref(beta), vp(y)) == 0
run(); torch.cuda.synchronize()
ref = A @ x.cpu().numpy()
err = np.abs(y.cpu().numpy() - ref).max() / np.abs(ref).max()
alg = 12 * nnz + 4 * (m + 1) + 16 * m
big = torch.ones(512 << 20 >> 2, dtype=torch.int32, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
cold = 0.0
for _ in range(reps):
    s = big.sum(); e0.record(); run(); e1.record(); e1.synchronize(); cold += e0.elapsed_time(e1)
cold /= reps
e0.record()
for _ in range(reps * 3): run()
e1.record(); e1.synchronize(); warm = e0.elapsed_time(e1) / (reps * 3)
print(f"rocsparse dcsrmv(adaptive) n={m} nnz={nnz} relerr={err:.1e} cold {cold*1e3:.1f} us {alg/cold/1e6:.0f} GB/s "
      f"warm {warm*1e3:.1f} us {alg/warm/1e6:.0f} GB/s", flush=True)
