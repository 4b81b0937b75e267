"""Launch-configuration sweep of the SELL-DIA SpMV (tools/sell_sweep.hip; diagnostics, not the product):
every (value type, slots per batch, MINW) configuration on the bench matrix, cold and warm, checked bit for bit
against the product's lspcg_spmv on the same SELL copy.

    python tools/sell_sweep.py --build          # in the container: hipcc -> tools/_sweep/libsellsweep.so
    python tools/sell_sweep.py [workload]       # on the GPU box: one JSON line per configuration
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "_sweep", "libsellsweep.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    pkg = os.path.join(ROOT, "learningsparsepreconditioner4gpu_amd")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950", "-ffp-contract=off",
           "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "sell_sweep.hip"), "-L" + pkg, "-llspcg_hip",
           "-Wl,-rpath," + pkg, "-o", LIB]
    print(" ".join(cmd))
    subprocess.check_call(cmd)


def main_bsr():
    """BSELL-64 block slots per batch on the C4 elasticity system (BSR 3x3)."""
    sys.path.insert(0, ROOT)
    import numpy as np
    import scipy.sparse as sp
    import torch

    from bench import FLUSH_BYTES, bsr3_bytes
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A_raw, _, _, _, _ = P.workload("elast")
    B = sp.bsr_matrix(sp.csr_matrix(A_raw), blocksize=(3, 3))
    B.sort_indices()
    B.data = B.data.astype(np.float32).astype(np.float64)
    ref = DeviceMatrix.from_scipy(sp.csr_matrix(B)).matvec
    lib = C.CDLL(LIB)
    rp = torch.from_numpy(B.indptr.astype(np.int32)).cuda()
    ci = torch.from_numpy(B.indices.astype(np.int32)).cuda()
    va = torch.from_numpy(np.ascontiguousarray(B.data)).cuda()
    n = B.shape[0]
    x = torch.randn(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    want = ref(x)
    alg = bsr3_bytes(n // 3, B.indices.size)
    p = lambda t: C.c_void_p(t.data_ptr())
    for cid in range(lib.sweep_bsr_count()):
        vb, qb = C.c_int(), C.c_int()
        lib.sweep_bsr_cfg(cid, C.byref(vb), C.byref(qb))
        cold, warm = C.c_double(), C.c_double()
        y.fill_(float("nan"))
        rc = lib.sweep_bsr_run(cid, C.c_int64(n // 3), C.c_int64(B.indices.size), p(rp), p(ci), p(va), p(x), p(y), 20,
                               C.c_int64(FLUSH_BYTES), C.byref(cold), C.byref(warm))
        code = qb.value  # qb | 100 * (3: three waves per slice) | 1000 * MINW
        print(json.dumps({"workload": "elast BSR3", "values": "fp64" if vb.value == 8 else "fp32", "QB": code % 100,
                          "waves_per_slice": 3 if (code // 100) % 10 == 3 else 1, "minw": code // 1000,
                          "rc": rc, "cold_us": cold.value * 1e3, "warm_us": warm.value * 1e3,
                          "frac_alg_cold": alg / (cold.value * 1e-3) / 8e12, "bitexact": bool(torch.equal(y, want))}),
              flush=True)


def main_quad(wl):
    """SELL-DIA with quad-interleaved fp32 values (16-B value loads) against the slot-major kernel."""
    sys.path.insert(0, ROOT)
    import numpy as np
    import scipy.sparse as sp
    import torch

    from bench import FLUSH_BYTES, spmv_bytes
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A_raw, _, _, _, _ = P.workload(wl)
    A = sp.csr_matrix(A_raw)
    A.sort_indices()
    A.data = A.data.astype(np.float32).astype(np.float64)
    lib = C.CDLL(LIB)
    rp = torch.from_numpy(A.indptr.astype(np.int32)).cuda()
    ci = torch.from_numpy(A.indices.astype(np.int32)).cuda()
    va = torch.from_numpy(A.data).cuda()
    x = torch.randn(A.shape[0], dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    ref = DeviceMatrix.from_scipy(A).matvec(x)
    alg = spmv_bytes(A.shape[0], A.nnz)
    p = lambda t: C.c_void_p(t.data_ptr())
    for qpb in (2, 4):
        cold, warm = C.c_double(), C.c_double()
        y.fill_(float("nan"))
        rc = lib.sweep_quad_run(qpb, C.c_int64(A.shape[0]), C.c_int64(A.nnz), p(rp), p(ci), p(va), p(x), p(y), 20,
                                C.c_int64(FLUSH_BYTES), C.byref(cold), C.byref(warm))
        print(json.dumps({"workload": wl, "layout": "quad fp32", "quads_per_batch": qpb, "rc": rc,
                          "cold_us": cold.value * 1e3, "warm_us": warm.value * 1e3,
                          "frac_alg_cold": alg / (cold.value * 1e-3) / 8e12, "bitexact": bool(torch.equal(y, ref))}),
              flush=True)


def main(wl):
    sys.path.insert(0, ROOT)
    import numpy as np
    import scipy.sparse as sp
    import torch

    from bench import FLUSH_BYTES, spmv_bytes
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A_raw, mask, _, _, _ = P.workload(wl)
    A = sp.csr_matrix(A_raw)
    A.sort_indices()
    A.data = A.data.astype(np.float32).astype(np.float64)  # fp32-exact, like the reference's matrices
    Ad = DeviceMatrix.from_scipy(A)
    lib = C.CDLL(LIB)
    rp = torch.from_numpy(A.indptr.astype(np.int32)).cuda()
    ci = torch.from_numpy(A.indices.astype(np.int32)).cuda()
    va = torch.from_numpy(A.data).cuda()
    x = torch.randn(2 * A.shape[0], dtype=torch.float64, device="cuda")  # [z | p] for the fused configs
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    ref = Ad.matvec(x[: A.shape[0]].contiguous())
    reff = Ad.matvec((x[A.shape[0]:] * 0.5 + x[: A.shape[0]]).contiguous())
    alg = spmv_bytes(A.shape[0], A.nnz)
    p = lambda t: C.c_void_p(t.data_ptr())
    for cid in range(lib.sweep_count()):
        vb, qb, mw, tr = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        lib.sweep_cfg(cid, C.byref(vb), C.byref(qb), C.byref(mw), C.byref(tr))
        cold, warm = C.c_double(), C.c_double()
        y.fill_(float("nan"))
        rc = lib.sweep_run(cid, C.c_int64(A.shape[0]), C.c_int64(A.nnz), p(rp), p(ci), p(va), p(x), p(y), 20,
                           C.c_int64(FLUSH_BYTES), C.byref(cold), C.byref(warm))
        print(json.dumps({"workload": wl, "values": "fp64" if vb.value == 8 else "fp32", "SB": qb.value,
                          "MINW": mw.value, "fused_gather": tr.value == 1, "x_const": tr.value == 3,
                          "cluster": {4: "all loads", 5: "reuse (bound)", 6: "dpp shift"}.get(tr.value), "rc": rc,
                          "cold_us": cold.value * 1e3, "warm_us": warm.value * 1e3,
                          "frac_alg_cold": alg / (cold.value * 1e-3) / 8e12,
                          "bitexact": bool(torch.equal(y, reff if tr.value == 1 else ref))}),
              flush=True)


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    elif "--bsr" in sys.argv:
        main_bsr()
    elif "--quad" in sys.argv:
        main_quad("kuhn101")
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else "kuhn101")
