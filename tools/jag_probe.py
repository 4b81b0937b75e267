"""Standalone SpMV timing on one workload (measurement only, GPU box): the fp64 analysis-step SpMV
and the loop's fp32-value form (lspcg_spmv_sell_timed), cold / warm.  Run against variant
libraries with LSPCG_LIB=<path> (tools/build_variant.py) to A/B kernel experiments.

    python tools/jag_probe.py [delaunay1m] [label]
"""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import bench
from learningsparsepreconditioner4gpu_amd import _lib
from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "delaunay1m"
    label = sys.argv[2] if len(sys.argv) > 2 else "base"
    A = P.workload(wl)[0]
    A.data = A.data.astype(np.float32).astype(np.float64)
    D = DeviceMatrix.from_scipy(A)
    x = torch.randn(A.shape[0], dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    kind = D.prepare_spmv()
    ok = bool(np.array_equal(D.matvec(x).cpu().numpy(), A @ x.cpu().numpy()))
    out = {"workload": wl, "label": label, "kind": kind, "bitexact": ok}
    for rnd in range(3):
        out.setdefault("f64_cold_us", []).append(D.spmv_timed(x, y, 20, flush_bytes=bench.FLUSH_BYTES) * 1e3)
        out.setdefault("f64_warm_us", []).append(D.spmv_timed(x, y, 60) * 1e3)
        for lab, fl in (("f32v_cold_us", bench.FLUSH_BYTES), ("f32v_warm_us", 0)):
            ms = C.c_double()
            _lib.call("lspcg_spmv_sell_timed", D.ctx.handle, D.handle, 3 | (16 if kind == 17 else 0),
                      C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 20 if fl else 60, fl, C.byref(ms))
            out.setdefault(lab, []).append(ms.value * 1e3)
    for k in [k for k in out if k.endswith("_us")]:
        out[k] = float(np.median(out[k]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
