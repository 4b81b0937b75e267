"""ctypes binding of liblspcg_hip.so (the C ABI declared in include/lspcg.h).

The HIP library is the only compute path of this package: if it is missing or
fails to load, every compute entry point raises ``LspcgUnavailable`` -- there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("LSPCG_LIB", PKG / "liblspcg_hip.so"))

OK, NOT_CONVERGED = 0, 1
ERR_ARG, ERR_HIP, ERR_UNSUPPORTED, ERR_FORMAT, ERR_BREAKDOWN, ERR_SINGULAR = -1, -2, -3, -4, -5, -6
F32, F64 = 0, 1
PRECOND = {"none": 0, "diagonal": 1, "ext_spai": 2, "ext_spai_scaled": 3, "ic": 4}
DOT_ORDER = {"compensated": 0, "openblas": 1}

p_i32 = C.POINTER(C.c_int32)
p_i64 = C.POINTER(C.c_int64)
p_f64 = C.POINTER(C.c_double)
vp = C.c_void_p
pp = C.POINTER(C.c_void_p)


class lspcg_gnn_desc(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("node_in", "edge_in", "hidden", "mlp_layers", "num_mp_layers",
                                      "edge_out", "node_residual", "edge_residual")]


# name -> (restype, argtypes); the list IS the exported ABI (tests check it against include/lspcg.h)
SIGNATURES = {
    "lspcg_last_error": (C.c_char_p, []),
    "lspcg_version": (C.c_int, []),
    "lspcg_build_id": (C.c_char_p, []),
    "lspcg_ctx_create": (C.c_int, [C.c_int, vp, pp]),
    "lspcg_ctx_destroy": (C.c_int, [vp]),
    "lspcg_ctx_synchronize": (C.c_int, [vp]),
    "lspcg_mat_create_csr": (C.c_int, [vp, C.c_int64, C.c_int64, vp, vp, vp, C.c_int, pp]),
    "lspcg_mat_create_bsr": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int, vp, vp, vp, C.c_int, pp]),
    "lspcg_mat_destroy": (C.c_int, [vp]),
    "lspcg_mat_info": (C.c_int, [vp, p_i64, p_i64, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "lspcg_mat_copy_out": (C.c_int, [vp, vp, vp, vp]),
    "lspcg_mat_transpose": (C.c_int, [vp, pp]),
    "lspcg_mat_diagonal": (C.c_int, [vp, vp]),
    "lspcg_mat_rcm": (C.c_int, [vp, vp, C.POINTER(C.c_int), p_f64, p_f64]),
    "lspcg_mat_scale_columns": (C.c_int, [vp, vp]),
    "lspcg_spmv": (C.c_int, [vp, vp, vp, vp]),
    "lspcg_spmv_timed": (C.c_int, [vp, vp, vp, vp, C.c_int, C.c_int64, p_f64]),
    "lspcg_spmv_variant_timed": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int64, p_f64]),
    "lspcg_spmv_sell_timed": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int64, p_f64]),
    "lspcg_mat_prepare_spmv": (C.c_int, [vp, C.POINTER(C.c_int)]),
    "lspcg_mat_spmv_reorder_info": (C.c_int, [vp, C.POINTER(C.c_int), p_f64, p_f64]),
    "lspcg_read_timed": (C.c_int, [vp, C.c_int64, C.c_int, C.c_int64, p_f64]),
    "lspcg_ic0": (C.c_int, [vp, pp, p_f64]),
    "lspcg_ainv0": (C.c_int, [vp, pp, p_f64]),
    "lspcg_trsv": (C.c_int, [vp, C.c_int, vp, vp]),
    "lspcg_dot": (C.c_int, [vp, C.c_int64, C.c_int, vp, vp, p_f64]),
    "lspcg_solver_create": (C.c_int, [vp, vp, C.c_int, pp]),
    "lspcg_solver_set_spai": (C.c_int, [vp, vp, C.c_double, p_f64]),
    "lspcg_solver_set_ic": (C.c_int, [vp, p_f64]),
    "lspcg_solver_set_ic_factor": (C.c_int, [vp, vp, p_f64]),
    "lspcg_solver_solve": (C.c_int, [vp, vp, vp, C.c_double, C.c_int64, p_i64, p_f64, p_f64]),
    "lspcg_solver_time_kernels": (C.c_int, [vp, vp, C.c_int64, p_f64, C.POINTER(C.c_int)]),
    "lspcg_solver_views": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "lspcg_solver_reorder_info": (C.c_int, [vp, C.POINTER(C.c_int), p_f64, p_f64]),
    "lspcg_solver_set_dot_order": (C.c_int, [vp, C.c_int, C.c_int]),
    "lspcg_solver_destroy": (C.c_int, [vp]),
    "lspcg_batch_create": (C.c_int, [vp, C.c_int, pp, pp, C.c_double, pp]),
    "lspcg_batch_solve": (C.c_int, [vp, pp, pp, C.c_double, C.c_int64, p_i64, p_i32, C.POINTER(p_f64), p_f64]),
    "lspcg_batch_destroy": (C.c_int, [vp]),
    "lspcg_assemble": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int, vp, vp, C.c_int, vp, C.c_int, C.c_int,
                                 C.c_int, pp]),
    "lspcg_gnn_create": (C.c_int, [vp, C.POINTER(lspcg_gnn_desc), vp, C.c_int64, pp]),
    "lspcg_gnn_set_graph": (C.c_int, [vp, C.c_int64, C.c_int64, vp]),
    "lspcg_gnn_forward": (C.c_int, [vp, C.c_int64, C.c_int64, vp, vp, vp, vp]),
    "lspcg_gnn_precision": (C.c_int, [vp, C.POINTER(C.c_int), p_f64]),
    "lspcg_gnn_destroy": (C.c_int, [vp]),
    "lspcg_graph_create": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int, vp, pp]),
    "lspcg_graph_destroy": (C.c_int, [vp]),
    "lspcg_graph_spmv": (C.c_int, [vp, vp, C.c_int, C.c_int, vp, vp, vp]),
    "lspcg_graph_aatpe": (C.c_int, [vp, vp, C.c_int, C.c_double, vp, vp, vp, vp, vp]),
    "lspcg_part_create": (C.c_int, [vp, vp, vp, vp, C.c_int64, vp, C.c_int64, pp]),
    "lspcg_part_destroy": (C.c_int, [vp]),
    "lspcg_part_pack": (C.c_int, [vp, vp, vp]),
    "lspcg_part_norms": (C.c_int, [vp, vp, vp, vp]),
    "lspcg_part_lt": (C.c_int, [vp, vp, vp]),
    "lspcg_part_l": (C.c_int, [vp, vp, vp, C.c_double, vp, vp]),
    "lspcg_part_a": (C.c_int, [vp, vp, vp, vp]),
    "lspcg_part_update_p": (C.c_int, [vp, vp, vp, C.c_double, C.c_int]),
    "lspcg_part_update_xr": (C.c_int, [vp, C.c_double, vp, vp, vp, vp]),
    "lspcg_part_state_init": (C.c_int, [vp, C.c_double, C.c_int64, vp]),
    "lspcg_part_scalars": (C.c_int, [vp, vp, C.c_int, C.c_int]),
    "lspcg_part_update_p_dev": (C.c_int, [vp, vp, vp]),
    "lspcg_part_update_xr_dev": (C.c_int, [vp, vp, vp, vp, vp]),
    "lspcg_part_progress": (C.c_int, [vp, p_i64, C.POINTER(C.c_int), p_f64, p_f64]),
    "lspcg_part_set_rows": (C.c_int, [vp, C.c_int64]),
    "lspcg_part_status": (C.c_int, [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int)]),
}


class LspcgUnavailable(RuntimeError):
    """liblspcg_hip.so could not be loaded (not built, or no ROCm runtime)."""


class LspcgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"lspcg error {code}: {msg}")
        self.code = code


_lib = None


def load() -> C.CDLL:
    """Load the library (cached).  Raises LspcgUnavailable loudly on failure."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise LspcgUnavailable(
            f"{LIB_PATH} is missing: build it with `python -m learningsparsepreconditioner4gpu_amd._build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        lib = C.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime
        raise LspcgUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def build_id() -> str:
    """Hash of the sources, headers, flags and arch the loaded library was built from
    (``_build.tree_hash()`` at build time)."""
    return load().lspcg_build_id().decode()


def last_error() -> str:
    m = load().lspcg_last_error()
    return m.decode() if m else ""


def check(rc: int, allow_not_converged: bool = False) -> int:
    if rc == OK or (allow_not_converged and rc == NOT_CONVERGED):
        return rc
    raise LspcgError(rc, last_error())


def call(name: str, *args, allow_not_converged: bool = False) -> int:
    return check(getattr(load(), name)(*args), allow_not_converged)
