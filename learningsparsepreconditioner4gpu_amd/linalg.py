"""``pymathprim.linalg.PreconditionedConjugateGradient`` on MI355X.

Drop-in for the native solver the reference calls at
``neural_cg/utils/validate.py:79-80, 116-117, 151-156``::

    solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
    iters, prec_time_s, solve_time_s = solver(b, x, rtol, max_iter, ext_spai=(L, eps))

Arithmetic follows scipy 1.15 ``cg`` (the reference's own CPU restatement,
validate.py:163-341): see ``include/lspcg.h`` and DESIGN.md.  ``x`` is updated in place
with the solution (numpy arrays or device tensors).  Only the HIP path exists.

Device contract: the reference's own defaults are ``device="cpu"``
(``validate.py:61,98``: pymathprim's CPU backend), and ``infer.py:316-325`` calls both
devices from one loop.  This class replaces the ``device="cuda"`` backend only:
``PreconditionedConjugateGradient(A, device="cpu", ...)`` constructs pymathprim's own solver
(the reference's CPU row, unchanged) when pymathprim is importable, and otherwise raises
:class:`CpuBackendUnavailable` -- a ``RuntimeError``, the exception the reference's infer loop
already catches per sample (``infer.py:363``).  Nothing here runs a CPU solve of its own: there
is no CPU solver in the product.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple, Union

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from .sparse import Context, DeviceMatrix, _ptr, lspcg_dtype

GPU_DEVICES = ("cuda", "hip", "gpu", "rocm")
CPU_DEVICES = ("cpu",)
SUPPORTED = tuple(_lib.PRECOND) + ("ainv",)
NOT_BUILT = ("fsai",)  # commented out of the reference's baseline rows (infer.py:315)


class CpuBackendUnavailable(RuntimeError):
    """``device="cpu"`` without pymathprim: the reference's CPU backend is not installed.  A
    ``RuntimeError``, so the reference's infer loop (``except RuntimeError``, infer.py:363) logs it
    and moves on exactly as it does for a solver failure."""


def is_cpu_device(device) -> bool:
    return str(device).split(":")[0] in CPU_DEVICES


def cpu_backend():
    """pymathprim's ``PreconditionedConjugateGradient`` -- the class the reference's CPU rows
    construct (validate.py:73, 110, 145) -- or :class:`CpuBackendUnavailable`."""
    try:
        from pymathprim.linalg import PreconditionedConjugateGradient as host_pcg
    except ImportError as e:
        raise CpuBackendUnavailable(
            "device='cpu' is pymathprim's CPU backend (the reference's CPU rows), which is not installed; "
            "this framework replaces the device='cuda' backend only") from e
    return host_pcg


def _as_device_matrix(M, dtype, block_size: int, ctx: Context) -> DeviceMatrix:
    if isinstance(M, DeviceMatrix):
        if M.dtype_code != lspcg_dtype(dtype):
            raise TypeError(f"matrix dtype {M.dtype} differs from solver dtype {dtype}")
        return M
    return DeviceMatrix.from_scipy(sp.csr_matrix(M), dtype=dtype, block_size=block_size, ctx=ctx)


class PreconditionedConjugateGradient:
    def __new__(cls, matrix=None, device: str = "cuda", preconditioner: str = "none", dtype=np.float64,
                block_size: int = 1, ctx: Optional[Context] = None, dot_order: str = "compensated",
                dot_threads: int = 1):
        if is_cpu_device(device):
            # the reference's CPU row: pymathprim's solver with the reference's own arguments
            # (validate.py:79, 116, 151-156); the MI355X-only keywords have no meaning there
            if block_size != 1 or ctx is not None or dot_order != "compensated":
                raise ValueError("block_size / ctx / dot_order select the MI355X solver; device='cpu' is pymathprim's")
            return cpu_backend()(matrix=matrix, device=device, preconditioner=preconditioner, dtype=dtype)
        return super().__new__(cls)

    def __init__(self, matrix, device: str = "cuda", preconditioner: str = "none", dtype=np.float64,
                 block_size: int = 1, ctx: Optional[Context] = None, dot_order: str = "compensated",
                 dot_threads: int = 1):
        if str(device).split(":")[0] not in GPU_DEVICES:
            raise ValueError(
                f"device={device!r}: expected 'cuda' (this MI355X solver) or 'cpu' (pymathprim's CPU backend)")
        if preconditioner in NOT_BUILT:
            raise NotImplementedError(f"preconditioner {preconditioner!r} is not built (the reference's baseline "
                                      "rows use none / diagonal / ainv / ic, infer.py:310-315)")
        if preconditioner not in SUPPORTED:
            raise ValueError(f"unknown preconditioner {preconditioner!r}; expected one of {SUPPORTED}")
        dev = str(device).split(":")
        self.ctx = ctx or Context.get(int(dev[1]) if len(dev) > 1 else None)
        self.dtype = np.dtype(dtype)
        self.preconditioner = preconditioner
        self.A = _as_device_matrix(matrix, self.dtype, block_size, self.ctx)
        self.n = self.A.n
        # "ainv" runs as the ext_spai operator L Lᵀ + 0·I with L = Z D^{-1/2} (lspcg_ainv0)
        kind = "ext_spai" if preconditioner == "ainv" else preconditioner
        h = C.c_void_p()
        _lib.call("lspcg_solver_create", self.ctx.handle, self.A.handle, _lib.PRECOND[kind], C.byref(h))
        self.handle = h
        self._L = None
        self._spai_key = None
        self.dot_order = ("compensated", 1)
        self.setup_time = 0.0  # device setup of the ic / ainv preconditioner (seconds)
        if preconditioner == "ic":
            ms = C.c_double()
            _lib.call("lspcg_solver_set_ic", self.handle, C.byref(ms))
            self.setup_time = ms.value / 1e3
        elif preconditioner == "ainv":
            L, t = self.A.ainv0()
            self.setup_time = t + self.set_spai(L, 0.0)
            self._spai_key = ("ainv",)
        if dot_order != "compensated":
            self.set_dot_order(dot_order, dot_threads)

    def set_ic_factor(self, L) -> float:
        """``preconditioner="ic"`` with a given lower factor L (M⁻¹ = L⁻ᵀ L⁻¹; the reference's
        ``IncompleteCholeskyPreconditioner(L)``, validate.py:344-419).  Returns the setup time (s)."""
        if self.preconditioner != "ic":
            raise ValueError("set_ic_factor needs preconditioner='ic'")
        Ld = _as_device_matrix(L, self.dtype, 1, self.ctx)
        ms = C.c_double()
        try:
            _lib.call("lspcg_solver_set_ic_factor", self.handle, Ld.handle, C.byref(ms))
        except _lib.LspcgError as e:  # the reference's apply (spsolve_triangular) raises LinAlgError
            if e.code == _lib.ERR_SINGULAR:
                raise np.linalg.LinAlgError("A is singular: zero entry on diagonal.") from e
            raise
        self.setup_time = ms.value / 1e3
        return self.setup_time

    def set_dot_order(self, order: str = "compensated", threads: int = 1):
        """Summation order of the loop's dots and norms (include/lspcg.h lspcg_solver_set_dot_order).
        ``"compensated"`` (default): compensated dots in a fixed tree (~correctly rounded) on the
        fastest schedule.  ``"openblas"``: parity mode (fp64) -- numpy's ddot as in the container
        that recorded the reference's trajectories (OpenBLAS 0.3.29 SkylakeX, ``threads`` OpenBLAS
        threads), reproducing scipy cg's recorded count, history and x bit for bit, at the cost of
        one extra single-workgroup launch per dot."""
        if order not in _lib.DOT_ORDER:
            raise ValueError(f"unknown dot order {order!r}; expected one of {tuple(_lib.DOT_ORDER)}")
        _lib.call("lspcg_solver_set_dot_order", self.handle, _lib.DOT_ORDER[order], int(threads))
        self.dot_order = (order, int(threads) if order == "openblas" else 1)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.lspcg_solver_destroy(h)
            self.handle = None

    @property
    def views(self) -> dict:
        """The iteration views of A, L, Lᵀ (``lspcg_solver_views``): column storage (``"csr"``,
        ``"sdia"``, ``"sellc"`` (one-byte offset codes), ``"sell16"``, ``"sell32"``) and value bytes per
        slot (8, 4, or 1 = dictionary codes)."""
        ck, vb = (C.c_int * 3)(), (C.c_int * 3)()
        _lib.call("lspcg_solver_views", self.handle, ck, vb)
        names = {0: "csr", 1: "sdia", 8: "sellc", 16: "sell16", 17: "sell16j", 18: "sell16x", 32: "sell32"}
        return {m: {"columns": names.get(ck[w], str(ck[w])), "value_bytes": vb[w]}
                for w, m in enumerate(("A", "L", "LT"))}

    @property
    def reorder_info(self) -> dict:
        """The analysis step's verdict (``lspcg_solver_reorder_info``): whether the loop runs on the
        reverse-Cuthill-McKee-permuted system, and mean |col - row| before / after."""
        a, b0, b1 = C.c_int(), C.c_double(), C.c_double()
        _lib.call("lspcg_solver_reorder_info", self.handle, C.byref(a), C.byref(b0), C.byref(b1))
        return {"applied": bool(a.value), "mean_offset_before": b0.value, "mean_offset_after": b1.value}

    def set_spai(self, L, epsilon: float, block_size: int = 1) -> float:
        """Install M⁻¹ = L Lᵀ + εI (ext_spai); returns the device setup time in seconds."""
        Ld = _as_device_matrix(L, self.dtype, block_size, self.ctx)
        ms = C.c_double()
        _lib.call("lspcg_solver_set_spai", self.handle, Ld.handle, float(epsilon), C.byref(ms))
        self._L = Ld  # keep alive: the solver reads it
        self._spai_key = self._key(L, epsilon)
        return ms.value / 1e3

    @staticmethod
    def _key(L, epsilon):
        """Identity of an installed ext_spai factor: the object itself (held, so its id cannot be
        reused by another object), its in-place version (DeviceMatrix) and ε."""
        return (L, getattr(L, "version", None), float(epsilon))

    def _is_installed(self, L, epsilon) -> bool:
        k = self._spai_key
        return (k is not None and len(k) == 3 and k[0] is L and k[1] == getattr(L, "version", None)
                and k[2] == float(epsilon))

    def solve(self, b: torch.Tensor, x: torch.Tensor, rtol: float = 1e-6, max_iter: int = 0,
              return_history: bool = False):
        """Device-tensor form: returns ``(iters, converged, solve_time_s[, res_hist])``."""
        self._check_vector("b", b)
        self._check_vector("x", x)
        mi = int(max_iter) if max_iter and max_iter > 0 else self.n
        it = C.c_int64()
        ms = C.c_double()
        hist = np.empty(mi + 2, dtype=np.float64) if return_history else None
        rc = _lib.call("lspcg_solver_solve", self.handle, _ptr(b), _ptr(x), float(rtol), mi, C.byref(it),
                       hist.ctypes.data_as(_lib.p_f64) if hist is not None else None, C.byref(ms),
                       allow_not_converged=True)
        self.last_converged = rc == _lib.OK
        out = (it.value, rc == _lib.OK, ms.value / 1e3)
        if return_history:
            out = out + (hist[: min(it.value, mi) + 1].copy(),)  # NaN after a non-finite stop (lspcg.h)
        return out

    @property
    def torch_dtype(self) -> torch.dtype:
        return torch.float32 if self.dtype == np.float32 else torch.float64

    def _check_vector(self, name: str, v: torch.Tensor):
        """The C ABI copies n * sizeof(dtype) bytes from / to these pointers: reject anything
        that is not a contiguous length-n vector of the solver's dtype on the solver's device."""
        if not isinstance(v, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor on {self.ctx.torch_device}")
        if v.numel() != self.n:
            raise ValueError(f"{name} has {v.numel()} entries, the system has {self.n}")
        if v.dtype != self.torch_dtype:
            raise TypeError(f"{name} is {v.dtype}, the solver computes in {self.torch_dtype}")
        if v.device != self.ctx.torch_device:
            raise ValueError(f"{name} is on {v.device}, the solver runs on {self.ctx.torch_device}")
        if not v.is_contiguous():
            raise ValueError(f"{name} must be contiguous")

    KERNELS = ("KA t=L^T r", "KB z=L t+eps r, rho", "UP p, x", "KC q=A p, pi", "UR r")

    def time_kernels(self, b: torch.Tensor, iters: int = 40) -> dict:
        """Measurement only: mean device time (s) of each launch of the ext_spai iteration
        (HIP events around every launch, ``iters`` iterations from x0 = 0, no graphs)."""
        self._check_vector("b", b)
        out = (C.c_double * 8)()
        nk = C.c_int()
        _lib.call("lspcg_solver_time_kernels", self.handle, C.c_void_p(b.data_ptr()), int(iters), out, C.byref(nk))
        return {self.KERNELS[k]: out[k] / 1e3 for k in range(nk.value)}

    def __call__(self, b, x, rtol: float = 1e-6, max_iter: int = 0, ext_spai=None,
                 return_history: bool = False) -> Tuple:
        prec = self.setup_time
        if self.preconditioner in ("ext_spai", "ext_spai_scaled"):
            if ext_spai is None and self._L is None:
                raise ValueError("ext_spai=(L, epsilon) is required for this preconditioner")
            if ext_spai is not None:
                L, eps = ext_spai
                if not self._is_installed(L, eps):
                    prec = self.set_spai(L, eps, block_size=getattr(L, "block_size", 1)
                                         if isinstance(L, DeviceMatrix) else 1)
        tdt = self.torch_dtype
        dev = self.ctx.torch_device
        bt = torch.as_tensor(b).to(device=dev, dtype=tdt).contiguous().reshape(-1)
        xt = torch.as_tensor(x).to(device=dev, dtype=tdt).contiguous().reshape(-1)
        res = self.solve(bt, xt, rtol, max_iter, return_history)
        if not (isinstance(x, torch.Tensor) and x.is_cuda and x.data_ptr() == xt.data_ptr()):
            if isinstance(x, np.ndarray):
                x[...] = xt.cpu().numpy().reshape(x.shape)
            elif isinstance(x, torch.Tensor):
                x.copy_(xt.reshape(x.shape))
        iters, _conv, solve = res[:3]
        return (iters, prec, solve) + (tuple(res[3:]) if return_history else ())


def solve_many(jobs, rtol: float = 1e-6, max_iter: int = 0, concurrency: int = 4):
    """Independent solves ``[(solver, b, x), ...]`` with up to ``concurrency`` of them in flight on
    the device: every solver owns a non-blocking stream and ``lspcg_solver_solve`` releases the GIL
    (ctypes), so host threads overlap the solves' dependent launch chains.  Each solve returns what
    it returns alone (same iterate, count and history); ``[(iters, converged, solve_time_s), ...]``
    in job order, the times including the overlap."""
    jobs = list(jobs)
    if concurrency <= 1 or len(jobs) <= 1:
        return [s.solve(b, x, rtol, max_iter) for s, b, x in jobs]
    from concurrent.futures import ThreadPoolExecutor

    dev = jobs[0][0].ctx.device  # the pool's threads select the solvers' device (per-thread state)
    with ThreadPoolExecutor(min(int(concurrency), len(jobs)), initializer=torch.cuda.set_device, initargs=(dev,)) as ex:
        return list(ex.map(lambda j: j[0].solve(j[1], j[2], rtol, max_iter), jobs))


class BatchedConjugateGradient:
    """ext_spai PCG of several independent systems in lockstep (``lspcg_batch_*``).

    The reference solves its samples one at a time (``infer.py:278-331``: one
    ``get_pcg_iter_time`` per sample, ``validate.py:89-121``).  Mid-size systems are
    latency-bound on MI355X (a few hundred workgroups per launch, five dependent launches per
    iteration), so here a window of them shares every launch: the systems are laid out
    block-diagonally and each phase of the split schedule runs once for all of them, each system
    with its own scalars, convergence test and iteration count.  Per system the
    result is what ``PreconditionedConjugateGradient`` returns for it alone.

    ``As[k]``, ``Ls[k]``: matrix and ext_spai factor of system k (DeviceMatrix or scipy), one
    dtype and block size; ``epsilon``: the common ε of M⁻¹ = L Lᵀ + εI.  Raises ``LspcgError``
    with code ``ERR_UNSUPPORTED`` when no SELL view of the batch can be built (irregular rows).
    """

    def __init__(self, As, Ls, epsilon: float, dtype=np.float64, block_size: int = 1,
                 ctx: Optional[Context] = None):
        As, Ls = list(As), list(Ls)
        if not As or len(As) != len(Ls):
            raise ValueError("need one L per A and at least one system")
        self.ctx = ctx or (As[0].ctx if isinstance(As[0], DeviceMatrix) else Context.get())
        self.dtype = np.dtype(dtype)
        self.A = [_as_device_matrix(M, self.dtype, block_size, self.ctx) for M in As]
        self.L = [_as_device_matrix(M, self.dtype, block_size, self.ctx) for M in Ls]
        self.n = [M.n for M in self.A]
        self.epsilon = float(epsilon)
        k = len(self.A)
        ha = (C.c_void_p * k)(*[M.handle.value for M in self.A])
        hl = (C.c_void_p * k)(*[M.handle.value for M in self.L])
        h = C.c_void_p()
        _lib.call("lspcg_batch_create", self.ctx.handle, k, ha, hl, self.epsilon, C.byref(h))
        self.handle = h

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.lspcg_batch_destroy(h)
            self.handle = None

    def __len__(self):
        return len(self.n)

    @property
    def torch_dtype(self) -> torch.dtype:
        return torch.float32 if self.dtype == np.float32 else torch.float64

    def _check(self, name, vs):
        vs = list(vs)
        if len(vs) != len(self.n):
            raise ValueError(f"{name}: {len(vs)} vectors for {len(self.n)} systems")
        for k, v in enumerate(vs):
            if not isinstance(v, torch.Tensor) or v.numel() != self.n[k] or v.dtype != self.torch_dtype \
                    or v.device != self.ctx.torch_device or not v.is_contiguous():
                raise ValueError(f"{name}[{k}] must be a contiguous {self.torch_dtype} tensor of {self.n[k]} entries "
                                 f"on {self.ctx.torch_device}")
        return vs

    def solve(self, bs, xs, rtol: float = 1e-6, max_iter: int = 0, return_history: bool = False):
        """Solve every system from its x (in place).  Returns ``(results, solve_time_s)`` with
        ``results[k] = (iters, converged[, res_hist])``; the time is the whole batch's."""
        bs = self._check("b", bs)
        xs = self._check("x", xs)
        k = len(self.n)
        mi = [int(max_iter) if max_iter and max_iter > 0 else n for n in self.n]
        it = (C.c_int64 * k)()
        stt = (C.c_int32 * k)()
        ms = C.c_double()
        hists = [np.empty(m + 2, dtype=np.float64) for m in mi] if return_history else None
        hp = (_lib.p_f64 * k)(*[h.ctypes.data_as(_lib.p_f64) for h in hists]) if hists else None
        _lib.call("lspcg_batch_solve", self.handle, (C.c_void_p * k)(*[b.data_ptr() for b in bs]),
                  (C.c_void_p * k)(*[x.data_ptr() for x in xs]), float(rtol), int(max_iter) if max_iter else 0,
                  it, stt, hp, C.byref(ms), allow_not_converged=True)
        res = []
        for j in range(k):
            r = (int(it[j]), stt[j] == _lib.OK)
            if hists:
                r = r + (hists[j][: min(int(it[j]), mi[j]) + 1].copy(),)
            res.append(r)
        return res, ms.value / 1e3
