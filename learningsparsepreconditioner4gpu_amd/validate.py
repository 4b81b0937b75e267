"""Drop-in mirror of ``neural_cg/utils/validate.py``'s hot-path API, backed by HIP.

Same names, arguments, return values and error behaviour as the reference:

* ``to_csr_cpu``                 -- validate.py:22-51 (assembly runs on the GPU, result
  returned as a sorted scipy CSR like the reference)
* ``get_cg_iter_time``           -- validate.py:54-86 (raises ``RuntimeError("CG did not
  converge")`` when ``iter >= max_iter``, as :84-85)
* ``get_pcg_iter_time``          -- validate.py:89-121 (ext_spai, never raises)
* ``get_pcg_scaled_iter_time``   -- validate.py:124-160 (ext_spai_scaled)
* ``get_pcg_iter_time_batch``    -- not in the reference: ``get_pcg_iter_time`` over a window
  of independent systems solved as one lockstep batch
* ``get_pcg_iter_time_scipy`` / ``get_pcg_diagonal_iter_time_scipy`` /
  ``get_pcg_scaled_iter_time_scipy`` / ``get_cg_iter_time_scipy`` -- validate.py:163-341, the
  reference's host (scipy) restatements, re-exported from ``cpu_rows`` (host comparison rows
  only; never called by the functions above)

Matrices may be scipy CSR (uploaded) or :class:`DeviceMatrix` (already in HBM).

Device contract: the reference's default, ``device="cpu"`` (validate.py:61,98,133), is kept
and means what it means there: pymathprim's CPU backend.  ``device="cpu"`` runs the reference's
own host sequence (validate.py:64-86, 99-121, 134-160: ``b = A @ gt`` on the host, one
pymathprim solver per repeat) through ``linalg.PreconditionedConjugateGradient``, which hands
the CPU device to pymathprim or raises ``linalg.CpuBackendUnavailable`` (a ``RuntimeError``,
what the reference's infer loop catches) when pymathprim is absent.  ``device="cuda"`` is the
MI355X path, where right-hand sides are formed on the device exactly as ``b = A @ gt``
(bit-identical to scipy's csr_matvec).  No function here computes a solve on the host.
"""
from __future__ import annotations

import math
import time
from typing import List, Optional, Tuple, Union

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from .cpu_rows import (get_cg_iter_time_scipy, get_pcg_diagonal_iter_time_scipy,  # noqa: F401
                       get_pcg_iter_time_scipy, get_pcg_scaled_iter_time_scipy)
from .linalg import BatchedConjugateGradient, PreconditionedConjugateGradient, is_cpu_device
from .sparse import Context, DeviceMatrix, assemble, dot, lspcg_dtype


def to_numpy(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    if isinstance(x, np.ndarray):
        return x
    raise ValueError(f"Unknown type {type(x)}")


def to_csr_device(edge_index, edge_attr, n: int, mask, dtype=np.float64, block_output: bool = False) -> DeviceMatrix:
    """GPU assembly with to_csr_cpu semantics; the result stays in HBM."""
    ei = torch.as_tensor(edge_index)
    ea = torch.as_tensor(edge_attr)
    assert ei.ndim == 2 and ei.shape[0] == 2
    assert ea.ndim in [1, 3]
    m = None if mask is None else torch.as_tensor(mask)
    tdt = torch.float32 if np.dtype(dtype) == np.float32 else torch.float64
    return assemble(ei, ea, n, m, dtype=tdt, block_output=block_output)


def to_csr_cpu(edge_index, edge_attr, n: int, mask, dtype=np.float64) -> sp.csr_matrix:
    """validate.py:22-51.  Assembled on the GPU, returned as a sorted scipy CSR."""
    return to_csr_device(edge_index, edge_attr, n, mask, dtype).to_scipy()


def _device_rhs(A: DeviceMatrix, gt) -> torch.Tensor:
    g = torch.as_tensor(np.asarray(to_numpy(gt) if isinstance(gt, torch.Tensor) else gt)).reshape(-1)
    return A.matvec(g.to(device=A.ctx.torch_device, dtype=A.dtype))


def _prepare(A, dtype, block_size=1) -> DeviceMatrix:
    if isinstance(A, DeviceMatrix):
        return A
    return DeviceMatrix.from_scipy(sp.csr_matrix(A), dtype=dtype, block_size=block_size, ctx=Context.get())


def _no_device_options(info, dot_order, dot_threads):
    """``info`` / ``dot_order`` / ``dot_threads`` are options of the HIP path (not in the reference's
    signatures): the cpu row is pymathprim's own solver, which has neither, so asking for them with
    device="cpu" (the reference's default) is an error, not a silently empty ``info``."""
    if info is not None or dot_order != "compensated" or dot_threads != 1:
        raise ValueError("info / dot_order / dot_threads apply to device='cuda' only: device='cpu' is the "
                         "reference's pymathprim row (pass device='cuda' for the HIP solver)")


def _host_pcg_sequence(A, gt, spai, epsilon, rtol, max_iter, repeat, dtype, device, method, raise_on_max):
    """The reference's CPU rows as it runs them (validate.py:64-86 / 99-121 / 134-160): host
    ``b = A @ gt``, then per repeat one solver from ``PreconditionedConjugateGradient(device="cpu")``
    -- pymathprim's own class, or ``CpuBackendUnavailable`` -- called on host copies.  Host logic
    only: the solve is pymathprim's."""
    A = A.to_scipy() if isinstance(A, DeviceMatrix) else sp.csr_matrix(A)
    if isinstance(spai, DeviceMatrix):
        spai = spai.to_scipy()
    rows = A.shape[0]
    max_iter = max_iter if max_iter > 0 else rows
    b = np.asarray(A @ to_numpy(gt) if isinstance(gt, torch.Tensor) else A @ gt).astype(dtype).copy()
    A = A.astype(dtype)
    spai = None if spai is None else sp.csr_matrix(spai).astype(dtype)
    assert repeat > 0
    iter_cnt, time_prec, time_elp = 0, 0.0, 0.0
    x = np.zeros_like(b, dtype=dtype)
    for _ in range(repeat):
        x_copy, b_copy = x.copy(), b.copy()
        kw = {} if method == "ext_spai_scaled" else {"dtype": np.float64}  # validate.py:151-156 passes no dtype
        solver = PreconditionedConjugateGradient(matrix=A, device=device, preconditioner=method, **kw)
        if spai is None:
            this_iter, this_prec, this_solve = solver(b_copy, x_copy, rtol, max_iter)
        else:
            this_iter, this_prec, this_solve = solver(b_copy, x_copy, rtol, max_iter, ext_spai=(spai, epsilon))
        iter_cnt += this_iter
        time_prec += this_prec
        time_elp += this_solve
        if raise_on_max and this_iter >= max_iter:
            raise RuntimeError("CG did not converge")
    return iter_cnt / repeat, time_prec / repeat, time_elp / repeat


def get_cg_iter_time(A, gt, rtol=1e-6, max_iter=0, dtype=np.float64, repeat=1, device="cpu",
                     method="ainv", info: Optional[dict] = None, dot_order: str = "compensated",
                     dot_threads: int = 1) -> Tuple[float, float, float]:
    """validate.py:54-86: method none / diagonal / ic (IC(0), level-scheduled triangular solves) /
    ainv (AINV(0) as L Lᵀ); the prec time is the device setup of the preconditioner.
    ``dot_order`` / ``dot_threads`` (not in the reference's signature): the loop's dot order,
    ``"openblas"`` = parity mode (linalg.PreconditionedConjugateGradient.set_dot_order).
    ``device="cpu"`` (the reference's default) is the reference's pymathprim row (module doc)."""
    if is_cpu_device(device):
        _no_device_options(info, dot_order, dot_threads)
        return _host_pcg_sequence(A, gt, None, 0.0, rtol, max_iter, repeat, dtype, device, method, True)
    Ad = _prepare(A, dtype)
    rows = Ad.n
    max_iter = max_iter if max_iter > 0 else rows
    b = _device_rhs(Ad, gt)
    iter_cnt, time_prec, time_elp = 0, 0.0, 0.0
    x = torch.zeros_like(b)
    for _ in range(repeat):
        solver = PreconditionedConjugateGradient(Ad, device=device, preconditioner=method, dtype=dtype,
                                                 dot_order=dot_order, dot_threads=dot_threads)
        xs = x.clone()
        this_iter, this_prec, this_solve = solver(b.clone(), xs, rtol, max_iter)
        iter_cnt += this_iter
        time_prec += this_prec
        time_elp += this_solve
        if this_iter >= max_iter:
            raise RuntimeError("CG did not converge")
    if info is not None:
        info.update(x=xs, rel_res=relative_residual(Ad, xs, b), converged=bool(solver.last_converged),
                    iters=int(this_iter))
    return iter_cnt / repeat, time_prec / repeat, time_elp / repeat


def relative_residual(A: DeviceMatrix, x: torch.Tensor, b: torch.Tensor) -> float:
    """True relative residual ‖b − A x‖ / ‖b‖ on the device (one SpMV, compensated dots)."""
    r = b - A.matvec(x)
    bb = dot(b, b)
    return math.sqrt(dot(r, r) / bb) if bb > 0 else math.sqrt(dot(r, r))


def _pcg_generic(method, A, gt, spai, epsilon, rtol, max_iter, repeat, dtype, device, info=None,
                 dot_order="compensated", dot_threads=1):
    if is_cpu_device(device):
        _no_device_options(info, dot_order, dot_threads)
        return _host_pcg_sequence(A, gt, spai, epsilon, rtol, max_iter, repeat, dtype, device, method, False)
    Ad = _prepare(A, dtype)
    Ld = spai if isinstance(spai, DeviceMatrix) else _prepare(spai, dtype)
    rows = Ad.n
    max_iter = max_iter if max_iter > 0 else rows
    b = _device_rhs(Ad, gt)
    assert repeat > 0
    iter_cnt, time_elp, time_prec = 0, 0.0, 0.0
    x = torch.zeros_like(b)
    for _ in range(repeat):
        solver = PreconditionedConjugateGradient(Ad, device=device, preconditioner=method, dtype=dtype,
                                                 dot_order=dot_order, dot_threads=dot_threads)
        xs = x.clone()
        this_iter, this_prec, this_solve = solver(b.clone(), xs, rtol, max_iter, ext_spai=(Ld, epsilon))
        iter_cnt += this_iter
        time_prec += this_prec
        time_elp += this_solve
    if info is not None:  # the last solve's iterate, its true residual and the solver's verdict
        info.update(x=xs, rel_res=relative_residual(Ad, xs, b), converged=bool(solver.last_converged),
                    iters=int(this_iter))
    return iter_cnt / repeat, time_prec / repeat, time_elp / repeat


def get_pcg_iter_time(A, gt, spai, epsilon: float, rtol=1e-6, max_iter=0, repeat=1, dtype=np.float64,
                      device="cpu", info: Optional[dict] = None, dot_order: str = "compensated",
                      dot_threads: int = 1) -> Tuple[float, float, float]:
    """validate.py:89-121: ext_spai PCG, M⁻¹ = L Lᵀ + εI.  ``info`` (optional dict, not in the
    reference's signature) receives the last solve's x, true relative residual and convergence;
    ``dot_order`` / ``dot_threads`` (not in the reference's signature) select the loop's dot order
    (``"openblas"`` = parity mode: the reference's recorded scipy trajectories bit for bit)."""
    return _pcg_generic("ext_spai", A, gt, spai, epsilon, rtol, max_iter, repeat, dtype, device, info,
                        dot_order, dot_threads)


def get_pcg_iter_time_batch(As, gts, spais, epsilon: float, rtol=1e-6, max_iter=0, dtype=np.float64,
                            infos: Optional[list] = None, repeat: int = 1) -> List[Tuple[float, float, float]]:
    """get_pcg_iter_time over a window of independent systems solved as ONE lockstep batch
    (linalg.BatchedConjugateGradient; the reference calls get_pcg_iter_time once per sample,
    infer.py:322).  Per system ``(iters, prec_s, solve_s)``: the batch's setup (block-diagonal
    copy, Lᵀ and views: host wall) and device solve time split evenly over its systems, the solve
    averaged over ``repeat`` solves from x0 = 0 like get_pcg_iter_time (validate.py:111-121).  A
    window without a SELL view (irregular rows) is solved one system at a time instead, on the GPU."""
    Ads = [_prepare(A, dtype) for A in As]
    Lds = [L if isinstance(L, DeviceMatrix) else _prepare(L, dtype) for L in spais]
    bs = [_device_rhs(A, gt) for A, gt in zip(Ads, gts)]
    k = len(Ads)
    try:
        t0 = time.perf_counter()
        B = BatchedConjugateGradient(Ads, Lds, epsilon, dtype=dtype)
        prec = time.perf_counter() - t0
    except _lib.LspcgError as e:
        if e.code != _lib.ERR_UNSUPPORTED:
            raise
        out = []
        for j in range(k):
            info = {} if infos is not None else None
            out.append(get_pcg_iter_time(Ads[j], gts[j], Lds[j], epsilon, rtol, max_iter, repeat, dtype,
                                         device="cuda", info=info))
            if infos is not None:
                infos[j].update(info)
        return out
    t = 0.0
    for _ in range(max(1, int(repeat))):
        xs = [torch.zeros_like(b) for b in bs]
        res, dt = B.solve(bs, xs, rtol, max_iter)
        t += dt
    t /= max(1, int(repeat))
    out = []
    for j, (it, conv) in enumerate(res):
        if infos is not None:
            infos[j].update(x=xs[j], rel_res=relative_residual(Ads[j], xs[j], bs[j]), converged=bool(conv), iters=it)
        out.append((float(it), prec / k, t / k))
    return out


def get_pcg_scaled_iter_time(A, gt, spai, epsilon: float, rtol=1e-6, max_iter=0, repeat=1, dtype=np.float64,
                             device="cpu", info: Optional[dict] = None, dot_order: str = "compensated",
                             dot_threads: int = 1) -> Tuple[float, float, float]:
    """validate.py:124-160: ext_spai_scaled PCG, M⁻¹ r = L((Lᵀr)/d) + εr/d, d = diag(A)."""
    return _pcg_generic("ext_spai_scaled", A, gt, spai, epsilon, rtol, max_iter, repeat, dtype, device, info,
                        dot_order, dot_threads)
