"""The reference's host-side comparison rows: ``Neural`` and ``PCG-{none,diagonal}-cpu``.

``infer.py:310-331`` writes, beside its GPU rows, the same solves on the CPU
(``device="cpu"``: pymathprim's CPU backend).  pymathprim is not in this container; the
reference's own CPU stand-in is its scipy restatement (``neural_cg/utils/validate.py:163-341``,
used by ``workspace.py:146-147,168-171`` when pymathprim is missing).  This module is that
restatement under the reference's names, for ``infer --cpu-rows`` only:

* ``get_pcg_iter_time_scipy``          -- validate.py:163-201 (ext_spai, explicit-Lᵀ operator)
* ``get_pcg_diagonal_iter_time_scipy`` -- validate.py:235-264
* ``get_pcg_scaled_iter_time_scipy``   -- validate.py:267-302
* ``get_cg_iter_time_scipy``           -- validate.py:316-333

These are comparison rows, like bench.py's ``cpu_baseline``: nothing on the device path calls
them, and ``infer`` reaches them only after the GNN and the assembly have run on the GPU (no
HIP library, no rows).  Each returns the iteration count like the reference
(``with_time=True``: ``(count, seconds of the cg call)``, the reference's own timer placement).
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.linalg import LinearOperator, cg


class _Op(LinearOperator):
    def __init__(self, fn: Callable[[np.ndarray], np.ndarray], shape, dtype):
        self._fn = fn
        super().__init__(np.dtype(dtype), shape)

    def _matvec(self, x):
        return self._fn(x)


def _count(A, b, M, rtol, max_iter, with_time):
    counter = 0

    def cb(_x):
        nonlocal counter
        counter += 1

    t0 = time.time()
    cg(A, b, M=M, callback=cb, rtol=rtol, maxiter=max_iter)
    dt = time.time() - t0
    return (counter, dt) if with_time else counter


def get_pcg_iter_time_scipy(A: csr_matrix, gt: np.ndarray, spai: csr_matrix, epsilon: float, max_iter=0, rtol=1e-6,
                            dtype=np.float64, with_time: bool = False):
    """validate.py:163-201: M r = L (Lᵀ r) + ε r with Lᵀ an explicit CSR (``csr_matrix(spai.T)``)."""
    max_iter = max_iter if max_iter > 0 else A.shape[0]
    A = A.astype(dtype)
    spai = spai.astype(dtype)
    lt = csr_matrix(spai.T)
    M = _Op(lambda x: spai @ (lt @ x) + epsilon * x, spai.shape, spai.dtype)
    return _count(A, A @ gt, M, rtol, max_iter, with_time)


def get_pcg_diagonal_iter_time_scipy(A: csr_matrix, gt: np.ndarray, max_iter=0, rtol=1e-6, dtype=np.float64,
                                     with_time: bool = False):
    """validate.py:235-264: M r = r / diag(A)."""
    max_iter = max_iter if max_iter > 0 else A.shape[0]
    A = A.astype(dtype)
    d = A.diagonal()
    return _count(A, A @ gt, _Op(lambda x: x / d, A.shape, d.dtype), rtol, max_iter, with_time)


def get_pcg_scaled_iter_time_scipy(A: csr_matrix, gt: np.ndarray, spai: csr_matrix, epsilon: float, rtol=1e-6,
                                   max_iter=0, dtype=np.float64, with_time: bool = False):
    """validate.py:267-302: M r = L ((Lᵀ r) / d) + ε r / d, d = diag(A)."""
    max_iter = max_iter if max_iter > 0 else A.shape[0]
    A = A.astype(dtype)
    spai = spai.astype(dtype)
    lt = csr_matrix(spai.T)
    d = A.diagonal()
    M = _Op(lambda x: spai @ ((lt @ x) / d) + epsilon * x / d, spai.shape, spai.dtype)
    return _count(A, A @ gt, M, rtol, max_iter, with_time)


def get_cg_iter_time_scipy(A: csr_matrix, gt: np.ndarray, max_iter=0, rtol=1e-6, dtype=np.float64,
                           with_time: bool = False):
    """validate.py:316-333: unpreconditioned CG."""
    max_iter = max_iter if max_iter > 0 else A.shape[0]
    A = A.astype(dtype)
    return _count(A, A @ gt, None, rtol, max_iter, with_time)


def neural_row(A: csr_matrix, r: np.ndarray, L: csr_matrix, epsilon: float, rtol: float, scaled: bool = False,
               repeat: int = 1, threads: Optional[int] = None):
    """The ``Neural`` row (infer.py:322-330): ``(iters, solve_s)`` of the host ext_spai solve,
    averaged over ``repeat`` solves, at ``threads`` BLAS threads (None: the process default)."""
    fn = get_pcg_scaled_iter_time_scipy if scaled else get_pcg_iter_time_scipy
    return _repeat(lambda: fn(A, r, L, epsilon, rtol=rtol, with_time=True), repeat, threads)


def baseline_row(A: csr_matrix, r: np.ndarray, method: str, rtol: float, repeat: int = 1,
                 threads: Optional[int] = None):
    """A ``PCG-{method}-cpu`` row (infer.py:310-321) for method none / diagonal: ``(iters, solve_s)``.
    Like the reference's get_cg_iter_time, a solve that reaches max_iter raises RuntimeError."""
    fn = {"none": get_cg_iter_time_scipy, "diagonal": get_pcg_diagonal_iter_time_scipy}.get(method)
    if fn is None:
        raise ValueError(f"no host restatement of the {method!r} row (pymathprim / ilupp are absent)")

    def one():
        it, dt = fn(A, r, rtol=rtol, with_time=True)
        if it >= A.shape[0]:
            raise RuntimeError("CG did not converge")
        return it, dt

    return _repeat(one, repeat, threads)


def _repeat(fn, repeat: int, threads: Optional[int]):
    from contextlib import nullcontext

    ctx = nullcontext()
    if threads is not None:
        from threadpoolctl import threadpool_limits

        ctx = threadpool_limits(limits=int(threads))
    its, ts = 0.0, 0.0
    with ctx:
        for _ in range(max(1, int(repeat))):
            it, dt = fn()
            its += it
            ts += dt
    return its / max(1, int(repeat)), ts / max(1, int(repeat))
