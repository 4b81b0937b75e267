"""CPU restatement of the reference's solver harness -- TEST INFRASTRUCTURE ONLY.

Follows ``/root/reference/neural_cg/utils/validate.py`` and
``/root/reference/neural_cg/data.py`` line by line (cited per function) and the
PCG recurrence of scipy 1.15 ``scipy/sparse/linalg/_isolve/iterative.py:305-422``
(the reference's CPU restatement calls ``scipy.sparse.linalg.cg``).
"""
from __future__ import annotations

import math
import time
from typing import Callable, Optional, Tuple

import numpy as np
import scipy.sparse as sp
from scipy.sparse import bsr_matrix, coo_matrix, csr_matrix, diags
from scipy.sparse.linalg import LinearOperator, cg


# ---------------------------------------------------------------------------
# neural_cg/data.py:134-156 make_bsr_from_coo_inds
# ---------------------------------------------------------------------------
def make_bsr_from_coo_inds(bsr_values, rowinds, colinds, block_size, block_rows, block_cols) -> bsr_matrix:
    """data.py:134-156: pattern from (row, col) sorted via a CSR of ones, values
    taken in *input* order (assumes row-major sorted, duplicate-free edges)."""
    assert bsr_values.ndim == 3 and rowinds.size == colinds.size == bsr_values.shape[0]
    n = block_rows * block_size
    m = block_cols * block_size
    pat = csr_matrix((np.ones(rowinds.size), (rowinds, colinds)), shape=(block_rows, block_cols), copy=True)
    return bsr_matrix((bsr_values, pat.indices, pat.indptr), blocksize=(block_size, block_size),
                      shape=(n, m), copy=True)


# ---------------------------------------------------------------------------
# neural_cg/data.py:159-170 apply_dbc_masking
# ---------------------------------------------------------------------------
def apply_dbc_masking(mat, mask: np.ndarray):
    coo = coo_matrix(mat)
    mask_flat = mask.flatten()
    coo.data[mask_flat[coo.row] == 0] = 0
    coo.data[mask_flat[coo.col] == 0] = 0
    ident = (1 - mask_flat).copy()
    return coo + diags(ident, 0, shape=coo.shape)


# ---------------------------------------------------------------------------
# neural_cg/utils/validate.py:22-51 to_csr_cpu
# ---------------------------------------------------------------------------
def to_csr(edge_index: np.ndarray, edge_attr: np.ndarray, n: int, mask: Optional[np.ndarray],
           dtype=np.float64) -> csr_matrix:
    edge_index = np.asarray(edge_index)
    edge_attr = np.asarray(edge_attr)
    assert edge_index.ndim == 2 and edge_index.shape[0] == 2
    assert edge_attr.ndim in [1, 3]
    row, col = edge_index
    bsize = edge_attr.shape[-1]
    row_np = row.astype(np.int32)
    col_np = col.astype(np.int32)
    vals = edge_attr.astype(dtype)
    if vals.ndim == 3 and vals.shape[1] > 1:
        mat = make_bsr_from_coo_inds(vals, row_np, col_np, bsize, n // bsize, n // bsize)
    else:
        mat = csr_matrix((vals.flatten(), (row_np, col_np)), shape=(n, n), dtype=dtype)
    if mask is not None:
        mat = apply_dbc_masking(mat, mask=np.asarray(mask).flatten().astype(dtype))
    return csr_matrix(mat).sorted_indices()


# ---------------------------------------------------------------------------
# Preconditioners (validate.py:173-182, :243-251, :276-286)
# ---------------------------------------------------------------------------
def spai_operator(spai: csr_matrix, epsilon: float) -> Callable[[np.ndarray], np.ndarray]:
    """validate.py:173-182: ``z = L (Lᵀ r) + ε r`` with an explicit CSR ``Lᵀ``."""
    trans = csr_matrix(spai.T)
    return lambda x: spai @ (trans @ x) + epsilon * x


def spai_scaled_operator(A: csr_matrix, spai: csr_matrix, epsilon: float):
    """validate.py:276-286: ``z = L((Lᵀ r)/d) + ε r/d``, d = diag(A)."""
    trans = csr_matrix(spai.T)
    d = A.diagonal()
    return lambda x: spai @ ((trans @ x) / d) + epsilon * x / d


def diagonal_operator(A: csr_matrix):
    """validate.py:243-251: ``z = r / diag(A)``."""
    d = A.diagonal()
    return lambda x: x / d


# ---------------------------------------------------------------------------
# Dot products
# ---------------------------------------------------------------------------
def _two_prod(a: np.ndarray, b: np.ndarray):
    """Dekker TwoProduct (exact p + e = a*b), vectorised, no FMA needed."""
    p = a * b
    f = 134217729.0  # 2^27 + 1

    def split(x):
        c = f * x
        h = c - (c - x)
        return h, x - h

    ah, al = split(a)
    bh, bl = split(b)
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, e


def exact_dot(a: np.ndarray, b: np.ndarray) -> float:
    """Correctly rounded fp64 dot product (exact products + math.fsum)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    p, e = _two_prod(a, b)
    return math.fsum(np.concatenate([p, e]))


def pairwise_dot(a: np.ndarray, b: np.ndarray) -> float:
    """numpy pairwise summation of the products (a different, equally valid rounding order)."""
    return float(np.sum(np.asarray(a) * np.asarray(b)))


def openblas_dot(a: np.ndarray, b: np.ndarray, threads: int = 1) -> float:
    """The reference's own dot: numpy's cblas_ddot = OpenBLAS 0.3.29 (SkylakeX kernel) with
    ``threads`` OpenBLAS threads, restated in C (oracle/openblas_ddot.c, which cites the
    algorithm).  Equals np.dot bit for bit in the container the fixtures were made in."""
    from ._cbuild import lib

    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    assert a.shape == b.shape and a.ndim == 1
    return float(lib().lspcg_oracle_openblas_ddot(a.size, a.ctypes.data, b.ctypes.data, int(threads)))


# Dot orderings of the scipy-ordered PCG: "numpy" (whatever BLAS this process has -- the
# reference itself when run where the fixtures were made), "blas<T>" (that BLAS restated at T
# OpenBLAS threads: the recorded reference runs, machine independent), "exact" (correctly
# rounded: the HIP path's default compensated dots), "pairwise" (numpy's pairwise sum).
DOTS = {"numpy": np.dot, "exact": exact_dot, "pairwise": pairwise_dot,
        "blas1": lambda a, b: openblas_dot(a, b, 1), "blas8": lambda a, b: openblas_dot(a, b, 8)}


def dot_fn(dot: str):
    if dot in DOTS:
        return DOTS[dot]
    if dot.startswith("blas"):
        t = int(dot[4:])
        return lambda a, b: openblas_dot(a, b, t)
    raise KeyError(dot)


# ---------------------------------------------------------------------------
# scipy 1.15 cg, restated with a pluggable dot and recorded residual history
# ---------------------------------------------------------------------------
def pcg(A: csr_matrix, b: np.ndarray, psolve: Optional[Callable] = None, rtol: float = 1e-6,
        max_iter: int = 0, x0: Optional[np.ndarray] = None, dot: str = "numpy", dtype=np.float64):
    """scipy ``cg`` (iterative.py:359-418) restated.

    Returns ``(iters, x, res_hist)``; ``iters`` counts callbacks exactly like
    ``validate.py:189-199`` and ``res_hist[k] = ‖r_k‖`` (recurrence residual,
    the value compared with ``atol`` at the top of iteration k).
    ``dot='numpy'`` reproduces scipy bit-for-bit; ``dot='exact'`` replaces every
    dot/norm with the correctly rounded one (the HIP path's reductions).
    """
    dt = np.dtype(dtype).type
    d0 = dot_fn(dot)
    # scipy's scalars have the vectors' dtype (np.dot of float32 arrays is a float32): ρ, π, α, β
    # and ‖r‖ are rounded to it before they are used (a no-op for fp64)
    d = (lambda u, v: dt(d0(u, v))) if dot != "numpy" else d0
    b = np.asarray(b, dtype=dtype)
    n = b.shape[0]
    max_iter = max_iter if max_iter > 0 else n
    bnrm2 = np.sqrt(d(b, b)) if dot != "numpy" else np.linalg.norm(b)
    atol = max(0.0, float(rtol) * float(bnrm2))
    x = np.zeros_like(b) if x0 is None else np.array(x0, dtype=dtype)
    hist = []
    if bnrm2 == 0:
        return 0, b.copy(), [0.0]
    r = b - A @ x if x.any() else b.copy()
    rho_prev, p = None, None
    for iteration in range(max_iter):
        rn = np.sqrt(d(r, r)) if dot != "numpy" else np.linalg.norm(r)
        hist.append(float(rn))
        if rn < atol:
            return iteration, x, hist
        z = psolve(r) if psolve is not None else r
        rho_cur = d(r, z)
        if iteration > 0:
            beta = rho_cur / rho_prev
            p *= beta
            p += z
        else:
            p = np.empty_like(r)
            p[:] = z[:]
        q = A @ p
        alpha = rho_cur / d(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho_cur
    hist.append(float(np.sqrt(d(r, r)) if dot != "numpy" else np.linalg.norm(r)))
    return max_iter, x, hist


# ---------------------------------------------------------------------------
# The reference's scipy entry points (validate.py:163-201, :235-264, :267-302,
# :316-333), restated with timing as validate.py:196-198.
# ---------------------------------------------------------------------------
class _Op(LinearOperator):
    def __init__(self, fn, shape, dtype):
        self._fn = fn
        super().__init__(dtype, shape)

    def _matvec(self, x):
        return self._fn(x)


def _count_cg(A, b, M, rtol, max_iter):
    counter = 0

    def cb(_x):
        nonlocal counter
        counter += 1

    t0 = time.time()
    cg(A, b, M=M, callback=cb, rtol=rtol, maxiter=max_iter)
    return counter, time.time() - t0


def get_pcg_iter_time_scipy(A, gt, spai, epsilon, max_iter=0, rtol=1e-6, dtype=np.float64, with_time=False):
    rows = A.shape[0]
    max_iter = max_iter if max_iter > 0 else rows
    A = A.astype(dtype)
    spai = spai.astype(dtype)
    M = _Op(spai_operator(spai, epsilon), spai.shape, spai.dtype)
    b = A @ gt
    c, t = _count_cg(A, b, M, rtol, max_iter)
    return (c, t) if with_time else c


def get_pcg_scaled_iter_time_scipy(A, gt, spai, epsilon, rtol=1e-6, max_iter=0, dtype=np.float64, with_time=False):
    rows = A.shape[0]
    max_iter = max_iter if max_iter > 0 else rows
    A = A.astype(dtype)
    spai = spai.astype(dtype)
    M = _Op(spai_scaled_operator(A, spai, epsilon), spai.shape, spai.dtype)
    b = A @ gt
    c, t = _count_cg(A, b, M, rtol, max_iter)
    return (c, t) if with_time else c


def get_pcg_diagonal_iter_time_scipy(A, gt, max_iter=0, rtol=1e-6, dtype=np.float64, with_time=False):
    rows = A.shape[0]
    max_iter = max_iter if max_iter > 0 else rows
    A = A.astype(dtype)
    M = _Op(diagonal_operator(A), A.shape, A.dtype)
    b = A @ gt
    c, t = _count_cg(A, b, M, rtol, max_iter)
    return (c, t) if with_time else c


def get_cg_iter_time_scipy(A, gt, max_iter=0, rtol=1e-6, dtype=np.float64, with_time=False):
    rows = A.shape[0]
    max_iter = max_iter if max_iter > 0 else rows
    A = A.astype(dtype)
    b = A @ gt
    c, t = _count_cg(A, b, None, rtol, max_iter)
    return (c, t) if with_time else c


def spmv(A: csr_matrix, x: np.ndarray) -> np.ndarray:
    """scipy csr_matvec: sequential per-row sum in index order (the bit pattern
    the HIP SpMV reproduces)."""
    return A @ x
