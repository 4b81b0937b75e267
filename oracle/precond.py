"""CPU restatement of the baseline preconditioners -- TEST INFRASTRUCTURE ONLY.

The reference calls pymathprim's ``ic`` and ``ainv`` preconditioners (``infer.py:310-321``,
``validate.py:54-86``); pymathprim is unvendored and unversioned, so their arithmetic is
**parity unpinned** (SURVEY.md 8(c)).  This module fixes the published algorithms the GPU
implements, with an explicit operation order, so the HIP factors can be checked bit for bit:

* IC(0) -- incomplete Cholesky with the sparsity of tril(A) (row-oriented "up-looking" form).
  Its APPLY is the reference's own scipy restatement ``IncompleteCholeskyPreconditioner``
  (validate.py:344-369: two spsolve_triangular calls), restated bit for bit below and pinned
  against the reference's get_pcg_iter_time_scipy_ichol trajectories (ic_traj.npz).
* AINV(0) -- Benzi & Tůma's factorized approximate inverse A⁻¹ ≈ Z D⁻¹ Zᵀ by incomplete
  A-biconjugation (symmetric case), Z unit upper triangular restricted to the pattern of
  triu(A) (left-looking form; identical arithmetic to the right-looking one).  Applied as
  ``L Lᵀ`` with ``L = Z D^{-1/2}``, i.e. through the ext_spai path with ε = 0.

Pure Python loops: small systems only.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Tuple

import numpy as np
import scipy.sparse as sp


def _rows(M: sp.csr_matrix) -> List[Tuple[np.ndarray, np.ndarray]]:
    M = sp.csr_matrix(M)
    M.sort_indices()
    return [(M.indices[M.indptr[i]:M.indptr[i + 1]], M.data[M.indptr[i]:M.indptr[i + 1]]) for i in range(M.shape[0])]


def ic0(A: sp.csr_matrix) -> sp.csr_matrix:
    """IC(0): L lower triangular with the pattern of tril(A), A ≈ L Lᵀ.

    Row i, in increasing column k < i:  s = A_ik; s -= L_im L_km for common m < k in
    increasing m; L_ik = s / L_kk.  Then s = A_ii; s -= L_im L_im (increasing m < i);
    L_ii = sqrt(s).  Raises on a non-positive pivot (breakdown)."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    rows = _rows(sp.tril(A, format="csr"))
    L: List[Dict[int, float]] = []
    for i in range(n):
        cols, vals = rows[i]
        li: Dict[int, float] = {}
        aii = None
        for k, a in zip(cols.tolist(), vals.tolist()):
            if k == i:
                aii = a
                continue
            s = a
            lk = L[k]
            for m in sorted(li):
                if m >= k:
                    break
                if m in lk:
                    s = s - li[m] * lk[m]
            li[k] = s / lk[k]
        if aii is None:
            raise ValueError(f"IC(0): row {i} has no diagonal entry")
        s = aii
        for m in sorted(li):
            s = s - li[m] * li[m]
        if not s > 0.0:
            raise ValueError(f"IC(0) breakdown at row {i} (pivot {s})")
        li[i] = math.sqrt(s)
        L.append(li)
    indptr = np.zeros(n + 1, dtype=np.int64)
    indices, data = [], []
    for i, li in enumerate(L):
        ks = sorted(li)
        indices += ks
        data += [li[k] for k in ks]
        indptr[i + 1] = len(indices)
    return sp.csr_matrix((np.array(data), np.array(indices, dtype=np.int32), indptr), shape=(n, n))


# The reference's IC apply (validate.py:359-365) is scipy.sparse.linalg.spsolve_triangular on
# csc(L) then csc(Lᵀ).  scipy 1.15's arithmetic (scipy/sparse/linalg/_dsolve/linsolve.py
# spsolve_triangular -> SuperLU gstrs), restated: the columns are scaled by inv = 1/diag
# (A @ diags(inv)); the unit triangular solve then runs column by column, x_i -= x_j * A'_ij, so
# row i receives its updates in increasing j for the lower solve and in DECREASING j for the
# upper one; the lower solve's U phase divides by the scaled diagonal c = d * inv (not always
# exactly 1), the upper's L phase by 1; finally x *= inv.  Verified bit for bit against
# spsolve_triangular (tests/test_oracle_golden.py::test_trsv_is_spsolve_triangular).
def trsv_lower(L: sp.csr_matrix, r: np.ndarray) -> np.ndarray:
    """spsolve_triangular(csc(L), r, lower=True): y_i = r_i - Σ_{k<i, increasing} y_k (L_ik inv_k);
    x_i = (y_i / (d_i inv_i)) inv_i."""
    rows = _rows(L)
    d = np.asarray(sp.csr_matrix(L).diagonal(), dtype=np.float64)
    inv = 1.0 / d
    y = np.zeros(len(r))
    for i, (cols, vals) in enumerate(rows):
        s = float(r[i])
        for k, v in zip(cols.tolist(), vals.tolist()):
            if k < i:
                s = s - y[k] * (v * inv[k])
        y[i] = s
    return (y / (d * inv)) * inv


def trsv_upper(U: sp.csr_matrix, r: np.ndarray) -> np.ndarray:
    """spsolve_triangular(csc(U), r, lower=False): rows from the last, y_i = r_i - Σ_{j>i,
    DECREASING j} y_j (U_ij inv_j); x_i = y_i inv_i."""
    rows = _rows(U)
    d = np.asarray(sp.csr_matrix(U).diagonal(), dtype=np.float64)
    inv = 1.0 / d
    y = np.zeros(len(r))
    for i in range(len(r) - 1, -1, -1):
        cols, vals = rows[i]
        s = float(r[i])
        for j, v in zip(reversed(cols.tolist()), reversed(vals.tolist())):
            if j > i:
                s = s - y[j] * (v * inv[j])
        y[i] = s
    return y * inv


def ic_operator(L: sp.csr_matrix) -> Callable[[np.ndarray], np.ndarray]:
    """z = L⁻ᵀ L⁻¹ r (validate.py:358-365 IncompleteCholeskyPreconditioner._matvec: two
    spsolve_triangular calls), Lᵀ as an explicit CSR."""
    L = sp.csr_matrix(L)
    U = sp.csr_matrix(L.T)
    U.sort_indices()
    return lambda r: trsv_upper(U, trsv_lower(L, r))


def ainv0(A: sp.csr_matrix) -> Tuple[sp.csr_matrix, np.ndarray]:
    """AINV(0): returns (Zᵀ as CSR with the pattern of tril(A), d) with A⁻¹ ≈ Z D⁻¹ Zᵀ.

    Column j of Z (pattern P_j = {k <= j : A_kj != 0}, z_jj = 1): for every i < j whose row of A
    meets P_j, in increasing i:  p = Σ_{k in P_j} A_ik z_k (increasing k); if p != 0:
    f = p / d_i and z_k -= f * Z_ki for k in P_j ∩ pattern(z_i) (increasing k).  Finally
    d_j = Σ_{k in P_j} A_jk z_k (increasing k).  Raises on d_j <= 0."""
    A = sp.csr_matrix(A)
    A.sort_indices()
    n = A.shape[0]
    arow = _rows(A)
    arow_d = [dict(zip(c.tolist(), v.tolist())) for c, v in arow]
    Z: List[Dict[int, float]] = []
    d = np.zeros(n)
    for j in range(n):
        P = sorted(k for k in arow[j][0].tolist() if k <= j)
        if j not in P:
            P.append(j)
            P.sort()
        z = {k: 0.0 for k in P}
        z[j] = 1.0
        cand = sorted({i for k in P for i in arow[k][0].tolist() if i < j})
        for i in cand:
            ai = arow_d[i]
            p = 0.0
            for k in P:
                if k in ai:
                    p = p + ai[k] * z[k]
            if p != 0.0:
                f = p / d[i]
                zi = Z[i]
                for k in P:
                    if k in zi:
                        z[k] = z[k] - f * zi[k]
        aj = arow_d[j]
        dj = 0.0
        for k in P:
            if k in aj:
                dj = dj + aj[k] * z[k]
        if not dj > 0.0:
            raise ValueError(f"AINV(0) breakdown at column {j} (pivot {dj})")
        d[j] = dj
        Z.append(z)
    indptr = np.zeros(n + 1, dtype=np.int64)
    indices, data = [], []
    for j, z in enumerate(Z):
        ks = sorted(z)
        indices += ks
        data += [z[k] for k in ks]
        indptr[j + 1] = len(indices)
    Zt = sp.csr_matrix((np.array(data), np.array(indices, dtype=np.int32), indptr), shape=(n, n))
    return Zt, d


def ainv_spai_factor(A: sp.csr_matrix) -> sp.csr_matrix:
    """L = Z D^{-1/2} (so that L Lᵀ = Z D⁻¹ Zᵀ): entries z_j[k] / sqrt(d_j), as CSR."""
    Zt, d = ainv0(A)
    Lt = Zt.copy()
    rows = np.repeat(np.arange(Zt.shape[0]), np.diff(Zt.indptr))
    Lt.data = Zt.data / np.sqrt(d)[rows]
    L = sp.csr_matrix(Lt.T)
    L.sort_indices()
    return L
