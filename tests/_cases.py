"""Shared small test systems (CPU-side construction only)."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from learningsparsepreconditioner4gpu_amd import problems as P


def spai_like(A: sp.csr_matrix, seed: int = 0, scale: float = 0.05) -> sp.csr_matrix:
    """A factor on A's pattern: D^{-1/2} plus small random off-diagonal entries."""
    rng = np.random.default_rng(seed)
    A = sp.csr_matrix(A)
    L = A.copy().astype(np.float64)
    d = A.diagonal()
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    vals = rng.normal(size=A.nnz) * scale / np.sqrt(np.abs(d[rows]) + 1e-12)
    diag = rows == A.indices
    vals[diag] = 1.0 / np.sqrt(np.abs(d[rows[diag]]) + 1e-12)
    L.data = vals
    return L


def ragged_matrix(n: int = 3000, seed: int = 1) -> sp.csr_matrix:
    """Empty rows, a row longer than one SpMV chunk (5000 > 4096 entries), random lengths."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for i in range(n):
        if i % 97 == 5:
            continue  # empty row
        k = rng.integers(1, 40)
        c = rng.choice(n, size=k, replace=False)
        rows += [i] * k
        cols += list(c)
    k = min(2500, n)
    rows += [7] * k  # long row (+ beyond chunk with the neighbours)
    cols += list(rng.choice(n, size=k, replace=False))
    A = sp.csr_matrix((rng.normal(size=len(rows)), (rows, cols)), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    big = sp.csr_matrix((rng.normal(size=5000), (np.full(5000, 11), np.arange(5000) % n)), shape=(n, n))
    A = (A + big).tocsr()
    A.sort_indices()
    return A


def spd_cases():
    """(name, A, mask) small SPD systems covering the reference's configs."""
    out = []
    out.append(("synthetic-2048", P.generate_spd_sparse_matrix(2048, 2e-3, 1e-3, np.random.RandomState(3)), None))
    A, m, _ = P.poisson2d_grid(24, 20)
    out.append(("poisson2d-24x20", A, m))
    out.append(("kuhn-9", P.kuhn_laplacian(9), None))
    A, m, _ = P.heat_tet(7, 6, 5)
    out.append(("heat-tet", A, m))
    return out
