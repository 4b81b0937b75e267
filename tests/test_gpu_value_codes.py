"""GPU: SELL-DIA views with a value dictionary (1-byte codes; lspcg_sell.hip sdia_value_codes).

A matrix whose stored values take few distinct bit patterns (a structured grid's stencil: the
headline Kuhn-tet Laplacian has 9) keeps each slot as a one-byte index into a <= 256-entry
dictionary of the exact fp32 values, staged in LDS (opt-in: LSPCG_VALUE_CODES=1).  Every
multiply sees the same value, so the solve must be BIT-identical to the fp32-value views (the
default): count, every ‖r_k‖ and x.  Views with more than 256 values (the GNN's L) stay fp32.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from tests import _cases
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _system(kind):
    if kind == "kuhn41":
        A, m = P.kuhn_dirichlet(41)
    else:
        A, m0, _ = P.poisson2d_grid(128, 128)
        m = m0.ravel()
    A = sp.csr_matrix(A)
    A.sort_indices()
    A.data = A.data.astype(np.float32).astype(np.float64)
    L = _cases.spai_like(A, seed=1)
    L.data = L.data.astype(np.float32).astype(np.float64)
    return A, L, A @ np.asarray(m, dtype=np.float64).ravel()


def _solve(A, L, b, pre, monkeypatch, codes):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    monkeypatch.setenv("LSPCG_VALUE_CODES", "1" if codes else "0")
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=pre)
    if pre.startswith("ext_spai"):
        s.set_spai(L, 3e-3)
    bt = torch.as_tensor(b, device="cuda")
    x = torch.zeros_like(bt)
    it, conv, _t, h = s.solve(bt, x, rtol=1e-8, return_history=True)
    return s.views, it, conv, x.cpu().numpy(), h


@pytest.mark.parametrize("pre", ["none", "ext_spai", "ext_spai_scaled"])
@pytest.mark.parametrize("kind", ["kuhn41", "poisson128"])
def test_coded_views_bit_identical(gpu_ctx, monkeypatch, kind, pre):
    A, L, b = _system(kind)
    v1, it1, c1, x1, h1 = _solve(A, L, b, pre, monkeypatch, True)
    v0, it0, c0, x0, h0 = _solve(A, L, b, pre, monkeypatch, False)
    assert v1["A"] == {"columns": "sdia", "value_bytes": 1}, v1
    assert v0["A"]["value_bytes"] == 4, v0
    if pre.startswith("ext_spai"):
        assert v1["L"]["value_bytes"] == 4 and v1["LT"]["value_bytes"] == 4, v1  # continuous values
    assert c1 and it1 == it0 and np.array_equal(h1, h0) and np.array_equal(x1, x0), (it1, it0)
    ps = {"none": None, "ext_spai": O.spai_operator(L, 3e-3), "ext_spai_scaled": O.spai_scaled_operator(A, L, 3e-3)}[pre]
    it_o, x_o, _ = O.pcg(A, b, ps, rtol=1e-8, dot="exact")
    assert it1 == it_o and np.linalg.norm(x1 - x_o) <= 1e-12 * np.linalg.norm(x_o)


def test_coded_L_when_few_values(gpu_ctx, monkeypatch):
    """An L with few distinct values is coded too (all three views), still bit-identical."""
    A, _, b = _system("kuhn41")
    L = A.copy()
    L.data = np.where(A.indices == np.repeat(np.arange(A.shape[0]), np.diff(A.indptr)), 0.25, -0.015625)
    v1, it1, _, x1, h1 = _solve(A, L, b, "ext_spai", monkeypatch, True)
    _, it0, _, x0, h0 = _solve(A, L, b, "ext_spai", monkeypatch, False)
    assert all(v["value_bytes"] == 1 for v in v1.values()), v1
    assert it1 == it0 and np.array_equal(h1, h0) and np.array_equal(x1, x0)


def test_more_than_256_values_stay_fp32(gpu_ctx, monkeypatch):
    A, L, b = _system("kuhn41")
    A2 = A.copy()
    A2.data = (A2.data * (1 + 1e-3 * (np.arange(A2.nnz) % 300))).astype(np.float32).astype(np.float64)
    A2 = (A2 + A2.T) * 0.5  # symmetric again, > 256 distinct values
    A2 = sp.csr_matrix(A2)
    A2.sort_indices()
    A2.data = A2.data.astype(np.float32).astype(np.float64)
    v, it, conv, x, _ = _solve(A2, L, A2 @ np.ones(A2.shape[0]), "none", monkeypatch, True)
    assert v["A"]["value_bytes"] == 4, v
