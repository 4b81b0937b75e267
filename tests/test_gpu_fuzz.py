"""Randomised parity sweep: seeded random SPD systems of assorted sizes / row-length spreads,
random ext_spai factors (fp64 and fp32-exact values, so both the fp64 and the compact fp32-value
views run), GPU PCG against the oracle with correctly rounded dots: equal iteration count,
residual history and iterate 1e-12.  Sizes cross the SELL slice (64 rows), workgroup (256)
and group (64 workgroups) boundaries."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import linalg as O
from tests import _cases

pytestmark = pytest.mark.gpu


def _random_spd(n, seed):
    rng = np.random.default_rng(seed)
    per_row = rng.integers(1, 12, size=n)  # ragged rows
    rows = np.repeat(np.arange(n), per_row)
    span = max(2, int(rng.integers(2, max(3, n // 4))))
    cols = np.clip(rows + rng.integers(-span, span + 1, size=rows.size), 0, n - 1)
    B = sp.csr_matrix((rng.normal(size=rows.size), (rows, cols)), shape=(n, n))
    A = (B + B.T).tocsr()
    A.data = np.abs(A.data) * -1.0
    A.setdiag(0.0)
    A.eliminate_zeros()
    d = -np.asarray(A.sum(axis=1)).ravel() + rng.uniform(0.01, 1.0, size=n)
    A = (A + sp.diags(d)).tocsr()
    A.sort_indices()
    return A


SIZES = [63, 65, 257, 1000, 4097, 17000, 70000, 150000]


MODES = {  # "multi": the multi-kernel schedules at every size; "small": n <= 2560 runs k_pcg_small
    "multi": {"LSPCG_SMALL_N": "0"},
    "small": {"LSPCG_SMALL_N": "4096"},
}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("seed", range(16))
def test_random_spd_pcg_parity(gpu_ctx, seed, mode, monkeypatch):
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    rng = np.random.default_rng(100 + seed)
    n = SIZES[seed % len(SIZES)]
    A = _random_spd(n, seed)
    L = _cases.spai_like(A, seed=seed)
    if seed % 2:  # fp32-exact factor values: the compact (fp32-stored) views
        L.data = L.data.astype(np.float32).astype(np.float64)
    b = A @ rng.uniform(-1.0, 1.0, size=n)
    eps = float(rng.choice([1e-3, 3e-3]))
    it_o, x_o, h_o = O.pcg(A, b, O.spai_operator(L, eps), rtol=1e-8, max_iter=400, dot="exact")
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
    x = np.zeros(n)
    it, _, _, h = s(b.copy(), x, 1e-8, 400, ext_spai=(L, eps), return_history=True)
    assert it == it_o, (n, seed, it, it_o)
    np.testing.assert_allclose(h, h_o, rtol=1e-12, atol=0)
    assert np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


OB_SIZES = [37, 1000, 5000, 10001, 16417, 33000, 70000]


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("n", OB_SIZES)
def test_random_spd_openblas_order_bitexact(gpu_ctx, n, threads):
    """Parity mode (dot_order="openblas") on random systems: k_dot_openblas's chains, register
    double buffers (even / odd group counts, partial 16-element step, sequential tail) and the
    OpenBLAS thread split for n > 10,000 against oracle/openblas_ddot.c: count, every ‖r_k‖ and x
    bit for bit."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    rng = np.random.default_rng(7 * n + threads)
    A = _random_spd(n, n + threads)
    L = _cases.spai_like(A, seed=n)
    b = A @ rng.uniform(-1.0, 1.0, size=n)
    it_o, x_o, h_o = O.pcg(A, b, O.spai_operator(L, 3e-3), rtol=1e-8, max_iter=300, dot=f"blas{threads}")
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dot_order="openblas",
                                        dot_threads=threads)
    x = np.zeros(n)
    it, _, _, h = s(b.copy(), x, 1e-8, 300, ext_spai=(L, 3e-3), return_history=True)
    assert it == it_o, (n, threads, it, it_o)
    assert np.array_equal(np.asarray(h[:it]), np.asarray(h_o[:it])), (n, threads)
    assert np.array_equal(x, x_o), (n, threads, float(np.abs(x - x_o).max()))
