"""GPU parity: the baseline preconditioners (pymathprim "ic" / "ainv" rows of infer.py:310-321)
against oracle/precond.py -- factors and triangular solves bit-identical, PCG iteration
counts equal, solutions within 1e-12 (fp64)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from oracle import precond as OP
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _masked(A, mask):
    M = O.apply_dbc_masking(sp.csr_matrix(A), mask).tocsr()
    M.eliminate_zeros()
    M.sort_indices()
    return M


def _systems():
    A1, m1, _ = P.poisson2d_grid(16, 16)
    A2, m2 = P.kuhn_dirichlet(7)
    return {"poisson16": (_masked(A1, m1), m1.ravel()), "kuhn7": (_masked(A2, m2), m2.ravel()),
            "heat": (sp.csr_matrix(P.kuhn_laplacian(6, 1e-2)), None)}


def _dm(A, dtype=np.float64):
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    return DeviceMatrix.from_scipy(A, dtype=dtype)


@pytest.mark.parametrize("name", ["poisson16", "kuhn7", "heat"])
def test_ic0_factor_bitwise(gpu_ctx, name):
    A, _ = _systems()[name]
    L, _t = _dm(A).ic0()
    Lg = L.to_scipy()
    Lo = OP.ic0(A)
    assert np.array_equal(Lg.indptr, Lo.indptr) and np.array_equal(Lg.indices, Lo.indices)
    np.testing.assert_array_equal(Lg.data, Lo.data)


@pytest.mark.parametrize("name", ["poisson16", "kuhn7", "heat"])
def test_ainv0_factor_bitwise(gpu_ctx, name):
    A, _ = _systems()[name]
    L, _t = _dm(A).ainv0()
    Lg = L.to_scipy()
    Lo = OP.ainv_spai_factor(A)
    assert np.array_equal(Lg.indptr, Lo.indptr) and np.array_equal(Lg.indices, Lo.indices)
    np.testing.assert_array_equal(Lg.data, Lo.data)


@pytest.mark.parametrize("name", ["kuhn7", "kuhn31", "poisson100"])
def test_trsv_bitwise(gpu_ctx, name):
    """The sync-free one-launch solve (many blocks waiting on each other across 90-200 levels)
    gives the oracle's bits."""
    if name == "kuhn31":
        A = sp.csr_matrix(P.kuhn_laplacian(31))
    elif name == "poisson100":
        A1, m1, _ = P.poisson2d_grid(100, 100)
        A = _masked(A1, m1)
    else:
        A, _ = _systems()[name]
    L = OP.ic0(A)
    U = sp.csr_matrix(L.T)
    U.sort_indices()
    r = np.random.default_rng(3).normal(size=A.shape[0])
    rt = torch.from_numpy(r).cuda()
    y = _dm(L).trsv(rt, lower=True).cpu().numpy()
    np.testing.assert_array_equal(y, OP.trsv_lower(L, r))
    z = _dm(U).trsv(rt, lower=False).cpu().numpy()
    np.testing.assert_array_equal(z, OP.trsv_upper(U, r))


@pytest.mark.parametrize("method", ["ic", "ainv"])
@pytest.mark.parametrize("name", ["poisson16", "kuhn7", "heat"])
@pytest.mark.parametrize("rtol", [1e-6, 1e-8])
def test_pcg_baseline_counts_and_solution(gpu_ctx, method, name, rtol):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A, m = _systems()[name]
    gt = m if m is not None else np.ones(A.shape[0])
    b = A @ gt
    if method == "ic":
        ps = OP.ic_operator(OP.ic0(A))
    else:
        ps = O.spai_operator(OP.ainv_spai_factor(A), 0.0)
    it_o, x_o, _ = O.pcg(A, b, ps, rtol=rtol, dot="exact")
    solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner=method)
    x = np.zeros_like(b)
    it, prec, solve = solver(b, x, rtol=rtol)
    assert it == it_o, (method, name, it, it_o)
    assert prec > 0 and solve > 0
    assert np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


def test_get_cg_iter_time_baselines(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.validate import get_cg_iter_time

    A, m = _systems()["poisson16"]
    its = {mth: get_cg_iter_time(A, m, rtol=1e-8, method=mth, device="cuda")[0] for mth in ("none", "diagonal", "ainv", "ic")}
    assert its["ic"] < its["none"] and its["ainv"] < its["none"], its


def test_ic0_breakdown_is_reported(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd import _lib

    A = sp.csr_matrix(np.array([[1.0, 2.0], [2.0, 1.0]]))  # indefinite: pivot 1 - 4 < 0
    with pytest.raises(_lib.LspcgError) as e:
        _dm(A).ic0()
    assert e.value.code == _lib.ERR_BREAKDOWN


def test_ic_concurrent_solves_match_sequential(gpu_ctx):
    """Sync-free IC triangular solves under contention: four PCG-IC solves in flight on separate
    streams (linalg.solve_many: the solves' resident grids share the CUs and the hardware queues,
    so hand-offs wait behind other work) give the sequential results bit for bit -- a delayed
    dependency only waits longer (a wait beyond 2 s would fail the solve loudly, never silently)."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient, solve_many

    A = sp.csr_matrix(P.kuhn_laplacian(31, 1e-3))
    n = A.shape[0]
    b = torch.from_numpy(A @ np.ones(n)).cuda()
    solvers = [PreconditionedConjugateGradient(A, device="cuda", preconditioner="ic") for _ in range(4)]
    xs = [torch.zeros(n, dtype=torch.float64, device="cuda") for _ in solvers]
    seq = solvers[0].solve(b, xs[0].clone(), rtol=1e-8)
    x_seq = xs[0].clone()
    solvers[0].solve(b, x_seq, rtol=1e-8)
    res = solve_many([(s, b, x) for s, x in zip(solvers, xs)], rtol=1e-8, concurrency=4)
    for (it, conv, _), x in zip(res, xs):
        assert conv and it == seq[0]
        assert torch.equal(x, x_seq)


@pytest.mark.parametrize("dot_order", ["compensated", "openblas"])
@pytest.mark.parametrize("name", ["poisson16", "kuhn7", "poisson64"])
def test_pcg_ic_apply_matches_reference_ichol(gpu_ctx, name, dot_order):
    """PCG-IC with a GIVEN factor (lspcg_solver_set_ic_factor) vs the REFERENCE's
    get_pcg_iter_time_scipy_ichol on that factor (tests/golden/ic_traj.npz; validate.py:372-419,
    IncompleteCholeskyPreconditioner = two spsolve_triangular calls, whose arithmetic the device
    solves reproduce): counts equal, ‖r_k‖ within 1e-12 of max ‖r_k‖, x within 1e-12; in the recorded
    run's dot order, count, history and x bit for bit.  The factor is the oracle's IC(0) (the reference's ilupp
    factorization is absent: its arithmetic stays parity-unpinned; the device IC(0) equals the
    oracle's bit for bit, test_ic0_factor_bitwise)."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from tests.test_oracle_golden import _load, hist_dev, ic_system

    z = _load("ic_traj.npz")
    A, L, gt = ic_system(z, name)
    b = A @ gt
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ic", dot_order=dot_order)
    assert s.set_ic_factor(L) > 0
    for rtol in (6, 8):
        t = f"{name}__rtol{rtol}"
        x = np.zeros_like(b)
        it, _, _, h = s(b, x, 10.0 ** -rtol, return_history=True)
        assert it == int(z[f"{t}__count"]), (name, rtol, it)
        if dot_order == "openblas":  # the recorded run's own dot order: the same bits
            assert np.array_equal(h[:it], z[f"{t}__hist"]) and np.array_equal(x, z[f"{t}__x"])
        assert hist_dev(h, z[f"{t}__hist"]) <= 1e-12
        assert np.linalg.norm(x - z[f"{t}__x"]) <= 1e-12 * np.linalg.norm(z[f"{t}__x"])


def test_set_ic_factor_rejects_non_lower(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd import _lib
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.kuhn_laplacian(4))
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ic")
    with pytest.raises(_lib.LspcgError) as e:
        s.set_ic_factor(sp.csr_matrix(sp.triu(A)))
    assert e.value.code == _lib.ERR_FORMAT


def test_set_ic_factor_zero_diagonal_raises_like_spsolve_triangular(gpu_ctx):
    """a given factor with a zero diagonal entry is refused at installation with the
    error the reference's apply raises (scipy spsolve_triangular: LinAlgError "A is singular"),
    not a solve that stops as non-finite."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.kuhn_laplacian(4))
    L = sp.csr_matrix(sp.tril(A))
    L.sort_indices()
    L.data[L.indptr[6] - 1] = 0.0  # row 5's diagonal (stored last), kept as an explicit zero
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ic")
    with pytest.raises(np.linalg.LinAlgError, match="singular"):
        s.set_ic_factor(L)
    with pytest.raises(np.linalg.LinAlgError):  # the reference's own apply on the same factor
        from scipy.sparse.linalg import spsolve_triangular

        spsolve_triangular(L, np.ones(A.shape[0]), lower=True)
