"""GPU parity of the batched lockstep ext_spai PCG (lspcg_batch_*, linalg.BatchedConjugateGradient).

Every system of a batch must come out as the single-system solver (and the oracle) returns it:
the same iteration count, the residual history and the iterate within 1e-12 relative (fp64;
1e-5 fp32) -- the batch sums each system's compensated dot partials per row tile instead of per
resident workgroup, so the dots are the same correctly rounded values in practice and the test
also records whether the bits agree.  Covers ragged system sizes (tile padding), small systems
(which the single-system path solves in one workgroup), BSR 3x3, a zero right-hand side, max_iter
stops and repeated solves on one batch.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from tests import _cases
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _systems():
    out = []
    for nx, ny in ((24, 20), (40, 33), (7, 9), (64, 64)):
        A, m, _ = P.poisson2d_grid(nx, ny)
        out.append(A)
    out.append(P.kuhn_laplacian(9))
    out.append(P.kuhn_laplacian(23))
    out.append(P.heat_tet(7, 6, 5)[0])
    return out


def _single(A, L, b, eps, rtol, max_iter=0, dtype=np.float64, bs=1):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=dtype, block_size=bs)
    s.set_spai(L, eps, block_size=bs)
    bt = torch.from_numpy(b.astype(dtype)).cuda()
    x = torch.zeros_like(bt)
    it, conv, _, h = s.solve(bt, x, rtol=rtol, max_iter=max_iter, return_history=True)
    return it, conv, x.cpu().numpy(), h


def _batch(As, Ls, bs_, eps, rtol, max_iter=0, dtype=np.float64, bsz=1):
    from learningsparsepreconditioner4gpu_amd.linalg import BatchedConjugateGradient

    B = BatchedConjugateGradient(As, Ls, eps, dtype=dtype, block_size=bsz)
    bt = [torch.from_numpy(b.astype(dtype)).cuda() for b in bs_]
    xs = [torch.zeros_like(b) for b in bt]
    res, t = B.solve(bt, xs, rtol=rtol, max_iter=max_iter, return_history=True)
    assert t > 0
    return B, res, [x.cpu().numpy() for x in xs]


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("reduce", ["auto", "0", "1"])
def test_batch_matches_single_and_oracle(gpu_ctx, monkeypatch, reduce):
    """reduce: the window's reductions (auto / 0 = per-system last arrivers / 1 = consumer sums)."""
    if reduce != "auto":
        monkeypatch.setenv("LSPCG_BATCH_REDUCE", reduce)
    eps = 3e-3
    As = _systems()
    Ls = [_cases.spai_like(A, seed=k) for k, A in enumerate(As)]
    bs_ = [A @ np.ones(A.shape[0]) for A in As]
    _, res, xs = _batch(As, Ls, bs_, eps, 1e-8)
    same_bits = 0
    for A, L, b, (it, conv, h), x in zip(As, Ls, bs_, res, xs):
        it1, conv1, x1, h1 = _single(A, L, b, eps, 1e-8)
        assert (it, conv) == (it1, conv1), (A.shape, it, it1)
        np.testing.assert_allclose(h, h1, rtol=1e-12, atol=0)
        assert _rel(x, x1) <= 1e-12
        same_bits += int(np.array_equal(x, x1))
        it_o, x_o, h_o = O.pcg(sp.csr_matrix(A), b, O.spai_operator(sp.csr_matrix(L), eps), rtol=1e-8, dot="exact")
        assert it == it_o
        np.testing.assert_allclose(h, h_o, rtol=1e-12, atol=0)
        assert _rel(x, x_o) <= 1e-12
    print(f"batch iterates bit-identical to single solves: {same_bits}/{len(As)}")


def test_batch_fp32(gpu_ctx):
    eps = 3e-3
    As = [A.astype(np.float32) for A in _systems()[:5]]
    Ls = [_cases.spai_like(A, seed=k).astype(np.float32) for k, A in enumerate(As)]
    bs_ = [(A @ np.ones(A.shape[0], np.float32)).astype(np.float32) for A in As]
    _, res, xs = _batch(As, Ls, bs_, eps, 1e-5, dtype=np.float32)
    for A, L, b, (it, conv, h), x in zip(As, Ls, bs_, res, xs):
        it1, conv1, x1, h1 = _single(A, L, b, eps, 1e-5, dtype=np.float32)
        assert (it, conv) == (it1, conv1)
        assert _rel(x.astype(np.float64), x1.astype(np.float64)) <= 1e-5
        # the oracle's fp32 scipy cg with correctly rounded dots (scalars rounded to fp32 like
        # numpy's float32 dots): the same count, x within the fp32 tolerance
        it_o, x_o, _ = O.pcg(sp.csr_matrix(A), b, O.spai_operator(sp.csr_matrix(L), np.float32(eps)), rtol=1e-5,
                             dot="exact", dtype=np.float32)
        assert it == it_o, (A.shape, it, it_o)
        assert _rel(x.astype(np.float64), x_o.astype(np.float64)) <= 1e-5


@pytest.mark.parametrize("reduce", ["0", "1"])
def test_batch_bsr3(gpu_ctx, monkeypatch, reduce):
    monkeypatch.setenv("LSPCG_BATCH_REDUCE", reduce)
    eps = 1e-3
    As = []
    for dims in ((9, 5, 5), (12, 6, 5), (5, 4, 4)):
        A, _, _ = P.elasticity_box(*dims)
        As.append(sp.csr_matrix(A))
    Ls = [_cases.spai_like(A, seed=k, scale=0.02) for k, A in enumerate(As)]
    bs_ = [A @ np.ones(A.shape[0]) for A in As]
    _, res, xs = _batch(As, Ls, bs_, eps, 1e-8, max_iter=60, bsz=3)
    for A, L, b, (it, conv, h), x in zip(As, Ls, bs_, res, xs):
        it1, conv1, x1, h1 = _single(A, L, b, eps, 1e-8, max_iter=60, bs=3)
        assert (it, conv) == (it1, conv1)
        np.testing.assert_allclose(h, h1, rtol=1e-12, atol=0)
        assert _rel(x, x1) <= 1e-12


def test_batch_edge_cases_and_reuse(gpu_ctx):
    """A zero right-hand side (scipy returns b, 0 iterations), per-system max_iter stops, and a
    second solve on the same batch with other right-hand sides."""
    eps = 3e-3
    As = _systems()[:4]
    Ls = [_cases.spai_like(A, seed=k) for k, A in enumerate(As)]
    rng = np.random.default_rng(0)
    bs_ = [A @ rng.normal(size=A.shape[0]) for A in As]
    bs_[1] = np.zeros(As[1].shape[0])
    B, res, xs = _batch(As, Ls, bs_, eps, 1e-10, max_iter=15)
    assert res[1][0] == 0 and res[1][1] and not xs[1].any()
    for k in (0, 2, 3):
        it1, conv1, x1, h1 = _single(As[k], Ls[k], bs_[k], eps, 1e-10, max_iter=15)
        assert (res[k][0], res[k][1]) == (it1, conv1)
        assert _rel(xs[k], x1) <= 1e-12
    # reuse: new right-hand sides, default max_iter (each system's n)
    bs2 = [A @ np.ones(A.shape[0]) for A in As]
    bt = [torch.from_numpy(b).cuda() for b in bs2]
    x2 = [torch.zeros_like(b) for b in bt]
    res2, _ = B.solve(bt, x2, rtol=1e-8)
    for k, A in enumerate(As):
        it1, conv1, x1, _ = _single(A, Ls[k], bs2[k], eps, 1e-8)
        assert (res2[k][0], res2[k][1]) == (it1, conv1)
        assert _rel(x2[k].cpu().numpy(), x1) <= 1e-12


def test_batch_rejects_mixed_inputs(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd._lib import LspcgError
    from learningsparsepreconditioner4gpu_amd.linalg import BatchedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A1, A2 = _systems()[:2]
    L1 = _cases.spai_like(A1)
    with pytest.raises(TypeError):  # one dtype per batch
        BatchedConjugateGradient([DeviceMatrix.from_scipy(A1), DeviceMatrix.from_scipy(A2, dtype=np.float32)],
                                 [DeviceMatrix.from_scipy(L1), DeviceMatrix.from_scipy(L1)], 1e-3)
    with pytest.raises(LspcgError):  # L of another size
        BatchedConjugateGradient([A1, A2], [L1, L1], 1e-3)
    B = BatchedConjugateGradient([A1], [L1], 1e-3)
    with pytest.raises(ValueError):
        B.solve([torch.zeros(A1.shape[0], dtype=torch.float32, device="cuda")],
                [torch.zeros(A1.shape[0], dtype=torch.float64, device="cuda")])


def test_batch_many_systems_memory_map(gpu_ctx):
    """More systems than the kernel-argument map holds (16): the tile -> system map is read from
    device memory instead; every system still equals its single solve."""
    eps = 3e-3
    As = []
    for k in range(18):
        A, _, _ = P.poisson2d_grid(9 + (k * 7) % 23, 8 + (k * 5) % 17)
        As.append(A)
    Ls = [_cases.spai_like(A, seed=k) for k, A in enumerate(As)]
    bs_ = [A @ np.ones(A.shape[0]) for A in As]
    _, res, xs = _batch(As, Ls, bs_, eps, 1e-8)
    for A, L, b, (it, conv, h), x in zip(As, Ls, bs_, res, xs):
        it1, conv1, x1, h1 = _single(A, L, b, eps, 1e-8)
        assert (it, conv) == (it1, conv1)
        np.testing.assert_allclose(h, h1, rtol=1e-12, atol=0)
        assert _rel(x, x1) <= 1e-12


@pytest.mark.parametrize("small", ["1", "0"])
def test_batch_small_systems_one_workgroup_each(gpu_ctx, monkeypatch, small):
    """Windows of systems that fit the one-workgroup solve run it with one workgroup per system in
    ONE launch (small = 1, the default) or the lockstep phases (LSPCG_BATCH_SMALL=0): either way each
    system matches its single solve (count, history, iterate), a zero rhs returns b and max_iter
    stops per system."""
    monkeypatch.setenv("LSPCG_BATCH_SMALL", small)
    eps = 3e-3
    As = [P.poisson2d_grid(nx, ny)[0] for nx, ny in ((24, 20), (40, 33), (7, 9), (45, 50))]
    As += [P.kuhn_laplacian(9), P.kuhn_laplacian(13), P.heat_tet(7, 6, 5)[0]]
    Ls = [_cases.spai_like(A, seed=k) for k, A in enumerate(As)]
    bs_ = [A @ np.ones(A.shape[0]) for A in As]
    bs_[2] = np.zeros(As[2].shape[0])
    for max_iter in (0, 12):
        _, res, xs = _batch(As, Ls, bs_, eps, 1e-9, max_iter=max_iter)
        assert res[2][0] == 0 and res[2][1] and not xs[2].any()
        for A, L, b, (it, conv, h), x in zip(As, Ls, bs_, res, xs):
            it1, conv1, x1, h1 = _single(A, L, b, eps, 1e-9, max_iter=max_iter)
            assert (it, conv) == (it1, conv1), (A.shape, it, it1)
            np.testing.assert_allclose(h, h1, rtol=1e-12, atol=0)
            assert _rel(x, x1) <= 1e-12 or not np.linalg.norm(x1)
