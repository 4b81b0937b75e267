"""GPU parity: HIP SpMV / dot / PCG through the C ABI vs the CPU oracle.

Tolerances (BASELINE.json north_star): SpMV and elementwise updates are bit-identical to
scipy; PCG iteration counts equal the oracle's exactly; solutions agree within 1e-12
relative (fp64) / 1e-5 (fp32).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from tests import _cases
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _dm(A, dtype=np.float64, bs=1):
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    return DeviceMatrix.from_scipy(A, dtype=dtype, block_size=bs)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("which", ["synthetic", "poisson", "kuhn", "ragged"])
def test_spmv_bitwise_vs_scipy(gpu_ctx, which, dtype):
    A = {
        "synthetic": lambda: P.generate_spd_sparse_matrix(3000, 3e-3, 1e-5, np.random.RandomState(0)),
        "poisson": lambda: P.poisson2d_grid(40, 33)[0],
        "kuhn": lambda: P.kuhn_laplacian(13),
        "ragged": lambda: _cases.ragged_matrix(),
    }[which]().astype(dtype)
    x = np.random.default_rng(5).normal(size=A.shape[0]).astype(dtype)
    ref = A @ x
    y = _dm(A, dtype).matvec(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(y, ref), np.max(np.abs(y - ref))


def test_spmv_bsr3_matches_scalar_csr(gpu_ctx):
    A, mask, _ = P.elasticity_box(10, 5, 4)
    x = np.random.default_rng(2).normal(size=A.shape[0])
    B = sp.bsr_matrix(A, blocksize=(3, 3))
    ref = B.tocsr() @ x  # scalar CSR incl. in-block zeros: same summation sequence as the BSR kernel
    y = _dm(A, np.float64, 3).matvec(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(y, ref)
    assert np.allclose(y, A @ x, rtol=1e-14, atol=1e-14 * np.abs(A @ x).max())


def test_empty_matrix_and_zero_rows(gpu_ctx):
    A = sp.csr_matrix((5, 5))
    y = _dm(A).matvec(torch.ones(5, dtype=torch.float64, device="cuda")).cpu().numpy()
    assert np.array_equal(y, np.zeros(5))


def test_dot_is_correctly_rounded(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.sparse import dot

    rng = np.random.default_rng(0)
    for n in [0, 1, 1000, 100_003]:
        a = rng.normal(size=n) * np.exp(rng.normal(size=n) * 5)
        b = rng.normal(size=n)
        got = dot(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda())
        assert got == O.exact_dot(a, b)


def test_transpose_and_diagonal(gpu_ctx):
    A = _cases.ragged_matrix(800)
    Ad = _dm(A)
    T = Ad.transpose().to_scipy()
    ref = sp.csr_matrix(A.T)
    ref.sort_indices()
    assert np.array_equal(T.indptr, ref.indptr) and np.array_equal(T.indices, ref.indices)
    assert np.array_equal(T.data, ref.data)
    assert np.array_equal(Ad.diagonal().cpu().numpy(), A.diagonal())
    Ae, _, _ = P.elasticity_box(6, 4, 3)
    Bd = _dm(Ae, np.float64, 3)
    Tb = Bd.transpose().to_scipy().tocsr()
    assert abs(Tb - sp.csr_matrix(Ae.T)).max() == 0
    assert np.array_equal(Bd.diagonal().cpu().numpy(), Ae.diagonal())


@pytest.mark.parametrize("bs", [1, 3])
def test_transpose_symmetric_pattern_fast_path(gpu_ctx, bs):
    # symmetric pattern, nonsymmetric values (the ext_spai factor's case): value permutation path
    B = P.kuhn_laplacian(6).tocsr()
    if bs == 3:
        B = sp.kron(B, np.ones((3, 3))).tocsr()
    A = B.copy()
    A.data = np.random.default_rng(1).normal(size=A.nnz)
    A.sort_indices()
    T = _dm(A, np.float64, bs).transpose().to_scipy()
    T = sp.csr_matrix(T)
    ref = sp.csr_matrix(A.T)
    assert abs(T - ref).max() == 0
    # one entry without its mirror -> the general path must take over
    A2 = A.tolil()
    A2[0, A.shape[0] - 1] = 5.0
    A2 = sp.csr_matrix(A2)
    A2.sort_indices()
    T2 = sp.csr_matrix(_dm(A2, np.float64, 1).transpose().to_scipy())
    assert abs(T2 - sp.csr_matrix(A2.T)).max() == 0


@pytest.mark.parametrize("bs", [1, 3])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_transpose_symmetric_many_rows_and_empty_rows(gpu_ctx, bs, dtype):
    # > 256 block rows (several workgroups of the entry-parallel kernel), isolated vertices
    # (empty rows AND columns keep the pattern symmetric) at a workgroup boundary and inside
    B = P.kuhn_laplacian(9).tocsr()  # 729 rows
    keep = np.ones(B.shape[0], dtype=bool)
    keep[[0, 255, 256, 257, 400, 728]] = False
    D = sp.diags(keep.astype(np.float64))
    B = sp.csr_matrix(D @ B @ D)
    B.eliminate_zeros()
    if bs == 3:
        B = sp.csr_matrix(sp.kron(B, np.ones((3, 3))))
    A = B.copy()
    A.data = np.random.default_rng(2).normal(size=A.nnz).astype(dtype)
    A.sort_indices()
    T = sp.csr_matrix(_dm(A, dtype, bs).transpose().to_scipy())
    assert abs(T - sp.csr_matrix(A.T)).max() == 0


def _solve(A, b, method, L=None, eps=3e-3, rtol=1e-8, dtype=np.float64, max_iter=0):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=method, dtype=dtype)
    x = np.zeros(A.shape[0], dtype=dtype)
    it, prec, solve, hist = s(b.astype(dtype), x, rtol, max_iter,
                              ext_spai=(L, eps) if L is not None else None, return_history=True)
    return it, x, hist


def _oracle_psolve(method, A, L, eps):
    if method == "none":
        return None
    if method == "diagonal":
        return O.diagonal_operator(A)
    if method == "ext_spai":
        return O.spai_operator(L, eps)
    return O.spai_scaled_operator(A, L, eps)


@pytest.mark.parametrize("method", ["none", "diagonal", "ext_spai", "ext_spai_scaled"])
@pytest.mark.parametrize("case", range(4))
def test_pcg_parity_fp64(gpu_ctx, method, case):
    name, A, mask = _cases.spd_cases()[case]
    gt = np.ones(A.shape[0]) if mask is None else mask.ravel().astype(np.float64)
    b = A @ gt
    L = _cases.spai_like(A, seed=case) if method.startswith("ext_spai") else None
    eps = 3e-3
    it_o, x_o, h_o = O.pcg(A, b, _oracle_psolve(method, A, L, eps), rtol=1e-8, dot="exact")
    it, x, h = _solve(A, b, method, L, eps)
    assert it == it_o, (name, method, it, it_o)
    rel = np.linalg.norm(x - x_o) / max(np.linalg.norm(x_o), 1e-300)
    assert rel <= 1e-12, (name, method, rel)
    assert len(h) == it + 1
    np.testing.assert_allclose(h, h_o, rtol=1e-12, atol=0)


@pytest.mark.parametrize("method", ["none", "ext_spai"])
def test_pcg_parity_fp32(gpu_ctx, method):
    A, mask, _ = P.poisson2d_grid(20, 18)
    A32 = A.astype(np.float32)
    gt = mask.ravel().astype(np.float32)
    b = (A32 @ gt).astype(np.float32)
    L = _cases.spai_like(A).astype(np.float32) if method == "ext_spai" else None
    eps = 3e-3
    psolve = None if L is None else O.spai_operator(L, np.float32(eps))
    it_o, x_o, _ = O.pcg(A32, b, psolve, rtol=1e-6, dot="exact", dtype=np.float32)
    it, x, _ = _solve(A32, b, method, L, eps, rtol=1e-6, dtype=np.float32)
    assert it == it_o
    assert np.linalg.norm(x - x_o) / np.linalg.norm(x_o) <= 1e-5


def test_pcg_max_iter_and_zero_rhs(gpu_ctx):
    A = P.kuhn_laplacian(7)
    b = A @ np.ones(A.shape[0])
    it, x, h = _solve(A, b, "none", max_iter=5)
    it_o, x_o, _ = O.pcg(A, b, None, rtol=1e-8, max_iter=5, dot="exact")
    assert it == it_o == 5
    assert np.linalg.norm(x - x_o) <= 1e-13 * np.linalg.norm(x_o)
    it, x, _ = _solve(A, np.zeros(A.shape[0]), "none")
    assert it == 0 and not x.any()


def test_validate_api_raises_when_not_converged(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.validate import get_cg_iter_time

    A = P.kuhn_laplacian(9)
    with pytest.raises(RuntimeError, match="CG did not converge"):
        get_cg_iter_time(A, np.ones(A.shape[0]), rtol=1e-12, max_iter=3, method="none", device="cuda")
    it, prec, solve = get_cg_iter_time(A, np.ones(A.shape[0]), rtol=1e-8, method="none", device="cuda")
    assert it == O.pcg(A, A @ np.ones(A.shape[0]), None, rtol=1e-8, dot="exact")[0]


def test_reused_solver_reinstalls_a_changed_factor(gpu_ctx):
    # the reference calls the same solver with ext_spai=(L, eps) per solve (validate.py:116-117):
    # a reused solver must pick up a different L object and an in-place change of the same one
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    _, A, mask = _cases.spd_cases()[1]
    b = A @ (np.ones(A.shape[0]) if mask is None else mask.ravel().astype(np.float64))
    L1 = _cases.spai_like(A, seed=1)
    d = np.linspace(0.5, 2.0, A.shape[0])
    L2 = L1.copy()
    L2.data = L1.data * d[L1.indices]  # L1 diag(d), same stored order
    eps = 3e-3
    want = [O.pcg(A, b, O.spai_operator(L, eps), rtol=1e-8, dot="exact")[1] for L in (L1, L2)]
    assert np.linalg.norm(want[0] - want[1]) > 1e-10 * np.linalg.norm(want[0])  # distinguishable
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")

    def run(L, k):
        x = np.zeros_like(b)
        s(b.copy(), x, 1e-8, 0, ext_spai=(L, eps))
        assert np.linalg.norm(x - want[k]) <= 1e-12 * np.linalg.norm(want[k])

    run(L1, 0)
    run(L2, 1)  # another object
    Ld = DeviceMatrix.from_scipy(L1)
    run(Ld, 0)
    Ld.scale_columns_(torch.from_numpy(d))  # the same object, new values
    run(Ld, 1)


@pytest.mark.parametrize("small_n", ["0", "4096"])
@pytest.mark.parametrize("max_iter", [1, 4, 37, 64])
def test_pcg_max_iter_inside_queued_chunks(gpu_ctx, max_iter, small_n, monkeypatch):
    # the host keeps one chunk of up to 32 iterations queued ahead of its poll: a max_iter that
    # falls inside a queued chunk must still stop the iterate and the history at max_iter
    # (small_n "4096": the same n = 2048 system in the one-workgroup solve, 5-row template)
    monkeypatch.setenv("LSPCG_SMALL_N", small_n)
    _, A, mask = _cases.spd_cases()[0]
    gt = np.ones(A.shape[0]) if mask is None else mask.ravel().astype(np.float64)
    b = A @ gt
    L = _cases.spai_like(A, seed=0)
    it_full = O.pcg(A, b, O.spai_operator(L, 3e-3), rtol=1e-14, dot="exact")[0]
    assert it_full > max_iter
    it_o, x_o, h_o = O.pcg(A, b, O.spai_operator(L, 3e-3), rtol=1e-14, max_iter=max_iter, dot="exact")
    it, x, h = _solve(A, b, "ext_spai", L, 3e-3, rtol=1e-14, max_iter=max_iter)
    assert it == it_o == max_iter
    assert len(h) == it + 1
    np.testing.assert_allclose(h, h_o, rtol=1e-12, atol=0)
    assert np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


def test_time_kernels_reports_five_launches(gpu_ctx, monkeypatch):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    _, A, _ = _cases.spd_cases()[2]
    b = torch.from_numpy(A @ np.ones(A.shape[0])).cuda()
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
    s.set_spai(_cases.spai_like(A), 3e-3)
    k = s.time_kernels(b, 5)
    assert list(k) == list(s.KERNELS) and all(v > 0 for v in k.values())
    # the solver still solves correctly afterwards (the timing pass leaves no state behind)
    x = torch.zeros_like(b)
    it, conv, _ = s.solve(b, x, rtol=1e-8)
    L = _cases.spai_like(A)
    assert conv and it == O.pcg(A, A @ np.ones(A.shape[0]), O.spai_operator(L, 3e-3), rtol=1e-8, dot="exact")[0]
    monkeypatch.setenv("LSPCG_NO_SELL", "1")  # staged CSR views: the same split schedule (round 5)
    s2 = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
    s2.set_spai(L, 3e-3)
    k2 = s2.time_kernels(b, 5)
    assert list(k2) == list(s.KERNELS) and all(v > 0 for v in k2.values())
    monkeypatch.setenv("LSPCG_SPLIT_REDUCE", "0")  # last-arriver reductions: not instrumented
    s3 = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
    s3.set_spai(L, 3e-3)
    with pytest.raises(RuntimeError):
        s3.time_kernels(b, 5)


def test_solve_many_matches_one_by_one(gpu_ctx):
    """linalg.solve_many: concurrent independent solves (one stream per solver, GIL released in
    the native call) return each solve's own count and iterate, bit for bit."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient, solve_many

    jobs, ref = [], []
    for name, A, _ in _cases.spd_cases()[:4]:
        b = torch.from_numpy(A @ np.ones(A.shape[0])).cuda()
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
        s.set_spai(_cases.spai_like(A), 3e-3)
        x = torch.zeros_like(b)
        it, conv, _ = s.solve(b, x, rtol=1e-8)
        ref.append((it, conv, x.clone()))
        jobs.append((s, b, torch.zeros_like(b)))
    out = solve_many(jobs, rtol=1e-8, concurrency=4)
    for (it, conv, x), (it2, conv2, _), (_, _, x2) in zip(ref, out, jobs):
        assert (it, conv) == (it2, conv2)
        assert torch.equal(x, x2)


def test_solve_many_fresh_solvers_concurrent_capture(gpu_ctx):
    """Round-4 regression (DESIGN.md §6 "Concurrent solves"): 8 FRESH solvers above the
    one-workgroup bound (multi-kernel schedule, hipGraphs captured on first use) solved 4 at a
    time, so graph capture, instantiation and launches of different solvers overlap on four host
    threads, twice (the second pass captures the chunk lengths the first did not use).  Every
    result equals a sequential solve on its own fresh solver, bit for bit."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient, solve_many

    systems = []
    for k in range(8):
        if k % 2:
            A, _m, _ = P.poisson2d_grid(56 + 8 * k, 48 + 4 * k)
        else:
            A = P.kuhn_laplacian(15 + 2 * k)
        A = sp.csr_matrix(A)
        assert A.shape[0] > 2560  # not the one-workgroup solve: graphs are captured
        systems.append(A)

    def fresh(A, precond):
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=precond)
        if precond == "ext_spai":
            s.set_spai(_cases.spai_like(A), 3e-3)
        b = torch.from_numpy(A @ np.ones(A.shape[0])).cuda()
        return s, b, torch.zeros_like(b)

    precs = ["ext_spai", "diagonal", "ext_spai", "none"] * 2
    ref = []
    for A, pc in zip(systems, precs):
        s, b, x = fresh(A, pc)
        it, conv, _ = s.solve(b, x, rtol=1e-8)
        ref.append((it, conv, x.clone()))
    jobs = [fresh(A, pc) for A, pc in zip(systems, precs)]
    for _pass in range(2):
        for _, _, x in jobs:
            x.zero_()
        out = solve_many(jobs, rtol=1e-8, concurrency=4)
        torch.cuda.synchronize()
        for (it, conv, x), (it2, conv2, _), (_, _, x2) in zip(ref, out, jobs):
            assert (it, conv) == (it2, conv2)
            assert torch.equal(x, x2)


@pytest.mark.parametrize("case", ["sdia", "csr", "bsr3", "scaled", "fp32", "reordered"])
def test_new_spai_on_the_same_solver_equals_a_fresh_solver(gpu_ctx, monkeypatch, case):
    """set_spai with a new L on a solver that has solved before refills its L / Lᵀ views in place and
    keeps its captured iteration graphs when every address and ε are unchanged (GraphKey); the
    solve must equal a fresh solver's on the new L bit for bit -- also after an ε change (graphs
    dropped) and back, and through an L of another pattern (its views rebuilt: the key holds the
    patterns' arrays, not just their host addresses)."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    dtype = np.float32 if case == "fp32" else np.float64
    bs = 3 if case == "bsr3" else 1
    pre = "ext_spai_scaled" if case == "scaled" else "ext_spai"
    if case == "csr":
        monkeypatch.setenv("LSPCG_NO_SELL", "1")
    if case == "reordered":  # P L Pᵀ, Lᵀ and P Lᵀ Pᵀ overwritten in place too
        monkeypatch.setenv("LSPCG_REORDER", "1")
    if bs == 3:
        A0, _, _ = P.elasticity_box(16, 8, 8)
        A = sp.csr_matrix(A0)
    else:
        A = sp.csr_matrix(P.kuhn_laplacian(30, 1e-2))
    A.sort_indices()
    A.data = A.data.astype(np.float32).astype(np.float64)
    Ls = []
    for seed in (1, 2):
        L = _cases.spai_like(A, seed=seed)
        L.data = L.data.astype(np.float32).astype(np.float64)
        Ls.append(L)
    Lc = Ls[1].tocoo()  # block-lower-triangular part: a pattern other than A's
    keep = (Lc.row // bs) >= (Lc.col // bs)
    Ls.append(sp.csr_matrix((Lc.data[keep], (Lc.row[keep], Lc.col[keep])), shape=Lc.shape))
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    b = torch.from_numpy(A @ np.ones(A.shape[0])).to(tdt).cuda()
    rtol = 1e-8 if dtype == np.float64 else 1e-5

    def run(s):
        x = torch.zeros_like(b)
        it, conv, _, h = s.solve(b, x, rtol=rtol, return_history=True)
        return it, x.cpu().numpy(), h

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=pre, dtype=dtype, block_size=bs)
    seq = [(Ls[0], 3e-3), (Ls[1], 3e-3), (Ls[1], 2e-3), (Ls[0], 3e-3), (Ls[2], 3e-3), (Ls[2], 3e-3),
           (Ls[0], 3e-3)]
    for L, eps in seq:
        s.set_spai(L, eps, block_size=bs)
        got = run(s)
        got2 = run(s)  # the graphs of this L (kept or re-captured) replayed again
        f = PreconditionedConjugateGradient(A, device="cuda", preconditioner=pre, dtype=dtype, block_size=bs)
        f.set_spai(L, eps, block_size=bs)
        want = run(f)
        del f
        for g in (got, got2):
            assert g[0] == want[0] and np.array_equal(g[1], want[1]) and np.array_equal(g[2], want[2]), (case, eps)
