"""GPU: the reverse-Cuthill-McKee analysis step of the solver (lspcg_reorder.hip).

A solver whose A is numbered far from banded runs its loop on P A Pᵀ (and P L Pᵀ, P Lᵀ Pᵀ) with
every row's entries in their original order, so each SpMV row sum keeps scipy's bits; b and x are
permuted on the device around the loop.  Checked here:
  * auto mode picks it for a randomly renumbered grid and leaves structured / banded ones alone;
  * the permuted solve equals the oracle's correctly-rounded-dot trajectory (count exact, history
    and x to 1e-12) and the unpermuted solver's result, for none / diagonal / ext_spai /
    ext_spai_scaled, fp64 and fp32;
  * parity mode (numpy's ddot order over the ORIGINAL numbering) switches a reordered solver back
    and then equals an unpermuted parity solver bit for bit.
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
    if kind == "kuhn27rand":
        A, m = P.renumber(*P.kuhn_dirichlet(27), "rand")
    elif kind == "poisson160rand":
        A0, m0, _ = P.poisson2d_grid(160, 160)
        A, m = P.renumber(sp.csr_matrix(A0), m0.ravel(), "rand")
    else:
        raise KeyError(kind)
    A = sp.csr_matrix(A)
    A.sort_indices()
    A.data = A.data.astype(np.float32).astype(np.float64)
    L = _cases.spai_like(A, seed=3)
    L.data = L.data.astype(np.float32).astype(np.float64)
    b = A @ np.asarray(m, dtype=np.float64).ravel()
    return A, L, b


def _solver(A, L, pre, dtype=np.float64, **kw):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=pre, dtype=dtype, **kw)
    if pre.startswith("ext_spai"):
        s.set_spai(L, 3e-3)
    return s


def _run(s, b, rtol=1e-8, dtype=np.float64):
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    bt = torch.as_tensor(b, dtype=tdt, device="cuda")
    x = torch.zeros_like(bt)
    it, conv, _t, h = s.solve(bt, x, rtol=rtol, return_history=True)
    return it, conv, x.cpu().numpy().astype(np.float64), h


def test_auto_mode_decisions(gpu_ctx, monkeypatch):
    monkeypatch.delenv("LSPCG_REORDER", raising=False)
    A, L, _ = _system("kuhn27rand")
    s = _solver(A, L, "none")
    info = s.reorder_info
    assert info["applied"] and info["mean_offset_after"] < 0.1 * info["mean_offset_before"], info
    K = sp.csr_matrix(P.kuhn_dirichlet(27)[0])  # structured: already banded
    assert not _solver(K, None, "none").reorder_info["applied"]
    R = sp.csr_matrix(P.renumber(*P.kuhn_dirichlet(27), "rcm")[0])  # RCM-banded irregular
    assert not _solver(R, None, "none").reorder_info["applied"]


@pytest.mark.parametrize("pre", ["none", "diagonal", "ext_spai", "ext_spai_scaled"])
@pytest.mark.parametrize("kind", ["kuhn27rand", "poisson160rand"])
def test_reordered_solve_equals_oracle_and_unpermuted(gpu_ctx, monkeypatch, kind, pre):
    A, L, b = _system(kind)
    monkeypatch.setenv("LSPCG_REORDER", "1")
    sr = _solver(A, L, pre)
    assert sr.reorder_info["applied"]
    monkeypatch.setenv("LSPCG_REORDER", "0")
    su = _solver(A, L, pre)
    assert not su.reorder_info["applied"]
    it_r, conv_r, x_r, h_r = _run(sr, b)
    it_u, conv_u, x_u, h_u = _run(su, b)
    ps = {"none": None, "diagonal": O.diagonal_operator(A), "ext_spai": O.spai_operator(L, 3e-3),
          "ext_spai_scaled": O.spai_scaled_operator(A, L, 3e-3)}[pre]
    it_o, x_o, h_o = O.pcg(A, b, ps, rtol=1e-8, dot="exact")
    rec = {"kind": kind, "pre": pre, "reordered": it_r, "unpermuted": it_u, "oracle": it_o}
    assert conv_r and it_r == it_o == it_u, rec
    assert np.allclose(h_r[: it_o + 1], np.asarray(h_o)[: it_o + 1], rtol=1e-12, atol=0), rec
    assert np.linalg.norm(x_r - x_o) <= 1e-12 * np.linalg.norm(x_o), rec
    assert np.linalg.norm(x_r - x_u) <= 1e-12 * np.linalg.norm(x_u), rec


def test_reordered_fp32(gpu_ctx, monkeypatch):
    A, L, b = _system("kuhn27rand")
    monkeypatch.setenv("LSPCG_REORDER", "1")
    sr = _solver(A, L, "ext_spai", dtype=np.float32)
    assert sr.reorder_info["applied"]
    monkeypatch.setenv("LSPCG_REORDER", "0")
    su = _solver(A, L, "ext_spai", dtype=np.float32)
    it_r, conv_r, x_r, _ = _run(sr, b, rtol=1e-5, dtype=np.float32)
    it_u, conv_u, x_u, _ = _run(su, b, rtol=1e-5, dtype=np.float32)
    assert conv_r and conv_u and abs(it_r - it_u) <= 1, (it_r, it_u)
    assert np.linalg.norm(x_r - x_u) <= 1e-4 * np.linalg.norm(x_u)


def test_parity_mode_switches_reordering_off(gpu_ctx, monkeypatch):
    """set_spai on a reordered solver, then set_dot_order('openblas'): A's views are rebuilt for the
    unpermuted A (a pattern at the same host address, padding differently), so L's and Lᵀ's value
    arrays are rebuilt too, not refilled in place (the refill checks the array's entry
    count); the solve equals a parity solver that never reordered, and the recorded scipy run."""
    A, L, b = _system("kuhn27rand")
    monkeypatch.setenv("LSPCG_REORDER", "1")
    s1 = _solver(A, L, "ext_spai")
    assert s1.reorder_info["applied"]
    v_perm = s1.views
    s1.set_dot_order("openblas", 1)
    assert not s1.reorder_info["applied"]
    monkeypatch.setenv("LSPCG_REORDER", "0")
    s2 = _solver(A, L, "ext_spai", dot_order="openblas", dot_threads=1)
    assert s1.views == s2.views, (v_perm, s1.views, s2.views)
    it1, c1, x1, h1 = _run(s1, b)
    it2, c2, x2, h2 = _run(s2, b)
    assert c1 and it1 == it2 and np.array_equal(h1, h2) and np.array_equal(x1, x2)
    it_b, x_b, h_b = O.pcg(A, b, O.spai_operator(L, 3e-3), rtol=1e-8, dot="blas1")
    assert it1 == it_b and np.array_equal(x1, x_b)


def test_reordered_solver_reuse_and_new_spai(gpu_ctx, monkeypatch):
    """A reordered solver solves twice (same bits) and takes a second L (set_spai again)."""
    A, L, b = _system("poisson160rand")
    monkeypatch.setenv("LSPCG_REORDER", "1")
    s = _solver(A, L, "ext_spai")
    r1 = _run(s, b)
    r2 = _run(s, b)
    assert r1[0] == r2[0] and np.array_equal(r1[2], r2[2])
    L2 = _cases.spai_like(A, seed=9)
    L2.data = L2.data.astype(np.float32).astype(np.float64)
    s.set_spai(L2, 3e-3)
    it, conv, x, _ = _run(s, b)
    it_o, x_o, _ = O.pcg(A, b, O.spai_operator(L2, 3e-3), rtol=1e-8, dot="exact")
    assert conv and it == it_o and np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


def test_reordered_bsr3_equals_oracle(gpu_ctx, monkeypatch):
    """BSR 3×3 (the elasticity layout): block rows renumbered at random, then the solver's RCM on
    the block graph (block rows permuted, every block row's blocks in their original order)."""
    A0, m0, _ = P.elasticity_box(20, 12, 12)  # n = 8,640: above the one-workgroup bound
    nb = A0.shape[0] // 3
    pb = np.random.default_rng(2).permutation(nb)
    perm = (3 * pb[:, None] + np.arange(3)[None, :]).ravel()
    A = sp.csr_matrix(sp.csr_matrix(A0)[perm][:, perm])
    A.sort_indices()
    A.data = A.data.astype(np.float32).astype(np.float64)
    L = _cases.spai_like(A, seed=4)
    L.data = L.data.astype(np.float32).astype(np.float64)
    b = A @ np.asarray(m0, dtype=np.float64).ravel()[perm]
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("LSPCG_REORDER", mode)
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", block_size=3)
        s.set_spai(L, 3e-3, block_size=3)
        assert s.reorder_info["applied"] == (mode == "1")
        res[mode] = _run(s, b)
    it_o, x_o, h_o = O.pcg(A, b, O.spai_operator(L, 3e-3), rtol=1e-8, dot="exact")
    for mode, (it, conv, x, h) in res.items():
        assert conv and it == it_o, (mode, it, it_o)
        assert np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o), mode


@pytest.mark.parametrize("kind", ["kuhn27rand", "poisson160rand"])
def test_device_rcm_quality_matches_scipy(gpu_ctx, monkeypatch, kind):
    """The device's level-synchronous Cuthill-McKee reaches scipy's reverse_cuthill_mckee bandwidth
    (mean |col - row| within 15 %; the orders differ only in start-node and tie choices)."""
    from scipy.sparse.csgraph import reverse_cuthill_mckee

    A, L, _ = _system(kind)
    monkeypatch.setenv("LSPCG_REORDER", "1")
    info = _solver(A, L, "none").reorder_info
    p = reverse_cuthill_mckee(A, symmetric_mode=True)
    ip = np.empty_like(p)
    ip[p] = np.arange(p.size)
    C = A.tocoo()
    ref = np.abs(ip[C.col].astype(np.int64) - ip[C.row]).mean()
    assert info["applied"] and info["mean_offset_after"] <= 1.15 * ref, (info, ref)


def test_many_components_left_in_order(gpu_ctx, monkeypatch):
    """A graph of more than 256 non-trivial components is not reordered (one host round trip per BFS
    level would dominate); the solve still equals the oracle."""
    rng = np.random.default_rng(5)
    blocks = [sp.csr_matrix(np.array([[4.0, -1.0], [-1.0, 3.0 + k % 3]])) for k in range(400)]
    A0 = sp.block_diag(blocks, format="csr")
    pm = rng.permutation(A0.shape[0])
    A = sp.csr_matrix(A0[pm][:, pm])
    A.sort_indices()
    b = rng.standard_normal(A.shape[0])
    monkeypatch.setenv("LSPCG_REORDER", "1")
    s = _solver(A, None, "none")
    assert not s.reorder_info["applied"]
    it, conv, x, _ = _run(s, b)
    it_o, x_o, _ = O.pcg(A, b, None, rtol=1e-8, dot="exact")
    assert conv and it == it_o and np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


def _cuthill_mckee_reference(A):
    """Sequential restatement of the device analysis (lspcg_reorder.hip rcm_device): rows with no
    neighbour but themselves first (empty rows, then diagonal-only rows, by index); each remaining
    component from its (row length, index)-smallest row, moved to the smallest row of the last level
    of a BFS from there; Cuthill-McKee appending each row's unplaced neighbours by (row length,
    index); reversed."""
    A = sp.csr_matrix(A)
    n, rp, ci = A.shape[0], A.indptr, A.indices
    deg = np.diff(rp)
    pos = np.full(n, -1)
    order = []

    def place(v):
        pos[v] = len(order)
        order.append(v)

    only_self = np.array([np.all(ci[rp[i]:rp[i + 1]] == i) for i in range(n)])
    for want_empty in (True, False):
        for i in range(n):
            if only_self[i] and (deg[i] == 0) == want_empty:
                place(i)
    key = lambda v: (deg[v], v)
    while len(order) < n:
        start = min(np.flatnonzero(pos == -1), key=key)
        seen, level = {start}, [start]
        while True:
            nxt = []
            for u in level:
                for v in ci[rp[u]:rp[u + 1]]:
                    if pos[v] == -1 and v not in seen:
                        seen.add(v)
                        nxt.append(v)
            if not nxt:
                break
            level = nxt
        start = min(level, key=key)
        place(start)
        head = len(order) - 1
        while head < len(order):
            u = order[head]
            head += 1
            for v in sorted({int(v) for v in ci[rp[u]:rp[u + 1]] if pos[v] == -1}, key=key):
                place(v)
    return np.asarray(order[::-1], dtype=np.int32)


def _rcm_cases():
    rng = np.random.default_rng(11)
    A1, _ = P.renumber(*P.kuhn_dirichlet(17), "rand")
    A2 = sp.csr_matrix(P.renumber(sp.csr_matrix(P.poisson2d_grid(60, 50)[0]), np.ones(3000), "rand")[0])
    # three components, empty rows and diagonal-only rows, random extra edges
    R = sp.random(600, 600, density=0.004, random_state=3, format="csr")
    R = (R + R.T + sp.diags(np.where(np.arange(600) % 7 == 0, 1.0, 0.0))).tocsr()
    C = sp.csr_matrix(P.kuhn_dirichlet(6)[0])  # 216 rows
    # random graph (several components) | Kuhn grid | 20 empty rows | 20 diagonal-only rows | 14 empty
    D = sp.diags(np.r_[np.zeros(20), 2.0 * np.ones(20), np.zeros(14)])
    B = sp.block_diag([R, C, D], format="csr")
    B.eliminate_zeros()
    B.sort_indices()
    pb = rng.permutation(B.shape[0])
    B = sp.csr_matrix(B[pb][:, pb])
    B.sort_indices()
    # unsymmetric pattern with rows of 1..60 entries (the 16-entry register path and the long-row path)
    rows, cols = [], []
    for i in range(1500):
        k = int(rng.integers(1, 60)) if i % 9 == 0 else int(rng.integers(1, 8))
        rows += [i] * k
        cols += list(rng.choice(1500, size=k, replace=False))
    U = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(1500, 1500))
    U.sum_duplicates()
    return {"kuhn17rand": sp.csr_matrix(A1), "poisson60x50rand": A2, "components": B, "unsym-long-rows": U}


@pytest.mark.parametrize("case", ["kuhn17rand", "poisson60x50rand", "components", "unsym-long-rows"])
def test_device_rcm_equals_sequential_cuthill_mckee(gpu_ctx, case):
    """lspcg_mat_rcm's level-synchronous order (no sort, sizes kept on the device) equals the
    sequential Cuthill-McKee restatement above, index for index."""
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A = _rcm_cases()[case]
    A.sort_indices()
    Ad = DeviceMatrix.from_scipy(A, dtype=np.float64)
    perm, before, after = Ad.rcm()
    assert perm is not None
    ref = _cuthill_mckee_reference(A)
    got = perm.cpu().numpy()
    assert np.array_equal(np.sort(got), np.arange(A.shape[0]))
    assert np.array_equal(got, ref), (case, np.flatnonzero(got != ref)[:10])
    ip = np.empty_like(ref)
    ip[ref] = np.arange(ref.size)
    C = A.tocoo()
    assert after == pytest.approx(np.abs(ip[C.col].astype(np.int64) - ip[C.row]).mean(), rel=1e-12)


def test_device_rcm_block_graph(gpu_ctx):
    """BSR 3x3: the analysis runs on the block graph (one entry per block row)."""
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A0, _, _ = P.elasticity_box(12, 6, 5)
    nb = A0.shape[0] // 3
    pb = np.random.default_rng(2).permutation(nb)
    perm3 = (3 * pb[:, None] + np.arange(3)[None, :]).ravel()
    A = sp.csr_matrix(sp.csr_matrix(A0)[perm3][:, perm3])
    A.sort_indices()
    B = sp.bsr_matrix(A, blocksize=(3, 3))
    B.sort_indices()
    Ad = DeviceMatrix.from_scipy(B, dtype=np.float64, block_size=3)
    perm, _, _ = Ad.rcm()
    G = sp.csr_matrix((np.ones(B.indices.size), B.indices, B.indptr), shape=(nb, nb))
    assert np.array_equal(perm.cpu().numpy(), _cuthill_mckee_reference(G))


def test_device_rcm_leaves_unsorted_or_repeated_rows_in_order(gpu_ctx):
    """A row whose columns are not strictly increasing (unsorted or repeated: a CSR uploaded with
    keep_order) would count a child twice; the analysis leaves such a matrix in its order."""
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A = sp.csr_matrix(_rcm_cases()["kuhn17rand"])
    A.sort_indices()
    for how in ("unsorted", "repeated"):
        B = A.copy()
        r = 100
        a, b = B.indptr[r], B.indptr[r + 1]
        if how == "unsorted":
            B.indices[a:b] = B.indices[a:b][::-1].copy()
        else:
            B.indices[a + 1] = B.indices[a]
        B.has_sorted_indices = False
        Bd = DeviceMatrix.from_scipy(B, dtype=np.float64, keep_order=True)
        perm, before, after = Bd.rcm()
        assert perm is None and after == before, how


def _hubbed(A, hubs=6, far=80, seed=5):
    """A plus a few rows with `far` long-range symmetric couplings each (diagonally compensated, so
    still SPD): their slices hold more than 64 distinct offsets and stay uncoded in SELL-64C."""
    rng = np.random.default_rng(seed)
    n = A.shape[0]
    rows = np.repeat(np.linspace(0, n - 1, hubs).astype(np.int64), far)
    cols = rng.integers(0, n, rows.size)
    keep = rows != cols
    S = sp.csr_matrix((np.full(keep.sum(), -2.0 ** -10), (rows[keep], cols[keep])), shape=A.shape)
    S = S + S.T
    S = S + sp.diags(np.asarray(abs(S).sum(axis=1)).ravel())
    B = sp.csr_matrix(A + S)
    B.sum_duplicates()
    B.sort_indices()
    return B


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("pre", ["none", "ext_spai"])
@pytest.mark.parametrize("kind", ["rcm", "rcm_hubs", "rcm_unsorted"])
def test_sellc_views_equal_sell16_and_csr(gpu_ctx, monkeypatch, kind, pre, dtype):
    """SELL-64C (one-byte codes into per-slice offset dictionaries, 16-bit offsets for slices with
    more than 64) sums every row in the CSR order: the solve equals the 16-bit SELL-64 views' and the
    staged CSR kernel's bit for bit, and the oracle's.  rcm_unsorted: every row of A stored in a
    shuffled entry order (as a reordered solver's permuted rows are), summed in that order by all
    three paths and by scipy."""
    A, m = P.renumber(*P.kuhn_dirichlet(27), "rcm")
    A = sp.csr_matrix(A)
    A.sort_indices()
    if kind == "rcm_hubs":
        A = _hubbed(A)
    A.data = A.data.astype(np.float32).astype(np.float64)
    L = _cases.spai_like(A, seed=4)
    L.data = L.data.astype(np.float32).astype(np.float64)
    if kind == "rcm_unsorted":
        rng = np.random.default_rng(9)
        idx, dat = A.indices.copy(), A.data.copy()
        for i in range(A.shape[0]):
            p = A.indptr[i] + rng.permutation(A.indptr[i + 1] - A.indptr[i])
            idx[A.indptr[i]:A.indptr[i + 1]], dat[A.indptr[i]:A.indptr[i + 1]] = A.indices[p], A.data[p]
        A = sp.csr_matrix((dat, idx, A.indptr.copy()), shape=A.shape)
        assert not A.has_sorted_indices
    b = A @ np.asarray(m, dtype=np.float64).ravel()
    monkeypatch.setenv("LSPCG_REORDER", "0")
    rtol = 1e-8 if dtype == np.float64 else 1e-5
    runs = {}
    variants = (("sellc", {"LSPCG_SELLC": "1", "LSPCG_SELLC_MIN_N": "0"}),  # (the default takes >= 2^19 rows)
                ("sell16", {"LSPCG_SELLC": "0"}), ("csr", {"LSPCG_NO_SELL": "1"}))
    for name, env in variants:
        for k in ("LSPCG_SELLC", "LSPCG_SELLC_MIN_N", "LSPCG_NO_SELL"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        Ad = A
        if kind == "rcm_unsorted":  # upload the rows in their stored order (from_scipy sorts by default)
            from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

            Ad = DeviceMatrix.from_scipy(A, dtype=dtype, keep_order=True)
        s = _solver(Ad, L, pre, dtype=dtype)
        views = s.views
        want = "csr" if name == "csr" else name
        assert views["A"]["columns"] == want, (name, views)
        if pre == "ext_spai":
            assert views["L"]["columns"] == want and views["LT"]["columns"] == want, (name, views)
        runs[name] = _run(s, b, rtol=rtol, dtype=dtype)
        del s
    it, conv, x, h = runs["sellc"]
    assert conv
    for other in ("sell16", "csr"):
        it2, conv2, x2, h2 = runs[other]
        assert it == it2 and np.array_equal(x, x2) and np.array_equal(h, h2), (kind, pre, other)
    if dtype == np.float64:
        it_o, x_o, _ = O.pcg(A, b, O.spai_operator(L, 3e-3) if pre == "ext_spai" else None, rtol=1e-8, dot="exact")
        assert it == it_o and np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kind", ["kuhn27rand", "poisson160rand", "elast_rand"])
def test_prepare_spmv_reorders_far_from_banded(gpu_ctx, monkeypatch, kind, dtype):
    """The standalone SpMV's analysis step (lspcg_mat_prepare_spmv) applies the solver's rule: a
    numbering far from banded is analysed on P A Pᵀ (device RCM) and lspcg_spmv gathers x into that
    numbering and scatters y back -- scipy's bits (every row's entries keep their order).  BSR 3x3:
    the block graph's permutation, 3 scalars per block row.  Banded numberings are left alone."""
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    monkeypatch.delenv("LSPCG_REORDER", raising=False)
    bs = 1
    if kind == "elast_rand":  # 19,440 block rows, block rows randomly renumbered
        A0, _, _ = P.elasticity_box(60, 18, 18)
        nb = A0.shape[0] // 3
        pb = np.random.default_rng(1).permutation(nb)
        p = (3 * pb[:, None] + np.arange(3)[None, :]).ravel()
        B = sp.bsr_matrix(sp.csr_matrix(sp.csr_matrix(A0)[p][:, p]), blocksize=(3, 3))
        B.sort_indices()
        bs = 3
    else:
        A = _system(kind)[0]
        A.sort_indices()
        if dtype == np.float32:
            A.data = A.data.astype(np.float32).astype(np.float64)
    D = (DeviceMatrix.from_scipy(B, dtype=dtype, block_size=3) if bs == 3
         else DeviceMatrix.from_scipy(A, dtype=dtype))
    kind_v = D.prepare_spmv()
    info = D.spmv_reorder_info
    assert info["applied"] and info["mean_offset_after"] < 0.1 * info["mean_offset_before"], info
    assert kind_v != 0
    n = D.n
    x = np.random.default_rng(2).normal(size=n).astype(dtype)
    y = D.matvec(torch.as_tensor(x, device="cuda")).cpu().numpy()
    if bs == 3:  # scipy's bsr_matvec order: blocks by column, c = 0, 1, 2 inside a block
        ref = sp.bsr_matrix((B.data.astype(dtype), B.indices, B.indptr), shape=B.shape) @ x
    else:
        ref = (sp.csr_matrix((A.data.astype(dtype), A.indices, A.indptr), shape=A.shape) if dtype == np.float32
               else A) @ x
    assert np.array_equal(y, ref), (kind, dtype)
    ms = D.spmv_timed(torch.as_tensor(x, device="cuda"), torch.empty(n, dtype=torch.float64 if
                      dtype == np.float64 else torch.float32, device="cuda"), 3)
    assert ms > 0
    K = DeviceMatrix.from_scipy(sp.csr_matrix(P.kuhn_dirichlet(27)[0]))  # banded: analysed as given
    assert K.prepare_spmv() == 1 and not K.spmv_reorder_info["applied"]
