"""GPU: unstructured Delaunay tet meshes (problems.delaunay_heat; the shape of the reference's tetgen
meshes, datagen/heat_tetmesh.py) and the jagged SELL-64J layout their irregular rows take
(lspcg_sell.hpp kSellJag).  Checked here:
  * the generator's A on the box equals the container's (sha256 in tests/golden/delaunay_sha.json):
    qhull, numpy and scipy give the same mesh and the same matrix bits on both hosts;
  * the standalone SpMV on SELL-64J equals scipy's csr_matvec bit for bit (fp64 / fp32, sorted and
    stored-order rows, empty rows), and the solver's views take SELL-64J;
  * the solve on SELL-64J views equals the staged-CSR views' (count, history and x to 1e-12: lanes
    hold permuted rows of their slice, so the compensated dots' association may differ in the last
    bit) and the oracle's correctly-rounded-dot trajectory, for none / diagonal / ext_spai, fp64 and
    fp32;
  * from 2^18 rows, SELL-64X (the tile's x blocks staged in LDS, column words = LDS positions): the
    same SpMV bits (fp64 / fp32 vectors, a tail block past n, a tile over the LDS limit keeping
    SELL-64J) and the same solve.
"""
import json

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from tests import _cases
from tests.conftest import GOLDEN
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _sha_fixture():
    return json.loads((GOLDEN / "delaunay_sha.json").read_text())


@pytest.fixture(scope="module")
def d20k():
    A, m, nodes = P.delaunay_heat(20000)
    return sp.csr_matrix(A), m, nodes


def test_generator_bits_equal_the_container(d20k):
    fx = _sha_fixture()
    A, m, _ = d20k
    assert P.matrix_sha256(A) == fx["delaunay20k"]["A_sha256"]
    assert int((m == 0).sum()) == fx["delaunay20k"]["dirichlet"]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("case", ["delaunay", "unsorted", "ragged"])
def test_sell16j_spmv_bitexact(gpu_ctx, d20k, case, dtype):
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A = d20k[0].copy()
    keep = False
    if case == "unsorted":  # rows in a shuffled stored order, summed in that order
        rng = np.random.default_rng(2)
        idx, dat = A.indices.copy(), A.data.copy()
        for i in range(0, A.shape[0], 3):
            p = A.indptr[i] + rng.permutation(A.indptr[i + 1] - A.indptr[i])
            idx[A.indptr[i]:A.indptr[i + 1]], dat[A.indptr[i]:A.indptr[i + 1]] = A.indices[p], A.data[p]
        A = sp.csr_matrix((dat, idx, A.indptr.copy()), shape=A.shape)
        keep = True
    elif case == "ragged":  # empty rows and lengths 1..60 in one slice (no row beyond 64 entries)
        rng = np.random.default_rng(3)
        n = 5000
        lens = rng.integers(0, 61, n)
        lens[::17] = 0
        rows = np.repeat(np.arange(n), lens)
        cols = np.clip(rows + rng.integers(-3000, 3000, rows.size), 0, n - 1)
        A = sp.csr_matrix((rng.normal(size=rows.size), (rows, cols)), shape=(n, n))
        A.sum_duplicates()
        A.sort_indices()
    if dtype == np.float32:
        A.data = A.data.astype(np.float32).astype(np.float64)
    D = DeviceMatrix.from_scipy(A, dtype=dtype, keep_order=keep)
    kind = D.prepare_spmv()
    assert kind == 17, kind  # (SELL-64X from 2^18 rows: test_sell16x_*)
    x = np.random.default_rng(1).normal(size=A.shape[0]).astype(dtype)
    y = D.matvec(torch.as_tensor(x, device="cuda")).cpu().numpy()
    # (scipy's astype sorts a row's entries: build the fp32 copy from the stored arrays instead)
    As = sp.csr_matrix((A.data.astype(dtype), A.indices, A.indptr), shape=A.shape) if dtype == np.float32 else A
    ref = As @ x
    assert np.array_equal(y, ref)  # (stored-order rows: scipy sums in that order, as the device does)


def _solver(A, L, pre, dtype=np.float64):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=pre, dtype=dtype)
    if pre == "ext_spai":
        s.set_spai(L, 3e-3)
    return s


def _run(s, b, rtol, dtype):
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    bt = torch.as_tensor(b, dtype=tdt, device="cuda")
    x = torch.zeros_like(bt)
    it, conv, _t, h = s.solve(bt, x, rtol=rtol, return_history=True, max_iter=20000)
    return it, conv, x.cpu().numpy().astype(np.float64), np.asarray(h)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("pre", ["none", "diagonal", "ext_spai"])
def test_sell16j_solve_equals_csr_and_oracle(gpu_ctx, monkeypatch, d20k, pre, dtype):
    A, m, _ = d20k
    A = A.copy()
    A.data = A.data.astype(np.float32).astype(np.float64)
    L = _cases.spai_like(A, seed=4)
    L.data = L.data.astype(np.float32).astype(np.float64)
    b = A @ np.asarray(m, dtype=np.float64).ravel()
    rtol = 1e-8 if dtype == np.float64 else 1e-5
    monkeypatch.setenv("LSPCG_REORDER", "0")
    runs = {}
    for name in ("sell16j", "csr"):
        monkeypatch.delenv("LSPCG_NO_SELL", raising=False)
        if name == "csr":
            monkeypatch.setenv("LSPCG_NO_SELL", "1")
        s = _solver(A, L, pre, dtype)
        v = s.views
        assert v["A"]["columns"] == name, v
        if pre == "ext_spai":
            assert v["L"]["columns"] == name and v["LT"]["columns"] == name, v
        runs[name] = _run(s, b, rtol, dtype)
        del s
    it, conv, x, h = runs["sell16j"]
    it2, conv2, x2, h2 = runs["csr"]
    assert conv and conv2 and it == it2
    tol = 1e-12 if dtype == np.float64 else 1e-5
    assert np.linalg.norm(x - x2) <= tol * np.linalg.norm(x2)
    assert np.allclose(h, h2, rtol=tol * 1e2, atol=0)
    if dtype == np.float64:
        M = {"none": None, "diagonal": O.diagonal_operator(A), "ext_spai": O.spai_operator(L, 3e-3)}[pre]
        it_o, x_o, _ = O.pcg(A, b, M, rtol=1e-8, dot="exact", max_iter=20000)
        assert it == it_o and np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


def _banded_spd(n, spread, seed=0, long_tile=False):
    """Symmetric, strictly diagonally dominant (SPD) banded matrix with irregular rows (3..30 entries,
    columns within +-spread of the row): SELL-64 pads > 1.15, every 256-row tile reads
    (256 + 2 spread) / 16 x blocks at most.  long_tile: one tile's rows reach 8 spread away (over the
    256-block LDS limit for that tile only)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 15, n)
    rows = np.repeat(np.arange(n), lens)
    off = rng.integers(-spread, spread + 1, rows.size)
    if long_tile:
        sel = (rows >= 512) & (rows < 768)
        off[sel] = rng.integers(-8 * spread, 8 * spread + 1, int(sel.sum()))
    cols = rows + off
    keep = (cols >= 0) & (cols < n)
    B = sp.csr_matrix((rng.uniform(-1, 1, int(keep.sum())), (rows[keep], cols[keep])), shape=(n, n))
    B = B + B.T
    B = sp.csr_matrix(B + sp.diags(np.asarray(abs(B).sum(axis=1)).ravel() + 1.0))
    B.sum_duplicates()
    B.sort_indices()
    B.data = B.data.astype(np.float32).astype(np.float64)
    return B


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("case", ["staged", "over_limit"])
def test_sell16x_spmv_bitexact(gpu_ctx, case, dtype):
    import bench
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    n = 300001  # > 2^18 rows; the last x block runs past n
    A = _banded_spd(n, 1500, long_tile=case == "over_limit")
    xb = bench.xs_blocks(A.indptr, A.indices)
    assert (xb.max() <= bench.XS_MAX) == (case == "staged"), xb.max()
    D = DeviceMatrix.from_scipy(A, dtype=dtype)
    kind = D.prepare_spmv()
    assert kind == (18 if case == "staged" else 17) == bench.sell_kind(A.indptr, A.indices), kind
    x = np.random.default_rng(1).normal(size=n).astype(dtype)
    x[-3:] = dtype(7.5)  # the tail block's entries are read
    y = D.matvec(torch.as_tensor(x, device="cuda")).cpu().numpy()
    As = sp.csr_matrix((A.data.astype(dtype), A.indices, A.indptr), shape=A.shape)
    assert np.array_equal(y, As @ x)


@pytest.mark.parametrize("pre", ["none", "ext_spai"])
def test_sell16x_solve_equals_csr_and_oracle(gpu_ctx, monkeypatch, pre):
    A = _banded_spd(300001, 1500, seed=2)
    L = _cases.spai_like(A, seed=5)
    L.data = L.data.astype(np.float32).astype(np.float64)
    b = A @ np.random.default_rng(3).uniform(0, 1, A.shape[0])
    monkeypatch.setenv("LSPCG_REORDER", "0")
    runs = {}
    for name in ("sell16x", "csr"):
        monkeypatch.delenv("LSPCG_NO_SELL", raising=False)
        if name == "csr":
            monkeypatch.setenv("LSPCG_NO_SELL", "1")
        s = _solver(A, L, pre)
        v = s.views
        assert v["A"]["columns"] == name, v
        if pre == "ext_spai":
            assert v["L"]["columns"] == name and v["LT"]["columns"] == name, v
        runs[name] = _run(s, b, 1e-10, np.float64)
        del s
    (it, conv, x, h), (it2, conv2, x2, h2) = runs["sell16x"], runs["csr"]
    assert conv and conv2 and it == it2
    assert np.linalg.norm(x - x2) <= 1e-12 * np.linalg.norm(x2) and np.allclose(h, h2, rtol=1e-10, atol=0)
    it_o, x_o, _ = O.pcg(A, b, O.spai_operator(L, 3e-3) if pre == "ext_spai" else None, rtol=1e-10, dot="exact")
    assert it == it_o and np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)


# ---- the reference's own runs on the Delaunay systems (make_golden.py batch / headline) -----------
def _shaB(*arrs):
    import hashlib

    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


_BATCH = {}


def _delaunay_batch():
    """The C5 Delaunay variant as bench.c5_rows builds it (one seeded workspace for the batch), with
    every system's boo / A / L checked against the sha256 the reference's run recorded."""
    if _BATCH:
        return _BATCH["v"]
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    z = np.load(GOLDEN / "traj_delaunay_batch8.npz")
    samples = synthetic_dataset("delaunay_batch8")
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=1, seed=0)
    out = []
    for k, smp in enumerate(samples):
        d = smp.to("cuda")
        boo = ws.forward(d.x, d.edge_index, d.edge_attr)
        L = ws._assemble(d, boo, None)
        A = ws.system_matrix(d)
        Ah, Lh = sp.csr_matrix(A.to_scipy()), sp.csr_matrix(L.to_scipy())
        assert _shaB(boo.cpu().numpy()) == str(z[f"{k}__boo_sha256"]), k
        assert _shaB(Ah.indptr, Ah.indices, Ah.data) == str(z[f"{k}__A_sha256"]), k
        assert _shaB(Lh.indptr, Lh.indices, Lh.data) == str(z[f"{k}__L_sha256"]), k
        b = A.matvec(d.mask.reshape(-1).to(torch.float64))
        out.append((A, L, b))
    _BATCH["v"] = (z, ws.epsilon, out)
    return _BATCH["v"]


def _solve_full(A, L, b, eps, rtol, **kw):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", **kw)
    s.set_spai(L, eps)
    x = torch.zeros_like(b)
    it, conv, _t, h = s.solve(b, x, rtol=rtol, return_history=True)
    return it, conv, x, np.asarray(h)


@pytest.mark.parametrize("threads", [1, 8])
def test_delaunay_batch_parity_mode_equals_reference_runs(gpu_ctx, threads):
    """Parity mode (numpy's ddot order at T OpenBLAS threads) on every system of the C5 Delaunay
    variant: count, every ‖r_k‖ and sha256(x) equal to the reference's recorded scipy run."""
    z, eps, systems = _delaunay_batch()
    for k, (A, L, b) in enumerate(systems):
        it, conv, x, h = _solve_full(A, L, b, eps, float(z["rtol"]), dot_order="openblas", dot_threads=threads)
        want = int(z[f"{k}__ref_counts"][[1, 2, 4, 8].index(threads)])
        assert conv and it == want, (k, it, want)
        assert np.array_equal(h[:want], z[f"{k}__t{threads}__hist"]), k
        assert _shaB(x.cpu().numpy()) == str(z[f"{k}__t{threads}__x_sha256"]), k


def test_delaunay_batch_default_mode_equals_correctly_rounded_oracle(gpu_ctx):
    """Default (compensated) order: every system's count equals the oracle's correctly-rounded-dot
    count recorded beside the reference's runs (on these unstructured 1-1.6 k-iteration solves the
    reference's OpenBLAS order itself spreads over up to 10 iterations across thread counts and lies up
    to 9 above the correctly rounded count: the fixture's ref_counts), the true residual is below
    rtol, and the lockstep batch (BatchedConjugateGradient) gives every system the same count."""
    from learningsparsepreconditioner4gpu_amd.linalg import BatchedConjugateGradient

    z, eps, systems = _delaunay_batch()
    rtol = float(z["rtol"])
    its = []
    for k, (A, L, b) in enumerate(systems):
        it, conv, x, _ = _solve_full(A, L, b, eps, rtol)
        assert conv and it == int(z[f"{k}__oracle_exact_count"]), (k, it, int(z[f"{k}__oracle_exact_count"]),
                                                                      z[f"{k}__ref_counts"])
        tres = float(torch.linalg.vector_norm(b - A.matvec(x)) / torch.linalg.vector_norm(b))
        assert tres < rtol, (k, tres)
        its.append(it)
    B = BatchedConjugateGradient([s[0] for s in systems], [s[1] for s in systems], eps)
    xs = [torch.zeros_like(s[2]) for s in systems]
    res, _ = B.solve([s[2] for s in systems], xs, rtol)
    assert [r[0] for r in res] == its


def _delaunay1m():
    if "1m" in _BATCH:
        return _BATCH["1m"]
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    if not (GOLDEN / "traj_delaunay1m.npz").exists():  # (make_golden.py headline delaunay1m: ~2 h of scipy)
        pytest.skip("traj_delaunay1m.npz not generated yet")
    z = np.load(GOLDEN / "traj_delaunay1m.npz")
    fx = _sha_fixture()["delaunay1m"]
    A_raw, mask, feats, bs, e2n = P.workload("delaunay1m")
    assert P.matrix_sha256(A_raw) == fx["A_sha256"]  # the container's mesh, bit for bit
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], seed=0)
    d = s.to("cuda")
    boo = ws.forward(d.x, d.edge_index, d.edge_attr)
    assert _shaB(boo.cpu().numpy()) == str(z["boo_sha256"]), "GNN output differs from the recorded bench L"
    L = ws._assemble(d, boo, None)
    A = ws.system_matrix(d)
    Ah = sp.csr_matrix(A.to_scipy())
    assert _shaB(Ah.indptr, Ah.indices, Ah.data) == str(z["A_sha256"])
    del Ah
    b = A.matvec(d.mask.reshape(-1).to(torch.float64))
    _BATCH.clear()
    _BATCH["1m"] = (z, A, L, b)
    return _BATCH["1m"]


@pytest.mark.parametrize("threads", [1, 8])
def test_delaunay1m_parity_mode_equals_reference_run(gpu_ctx, threads):
    """The 1 M-vertex Delaunay system (bench irregular_1m.delaunay1m, SELL-64X views), the bench's GNN
    L, full 16 k-iteration solve in parity mode: count, every ‖r_k‖ and sha256(x) equal to the
    reference's recorded run (make_golden.py headline delaunay1m)."""
    z, A, L, b = _delaunay1m()
    it, conv, x, h = _solve_full(A, L, b, float(z["eps"]), float(z["rtol"]), dot_order="openblas",
                                 dot_threads=threads)
    want = int(z[f"t{threads}__count"])
    assert conv and it == want, (it, want)
    assert np.array_equal(h[:want], z[f"t{threads}__hist"])
    assert _shaB(x.cpu().numpy()) == str(z[f"t{threads}__x_sha256"])


def test_delaunay1m_default_mode(gpu_ctx):
    """Default order on the 1 M Delaunay system (SELL-64X views): the count equals the oracle's
    correctly-rounded-dot count (16,331: make_golden.py's exact-dot run of the reference's scipy
    recurrence on the same A and L), and every ‖r_k‖ and x equal the oracle's bit for bit, with a true
    residual below rtol.  The reference's own runs, which differ only in the OpenBLAS thread count (the dot
    order), spread over 16,810-17,282 iterations on this system: a 16 k-iteration CG is that sensitive
    to the dots' rounding, and the compensated dots reproduce the correctly rounded trajectory."""
    z, A, L, b = _delaunay1m()
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
    assert s.views["A"]["columns"] == "sell16x"
    del s
    rtol = float(z["rtol"])
    it, conv, x, h = _solve_full(A, L, b, float(z["eps"]), rtol)
    ex = int(z["oracle_exact_count"])
    assert conv and it == ex, (it, ex, [int(c) for c in z["ref_counts"]])
    ho = np.asarray(z["oracle_exact_hist"])[:ex]
    assert np.array_equal(h[:ex], ho), float(np.max(np.abs(h[:ex] - ho) / ho))  # every ‖r_k‖, bit for bit
    assert _shaB(x.cpu().numpy()) == str(z["oracle_exact_x_sha256"])
    tres = float(torch.linalg.vector_norm(b - A.matvec(x)) / torch.linalg.vector_norm(b))
    assert tres < rtol, tres
