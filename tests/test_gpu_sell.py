"""GPU parity of the SELL-64 iteration views (csrc/lspcg_sell.hpp) the PCG loop uses.

The SELL kernel must give the CSR kernel's (= scipy csr_matvec's) exact bits on every
matrix shape, and the PCG with SELL views the same iterate / residual history as with the
CSR views (LSPCG_NO_SELL=1) -- bit for bit, not within a tolerance.
"""
import ctypes as C
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from tests import _cases
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _dm(A, dtype=np.float64):
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    return DeviceMatrix.from_scipy(A, dtype=dtype)


def _sell_spmv(Ad, x, compact):
    from learningsparsepreconditioner4gpu_amd import _lib

    y = torch.full_like(x, float("nan"))
    ms = C.c_double()
    _lib.call("lspcg_spmv_sell_timed", Ad.ctx.handle, Ad.handle, int(compact), C.c_void_p(x.data_ptr()),
              C.c_void_p(y.data_ptr()), 1, 0, C.byref(ms))
    return y.cpu().numpy()


@pytest.fixture(autouse=True)
def _given_numbering(monkeypatch):
    """The layouts are tested on the numbering given: the analysis step's reverse-Cuthill-McKee
    reordering of far-from-banded matrices (tests/test_gpu_reorder.py) is turned off here."""
    monkeypatch.setenv("LSPCG_REORDER", "0")


MATS = {
    "synthetic": lambda: P.generate_spd_sparse_matrix(3000, 3e-3, 1e-5, np.random.RandomState(0)),
    "kuhn": lambda: P.kuhn_laplacian(13),
    "ragged": lambda: _cases.ragged_matrix(),  # empty rows, a 5000-entry row
    "n1": lambda: sp.csr_matrix(np.array([[2.5]])),
    "n65": lambda: sp.random(65, 65, density=0.2, random_state=3, format="csr") + sp.eye(65, format="csr"),
    # columns up to 70k rows away from the slice: 16-bit offsets do not fit -> int32 columns
    "wide": lambda: sum(sp.csr_matrix((np.full(70000, 0.5 + k), (np.arange(70000), (np.arange(70000) * (k + 1)
                                                                                  + 9000 * k) % 70000)),
                                      shape=(70000, 70000)) for k in range(4)).tocsr(),
    "zero-rows": lambda: sp.csr_matrix((sp.eye(130, format="csr").toarray() * (np.arange(130) % 3 == 0))),
    # rows 64..191 empty: two whole slices without a single group
    "empty-slices": lambda: sp.csr_matrix(sp.diags(np.where((np.arange(300) // 64) % 3 == 1, 0.0, 1.5 + np.arange(300)))
                                          + sp.diags(np.where((np.arange(299) // 64) % 3 == 1, 0.0, -0.25), 1)),
}


@pytest.mark.parametrize("which", list(MATS))
def test_sell_spmv_bitwise_vs_scipy(gpu_ctx, which):
    A = sp.csr_matrix(MATS[which]()).astype(np.float64)
    A.sort_indices()
    # fp32-representable values so that the compact (fp32-stored) variant is lossless too
    A.data = A.data.astype(np.float32).astype(np.float64)
    x = np.random.default_rng(5).normal(size=A.shape[0])
    x[::17] = -0.0
    ref = A @ x
    Ad = _dm(A)
    xt = torch.from_numpy(x).cuda()
    for flags in (0, 1, 2, 3, 8, 9, 10, 11):  # fp32 values x 16-bit column offsets x SELL-DIA
        y = _sell_spmv(Ad, xt, flags)
        assert np.array_equal(y, ref), (which, flags, np.nanmax(np.abs(y - ref)))


def test_sell_skips_padding_with_inf(gpu_ctx):
    # a short row next to long ones: padded slots must not add 0*inf (NaN) into the sum
    A = sp.csr_matrix(np.triu(np.ones((70, 70))))
    x = np.ones(70)
    x[0] = np.inf
    ref = A @ x
    for flags in (0, 2, 8):
        y = _sell_spmv(_dm(A), torch.from_numpy(x).cuda(), flags)
        assert np.array_equal(np.isnan(y), np.isnan(ref)) and np.array_equal(y[~np.isnan(y)], ref[~np.isnan(ref)])


def _v(no_sell="0", split="1", small="0"):
    return {"LSPCG_NO_SELL": no_sell, "LSPCG_SPLIT_REDUCE": split, "LSPCG_SMALL_N": small}


VARIANTS = [_v(no_sell="1"), _v(), _v(split="0"), _v(small="1000000"), _v(no_sell="1", small="1000000")]


@pytest.mark.parametrize("precond", ["none", "diagonal", "ext_spai", "ext_spai_scaled"])
@pytest.mark.parametrize("case", [0, 1, 2, 3])
def test_pcg_sell_equals_csr_views(gpu_ctx, precond, case, monkeypatch):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    name, A, mask = _cases.spd_cases()[case]
    A = sp.csr_matrix(A).astype(np.float64)
    n = A.shape[0]
    b = torch.from_numpy(A @ np.ones(n)).cuda()
    out = []
    # CSR views (5 kernels); SELL views (split group reductions vs last-arriver reductions);
    # then the one-workgroup solve (k_pcg_small) on the SELL copies and on the CSR views
    # (LSPCG_NO_SELL=1), which every other variant has switched off
    for env in VARIANTS:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=precond)
        if precond.startswith("ext_spai"):
            s.set_spai(_cases.spai_like(A), 1e-3)
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        it, conv, _, hist = s.solve(b, x, rtol=1e-8, return_history=True)
        out.append((it, x.cpu().numpy(), hist))
        del s
    for o in out[1:]:
        assert out[0][0] == o[0], (name, out[0][0], o[0])
        assert np.array_equal(out[0][1], o[1]), name
        assert np.array_equal(out[0][2], o[2]), name


@pytest.mark.parametrize("precond", ["none", "ext_spai"])
def test_pcg_sell_int32_columns_equals_csr_views(gpu_ctx, precond, monkeypatch):
    """A randomly renumbered 3-D grid (n = 42,875): columns up to n rows away from their slice, so
    the loop's SELL views carry int32 columns (16-bit offsets do not fit); same bits as the CSR
    views."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    K = sp.csr_matrix(P.kuhn_laplacian(35, 1e-2))
    perm = np.random.default_rng(2).permutation(K.shape[0])
    A = sp.csr_matrix(K[perm][:, perm])
    A.sort_indices()
    assert _expected_kind(A) == 32
    n = A.shape[0]
    b = torch.from_numpy(A @ np.ones(n)).cuda()
    out = []
    for no_sell in ("1", "0"):
        monkeypatch.setenv("LSPCG_NO_SELL", no_sell)
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=precond)
        if precond == "ext_spai":
            s.set_spai(_cases.spai_like(A), 1e-3)
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        it, conv, _, hist = s.solve(b, x, rtol=1e-8, return_history=True)
        out.append((it, x.cpu().numpy(), hist))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("grid", [11, 13])
def test_small_solve_1024_threads(gpu_ctx, grid, monkeypatch):
    """n = 1331 (2 rows per thread) and 2197 (3 rows): the 1024-thread one-workgroup solve gives the
    5-kernel schedule's count, history and iterate bit for bit."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.kuhn_laplacian(grid, 1e-2))
    n = A.shape[0]
    b = torch.from_numpy(A @ np.ones(n)).cuda()
    out = []
    for small in ("0", "4096"):
        monkeypatch.setenv("LSPCG_SMALL_N", small)
        for pre in ("none", "ext_spai"):
            s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=pre)
            if pre == "ext_spai":
                s.set_spai(_cases.spai_like(A), 1e-3)
            x = torch.zeros(n, dtype=torch.float64, device="cuda")
            it, conv, _, hist = s.solve(b, x, rtol=1e-10, return_history=True)
            out.append((it, x.cpu().numpy(), hist))
    for a, c in ((0, 2), (1, 3)):
        assert out[a][0] == out[c][0]
        assert np.array_equal(out[a][1], out[c][1]) and np.array_equal(out[a][2], out[c][2])


def _dia_slots(A):
    """(max distinct row-relative offsets col - row in a 64-row slice, sum over slices of that count)
    for a CSR with sorted rows."""
    n = A.shape[0]
    rows = np.repeat(np.arange(n), np.diff(A.indptr)).astype(np.int64)
    if rows.size == 0:
        return 0, 0
    key = np.unique((rows // 64) * (1 << 33) + (A.indices.astype(np.int64) - rows + (1 << 32)))
    cnt = np.bincount(key >> 33)
    return int(cnt.max()), int(cnt.sum())


def _expected_kind(A, max_pad=2.0, dia=True, jag=True):
    """lspcg_mat_prepare_spmv's rule: SELL-DIA (kind 1) if SELL-64's padded slots stay <= max_pad * nnz,
    every 64-row slice has <= 16 distinct offsets col - row and the slices' offset counts sum to no more
    than the 4-entry groups' slots (sorted rows); else, where 16-bit column offsets fit (every
    |col - 64*slice| <= 32767), SELL-64J (kind 17) when SELL-64 would pad more than 1.15 * nnz and no
    row has more than 64 entries -- SELL-64X (18) when n >= 2^18 and every 256-row tile reads <= 256
    16-entry x blocks; else none (0) past max_pad; else 16-bit offsets or int32 columns."""
    n = A.shape[0]
    lens = np.diff(A.indptr)
    if n == 0 or A.nnz == 0:
        return 0
    ns = (n + 63) // 64
    pad = np.zeros(ns * 64, dtype=np.int64)
    pad[:n] = lens
    groups = ((pad.reshape(ns, 64).max(axis=1) + 3) // 4).sum()
    overpad = 256 * groups > max_pad * A.nnz
    mx, tot = _dia_slots(A)
    if not overpad and dia and mx <= 16 and tot <= 4 * groups:
        return 1
    rows = np.repeat(np.arange(n), lens)
    off = A.indices - (rows // 64) * 64
    fit16 = bool(np.all(np.abs(off) <= 32767))
    if jag and fit16 and 256 * groups > 1.15 * A.nnz and lens.max() <= 64:
        key = np.unique((rows // 256) * (1 << 32) + A.indices.astype(np.int64) // 16)
        return 18 if n >= 262144 and np.bincount(key >> 32).max() <= 256 else 17  # SELL-64X: large, tiles fit
    if overpad:
        return 0
    return 16 if fit16 else 32


@pytest.mark.parametrize("which", list(MATS))
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_prepare_spmv_keeps_bits(gpu_ctx, which, dtype):
    A = sp.csr_matrix(MATS[which]()).astype(dtype)
    A.sort_indices()
    x = np.random.default_rng(7).normal(size=A.shape[0]).astype(dtype)
    ref = A @ x
    Ad = _dm(A, dtype)
    xt = torch.from_numpy(x).cuda()
    kind = Ad.prepare_spmv()
    assert kind == _expected_kind(A), which
    assert np.array_equal(Ad.matvec(xt).cpu().numpy(), ref), (which, kind)


def test_prepare_spmv_dropped_by_scale_columns(gpu_ctx):
    A = sp.csr_matrix(P.kuhn_laplacian(7))
    Ad = _dm(A)
    assert Ad.prepare_spmv() == 1  # 15 stencil offsets: SELL-DIA
    d = np.random.default_rng(0).uniform(0.5, 2.0, size=A.shape[0])
    Ad.scale_columns_(torch.from_numpy(d).cuda())
    x = np.random.default_rng(1).normal(size=A.shape[0])
    B = A.copy()
    B.data = B.data * d[B.indices]  # lspcg_mat_scale_columns: vals[k] * d[col[k]]
    ref = B @ x
    assert np.array_equal(Ad.matvec(torch.from_numpy(x).cuda()).cpu().numpy(), ref)


@pytest.mark.parametrize("precond", ["none", "ext_spai"])
def test_pcg_bsr3_sell_equals_block_kernel(gpu_ctx, precond, monkeypatch):
    """BSR 3x3 systems: the expanded scalar SELL views give the block kernel's bits."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A, mask, _ = P.elasticity_box(9, 5, 4)
    A = sp.csr_matrix(A)
    n = A.shape[0]
    L = sp.csr_matrix(sp.bsr_matrix(_cases.spai_like(A), blocksize=(3, 3)))
    b = torch.from_numpy(A @ mask.reshape(-1).astype(np.float64)).cuda()
    out = []
    monkeypatch.setenv("LSPCG_SMALL_N", "0")  # block views never take the one-workgroup solve
    for env in ("1", "0"):
        monkeypatch.setenv("LSPCG_NO_SELL", env)
        Ad = DeviceMatrix.from_scipy(A, block_size=3)
        s = PreconditionedConjugateGradient(Ad, device="cuda", preconditioner=precond)
        if precond == "ext_spai":
            s.set_spai(DeviceMatrix.from_scipy(L, block_size=3), 1e-3, block_size=3)
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        it, conv, _, hist = s.solve(b, x, rtol=1e-8, return_history=True)
        out.append((it, x.cpu().numpy(), hist))
        del s
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("bsdia", ["1", "0"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("case", ["elast", "elast-zeros", "ragged"])
def test_prepare_spmv_bsr3_keeps_bits(gpu_ctx, monkeypatch, dtype, case, bsdia):
    """BSR 3x3 analysis step: the BSELL-DIA block copy (a structured mesh: <= 16 block offsets per
    64-block-row slice, no columns) or the BSELL-64 one (one column per block; LSPCG_BSDIA=0, and the
    ragged pattern) gives scipy's bsr_matvec bits (per block row: blocks in column order, c = 0, 1, 2
    inside)."""
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    monkeypatch.setenv("LSPCG_BSDIA", bsdia)
    if case == "ragged":  # block rows of 1..40 blocks, some empty, columns up to the whole range
        rng = np.random.default_rng(4)
        nb = 700
        rows, cols = [], []
        for I in range(nb):
            if I % 53 == 7:
                continue
            k = int(rng.integers(1, 40))
            rows += [I] * k
            cols += list(rng.choice(nb, size=k, replace=False))
        pat = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(nb, nb))
        pat.sort_indices()
        B = sp.bsr_matrix((rng.normal(size=(pat.nnz, 3, 3)), pat.indices, pat.indptr), shape=(3 * nb, 3 * nb))
    else:
        A, _, _ = P.elasticity_box(13, 6, 5)
        B = sp.bsr_matrix(sp.csr_matrix(A), blocksize=(3, 3))
        B.sort_indices()
        if case == "elast-zeros":  # in-block zeros and whole zero blocks (Dirichlet masking keeps them)
            z = np.random.default_rng(1).random(B.data.shape) < 0.2
            B.data[z] = 0.0
    B = sp.bsr_matrix((B.data.astype(dtype), B.indices, B.indptr), shape=B.shape)
    x = np.random.default_rng(9).normal(size=B.shape[0]).astype(dtype)
    ref = B @ x
    Ad = DeviceMatrix.from_scipy(B, dtype=dtype, block_size=3)
    y0 = Ad.matvec(torch.from_numpy(x).cuda()).cpu().numpy()  # staged block kernel
    kind = Ad.prepare_spmv()
    if case == "ragged":
        assert kind in (0, 16, 32)
    else:
        assert kind == (1 if bsdia == "1" else 16), kind
    y = Ad.matvec(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(y0, ref) and np.array_equal(y, ref), (case, kind)


def _offset_matrix(n, offsets, seed=0):
    """Banded matrix with the given row-relative offsets (clipped at the borders)."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for o in offsets:
        i = np.arange(max(0, -o), min(n, n - o))
        rows.append(i)
        cols.append(i + o)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    A = sp.csr_matrix((rng.uniform(-1, 1, rows.size).astype(np.float32).astype(np.float64), (rows, cols)),
                      shape=(n, n))
    A.sort_indices()
    return A


@pytest.mark.parametrize("case", ["15-offsets", "16-offsets", "17-offsets", "tail-slice", "far-offsets", "2d-5pt",
                                  "lower"])
def test_dia_rule_and_bits(gpu_ctx, case):
    """SELL-DIA is chosen exactly when every slice has <= 16 distinct offsets (15 = the Kuhn-tet
    stencil; 17 falls back to 16-bit offsets); offsets far beyond the 16-bit range are fine; a
    ragged last slice (n % 64 != 0) and a non-symmetric (lower-triangular) pattern give scipy's bits."""
    offs15 = [-4097, -4096, -65, -64, -63, -2, -1, 0, 1, 2, 63, 64, 65, 4096, 4097]
    A = {"15-offsets": lambda: _offset_matrix(20000, offs15),
         "16-offsets": lambda: _offset_matrix(20000, offs15 + [5000]),
         "17-offsets": lambda: _offset_matrix(20000, offs15 + [5000, -5000]),
         "tail-slice": lambda: _offset_matrix(4099, offs15, 1),
         "far-offsets": lambda: _offset_matrix(150000, [-120000, -2, -1, 0, 1, 2, 120000], 2),
         "2d-5pt": lambda: sp.csr_matrix(P.poisson2d_grid(70, 61)[0]),
         "lower": lambda: sp.csr_matrix(sp.tril(_offset_matrix(20000, offs15, 3)))}[case]()
    A.sort_indices()
    kind_expected = {"17-offsets": 16}.get(case, 1)
    assert _expected_kind(A) == kind_expected
    x = np.random.default_rng(3).normal(size=A.shape[0])
    x[::13] = -0.0
    ref = A @ x
    Ad = _dm(A)
    assert Ad.prepare_spmv() == kind_expected
    assert np.array_equal(Ad.matvec(torch.from_numpy(x).cuda()).cpu().numpy(), ref)
    for flags in (8, 9, 10, 11):
        assert np.array_equal(_sell_spmv(Ad, torch.from_numpy(x).cuda(), flags), ref), flags


def test_dia_unsorted_rows_fall_back(gpu_ctx):
    """Rows uploaded in a stored, unsorted order (keep_order): SELL-DIA's slot order would not be the
    row's order, so the build takes 16-bit offsets (here the jagged SELL-64J layout: the rows' lengths
    vary) and the sums keep the stored order."""
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    A = _offset_matrix(9000, [-300, -1, 0, 1, 300], 4)
    B = A.copy()
    for i in range(0, B.shape[0], 3):  # reverse every third row
        a, b = B.indptr[i], B.indptr[i + 1]
        B.indices[a:b] = B.indices[a:b][::-1].copy()
        B.data[a:b] = B.data[a:b][::-1].copy()
    B.has_sorted_indices = False
    x = np.random.default_rng(5).normal(size=B.shape[0])
    ref = B @ x  # scipy's csr_matvec sums each row in stored order
    Ad = DeviceMatrix.from_scipy(B, keep_order=True)
    assert Ad.prepare_spmv() == _expected_kind(B, dia=False) == 17
    assert np.array_equal(Ad.matvec(torch.from_numpy(x).cuda()).cpu().numpy(), ref)


@pytest.mark.parametrize("precond", ["none", "ext_spai", "ext_spai_scaled"])
def test_pcg_dia_views_equal_csr_views(gpu_ctx, precond, monkeypatch):
    """A Kuhn grid (n = 5832) on SELL-DIA views: count, history and iterate equal the CSR views' bit
    for bit, under every reduction form and in the one-workgroup solve."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.kuhn_laplacian(18, 1e-2))
    A.sort_indices()
    assert _expected_kind(A) == 1
    n = A.shape[0]
    b = torch.from_numpy(A @ np.ones(n)).cuda()
    out = []
    for env in (_v(no_sell="1"), _v(), _v(split="0"), _v(split="2"), _v(small="1000000")):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=precond)
        if precond.startswith("ext_spai"):
            s.set_spai(_cases.spai_like(A), 1e-3)
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        it, conv, _, hist = s.solve(b, x, rtol=1e-9, return_history=True)
        out.append((it, x.cpu().numpy(), hist))
        del s
    for o in out[1:]:
        assert out[0][0] == o[0]
        assert np.array_equal(out[0][1], o[1]) and np.array_equal(out[0][2], o[2])


def test_pcg_dia_nonsymmetric_L(gpu_ctx, monkeypatch):
    """L with a lower-triangular pattern (not A's): L and its transpose get SELL-DIA views of their own
    (offsets <= 0 / >= 0); same bits as the CSR views."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.kuhn_laplacian(17, 1e-2))
    A.sort_indices()
    L = sp.csr_matrix(sp.tril(_cases.spai_like(A)))
    L.sort_indices()
    n = A.shape[0]
    b = torch.from_numpy(A @ np.ones(n)).cuda()
    out = []
    for env in (_v(no_sell="1"), _v()):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
        s.set_spai(L, 1e-3)
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        it, conv, _, hist = s.solve(b, x, rtol=1e-9, max_iter=400, return_history=True)
        out.append((it, x.cpu().numpy(), hist))
        del s
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("seed", range(8))
def test_dia_randomized_structured(gpu_ctx, seed):
    """Randomized SELL-DIA cases: a random offset set (3..16 offsets, some far apart), random n
    (not a multiple of 64), ~30 % of the entries dropped (ragged rows inside a slice, empty rows),
    explicit zeros kept, fp64 and fp32 values: the analysis step takes SELL-DIA exactly when the rule
    says so and the SpMV gives scipy's bits; x carries -0.0 and a few huge values."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(200, 40000))
    k = int(rng.integers(3, 17))
    offs = sorted(set(int(o) for o in rng.choice(np.r_[np.arange(-70, 71), [-9000, -4096, 4096, 9000]], k,
                                                 replace=False)) | {0})[:16]
    A = _offset_matrix(n, offs, seed)
    drop = rng.random(A.nnz) < 0.3
    A.data[rng.random(A.nnz) < 0.05] = 0.0  # explicit zeros stay stored
    A = sp.csr_matrix((A.data[~drop], A.indices[~drop],
                       np.r_[0, np.cumsum(np.add.reduceat(~drop, A.indptr[:-1]) * (np.diff(A.indptr) > 0))]),
                      shape=A.shape)
    A.sort_indices()
    for dtype in (np.float64, np.float32):
        B = A.astype(dtype)
        x = rng.normal(size=n).astype(dtype)
        x[::11] = -0.0
        x[5::997] = dtype(1e30)
        ref = B @ x
        Ad = _dm(B, dtype)
        kind = Ad.prepare_spmv()
        assert kind == _expected_kind(B), (n, offs, kind)
        y = Ad.matvec(torch.from_numpy(x).cuda()).cpu().numpy()
        assert np.array_equal(y, ref) or np.array_equal(np.isnan(y), np.isnan(ref)) and np.array_equal(
            y[~np.isnan(y)], ref[~np.isnan(ref)]), (n, offs, dtype)
