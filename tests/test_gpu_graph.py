"""GraphSpmv / AATPE / LLT (basic_layers.py:112-142, 228-275) on the HIP edge-list kernels
(lspcg_graph_*) vs the oracle's fp64 restatement of PyG's message passing (oracle/gnn.py):
b = 1 and b = 3, unsorted edges with duplicates, mask and diag, fp32 (1e-5, the north_star's
fp32 tolerance) and fp64 (1e-12)."""
import numpy as np
import pytest
import torch

from oracle import gnn as OG

pytestmark = pytest.mark.gpu


def _graph(N, E, seed):
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, N, (2, E), generator=g)
    ei[:, : E // 10] = ei[:, E // 2: E // 2 + E // 10]  # duplicated (row, col) pairs: summed
    return ei


def _rel(a, b):
    a, b = a.double().cpu(), torch.as_tensor(b).double()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-300))


TOL = {torch.float32: 1e-5, torch.float64: 1e-12}


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("bs", [1, 3])
@pytest.mark.parametrize("transpose", [False, True])
@pytest.mark.parametrize("with_mask", [False, True])
def test_graph_spmv(gpu_ctx, dtype, bs, transpose, with_mask):
    from learningsparsepreconditioner4gpu_amd.nn import GraphSpmv

    N, E = 1500, 9000
    ei = _graph(N, E, 1 + bs)
    g = torch.Generator().manual_seed(7)
    A = torch.randn(E, bs, bs, generator=g, dtype=dtype)
    X = torch.randn(N, bs, generator=g, dtype=dtype)
    mask = (torch.rand(N, bs, generator=g) > 0.2).to(dtype) if with_mask else None
    y = GraphSpmv(use_transpose=transpose)(X.cuda(), ei.cuda(), A.cuda(), None if mask is None else mask.cuda())
    ref = OG.graph_spmv(X, ei, A, mask, transpose=transpose)
    assert y.shape == X.shape and y.dtype == dtype
    assert _rel(y, ref) <= TOL[dtype], _rel(y, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("bs", [1, 3])
@pytest.mark.parametrize("with_diag", [False, True])
def test_aatpe(gpu_ctx, dtype, bs, with_diag):
    from learningsparsepreconditioner4gpu_amd.nn import AATPE, LLT

    N, E = 2000, 14000
    ei = _graph(N, E, 11 + bs)
    g = torch.Generator().manual_seed(3)
    A = torch.randn(E, bs, bs, generator=g, dtype=dtype)
    x = torch.randn(N, bs, generator=g, dtype=dtype)
    mask = (torch.rand(N, bs, generator=g) > 0.1).to(dtype)
    diag = torch.rand(N, bs, generator=g, dtype=dtype) + 0.5 if with_diag else None
    y = AATPE(3e-3)(x.cuda(), ei.cuda(), A.cuda(), mask.cuda(), None if diag is None else diag.cuda())
    ref = OG.aatpe(x, ei, A, 3e-3, mask, diag)
    assert _rel(y, ref) <= TOL[dtype], _rel(y, ref)
    if not with_diag:
        z = LLT()(x.cuda(), ei.cuda(), A.cuda(), mask.cuda())
        assert _rel(z, OG.aatpe(x, ei, A, 0.0, mask)) <= TOL[dtype]


def test_aatpe_is_the_ext_spai_apply(gpu_ctx):
    """Unmasked AATPE on the GNN's row-major edge list = the solver's M⁻¹ r = L(Lᵀr) + εr on the
    assembled L (fp64: same products, same per-row order -> equal to 1e-15)."""
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.nn import AATPE
    from learningsparsepreconditioner4gpu_amd.sparse import assemble

    A = P.kuhn_laplacian(9)
    g = P.to_block_graph(A, 1)
    vals = torch.from_numpy(g.block_values).cuda()
    ei = torch.from_numpy(g.edge_index).cuda()
    L = assemble(ei, vals, A.shape[0])
    Lt = L.transpose()
    r = torch.randn(A.shape[0], dtype=torch.float64, device="cuda")
    z_ref = L.matvec(Lt.matvec(r)) + 3e-3 * r
    z = AATPE(3e-3)(r.reshape(-1, 1), ei, vals).reshape(-1)
    assert _rel(z, z_ref.cpu()) <= 1e-15


def test_graph_empty_and_out_of_range(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd import _lib
    from learningsparsepreconditioner4gpu_amd.nn import GraphSpmv

    X = torch.randn(5, 1, device="cuda")
    y = GraphSpmv()(X, torch.zeros(2, 0, dtype=torch.int64, device="cuda"), torch.zeros(0, 1, 1, device="cuda"))
    assert torch.equal(y, torch.zeros_like(X))
    with pytest.raises(_lib.LspcgError):
        GraphSpmv()(X, torch.tensor([[0, 7], [1, 2]], device="cuda"), torch.ones(2, 1, 1, device="cuda"))


@pytest.mark.parametrize("bs", [1, 3])
@pytest.mark.parametrize("dn", ["f64", "f32"])
def test_graph_ops_match_reference_fixture(gpu_ctx, bs, dn):
    """GraphSpmv / AATPE / LLT on the HIP kernels vs the REFERENCE's own modules' outputs
    (graph_spmv.npz: basic_layers.py:112-142, 228-275 over PyG's dispatch, run in the same
    dtype): fp64 within 1e-12, fp32 within 1e-5."""
    from learningsparsepreconditioner4gpu_amd.nn import AATPE, LLT, GraphSpmv
    from tests.test_oracle_golden import _load, graph_fixture

    z = _load("graph_spmv.npz")
    dt = torch.float64 if dn == "f64" else torch.float32
    X, ei, A, m, d = (t.cuda() for t in graph_fixture(z, bs))
    X, A, m, d = X.to(dt), A.to(dt), m.to(dt), d.to(dt)
    eps = float(z["epsilon"])
    got = {
        "spmv_t0": GraphSpmv()(X, ei, A), "spmv_t1": GraphSpmv(True)(X, ei, A),
        "spmv_t0_mask": GraphSpmv()(X, ei, A, m), "spmv_t1_mask": GraphSpmv(True)(X, ei, A, m),
        "aatpe": AATPE(eps)(X, ei, A), "aatpe_mask": AATPE(eps)(X, ei, A, m),
        "aatpe_mask_diag": AATPE(eps)(X, ei, A, m, d), "llt_mask": LLT()(X, ei, A, m),
    }
    tol = TOL[dt]
    for k, y in got.items():
        assert y.dtype == dt
        err = _rel(y, z[f"b{bs}__{dn}__{k}"])
        assert err <= tol, (k, err)
