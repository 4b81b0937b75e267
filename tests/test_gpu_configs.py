"""GPU parity at BASELINE.json's configurations (full sizes), through the product's API.

C1  synthetic N=10240, unpreconditioned CG, rtol 1e-8: the correctly-rounded-dot count (default)
    and the reference's recorded counts in the parity dot order (its own count moves with the
    OpenBLAS thread count: 3236 at 1 thread, 3229 at 8)
C2  Poisson-2D 256x256 (N=65,536) fp64, GNN-inferred L, ext_spai PCG rtol 1e-8: GNN output vs
    the torch restatement (fp32, 1e-5), iteration count equal to the oracle's, solution 1e-12
C3  heat on the voxelised bunny (6,310 vertices, 5 % Dirichlet, F_in = 5) fp32, GNN + PCG to 1e-6:
    GNN input width, count equal to the oracle's, solution 1e-5
C4  elasticity box 117x30x30 (N=315,900 dof) BSR 3x3 fp64: full-size block SpMV bit-identical to
    scalar CSR, and the first 25 PCG iterations bit-for-bit against the oracle (residual history
    1e-10, iterate 1e-12) -- the full oracle solve would take minutes on the CPU
C5  the 8 heat systems (400-32000 vertices) of the sharded batch, each count equal to the oracle's
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import gnn as OG
from oracle import linalg as O
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _system(A_raw, mask, feats=None, bs=1, e2n="disable", seed=0):
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs,
                                  seed=seed)
    ds = s.to("cuda")
    L, _ = ws.inference_step(ds)
    A = ws.system_matrix(ds)
    return s, ws, A, L


def _csr(M):
    m = M.to_scipy()
    return sp.csr_matrix(m.tocsr() if M.block_size > 1 else m)


def _solve(A, L, b, eps, rtol, max_iter=0, dtype=np.float64):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai" if L is not None else "none",
                                        dtype=dtype)
    if L is not None:
        s.set_spai(L, eps, block_size=L.block_size)
    bt = torch.from_numpy(np.asarray(b, dtype=dtype)).cuda()
    x = torch.zeros_like(bt)
    it, conv, _, hist = s.solve(bt, x, rtol=rtol, max_iter=max_iter, return_history=True)
    return it, conv, x.cpu().numpy(), hist


def test_c1_synthetic_cg_counts(gpu_ctx):
    """Config 1 built by the product's generator (== the reference's, golden synthetic.npz): the
    default order gives the correctly-rounded-dot count, the parity order the reference's recorded
    counts (3236 at 1 OpenBLAS thread, 3229 at 8; tests/golden/pcg_traj.npz)."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from tests.test_gpu_traj import Z

    A = P.synthetic_c1()
    b = A @ np.ones(A.shape[0])
    it, conv, x, _ = _solve(A, None, b, 0.0, 1e-8)
    assert conv and it == int(Z["synthetic10240__none__oracle_exact_count"]), it
    assert np.linalg.norm(b - A @ x) / np.linalg.norm(b) < 1e-7
    for th, want in ((1, 3236), (8, 3229)):
        s = PreconditionedConjugateGradient(A, device="cuda", dot_order="openblas", dot_threads=th)
        it, _, _ = s(b, np.zeros(A.shape[0]), 1e-8)
        assert it == want == int(Z[f"synthetic10240__none__t{th}__count"]), (th, it)


def test_c2_poisson_gnn_spai_pcg(gpu_ctx):
    A_raw, mask, _ = P.poisson2d_grid(256, 256)
    s, ws, A, L = _system(A_raw, mask)
    assert A.n == 65536
    # the GNN output against the torch restatement with the same seeded weights
    ref = OG.build(s.x.shape[1], s.edge_attr.shape[1], 1, seed=0)
    with torch.no_grad():
        boo = ref(s.x, s.edge_index, s.edge_attr)[1].reshape(-1, 1, 1).numpy()
    L_ref = O.to_csr(s.edge_index.numpy(), boo, A.n, s.mask.numpy())
    L_h = _csr(L)
    assert np.array_equal(L_h.indptr, L_ref.indptr) and np.array_equal(L_h.indices, L_ref.indices)
    assert np.abs(L_h.data - L_ref.data).max() <= 1e-5 * max(1.0, np.abs(L_ref.data).max())
    # PCG on the GPU's own L: same trajectory as the oracle with correctly rounded dots
    A_h = _csr(A)
    gt = s.mask.numpy().ravel().astype(np.float64)
    b = A_h @ gt
    it_o, x_o, h_o = O.pcg(A_h, b, O.spai_operator(L_h, ws.epsilon), rtol=1e-8, dot="exact")
    it, conv, x, h = _solve(A, L, b, ws.epsilon, 1e-8)
    assert conv and it == it_o, (it, it_o)
    assert np.linalg.norm(x - x_o) / np.linalg.norm(x_o) <= 1e-12
    np.testing.assert_allclose(h, h_o, rtol=1e-12, atol=0)


def test_c3_heat_fp32(gpu_ctx):
    A_raw, mask, feats = P.heat_bunny()
    assert 5500 <= A_raw.shape[0] <= 7000
    s, ws, A64, L64 = _system(A_raw, mask, feats)
    assert s.x.shape[1] == 5 and (mask == 0).any()
    A32 = _csr(A64).astype(np.float32)
    L32 = _csr(L64).astype(np.float32)
    b = (A32 @ mask.ravel().astype(np.float32)).astype(np.float32)
    it_o, x_o, _ = O.pcg(A32, b, O.spai_operator(L32, np.float32(ws.epsilon)), rtol=1e-6, dot="exact",
                         dtype=np.float32)
    from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix

    Ad = DeviceMatrix.from_scipy(A32, dtype=np.float32)
    Ld = DeviceMatrix.from_scipy(L32, dtype=np.float32)
    it, conv, x, _ = _solve(Ad, Ld, b, ws.epsilon, 1e-6, dtype=np.float32)
    assert conv and it == it_o, (it, it_o)
    assert np.linalg.norm(x - x_o) / np.linalg.norm(x_o) <= 1e-5


def test_c4_elasticity_bsr3_full_size(gpu_ctx):
    A_raw, mask, feats, bs, e2n = P.workload("elast")
    s, ws, A, L = _system(A_raw, mask, feats, bs=bs, e2n=e2n)
    assert A.block_size == 3 and A.n == 315900
    A_h = A.to_scipy().tocsr()  # keeps the in-block zeros: the block kernel's summation sequence
    x = np.random.default_rng(3).normal(size=A.n)
    y = A.matvec(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(y, A_h @ x)
    # first 25 ext_spai iterations against the oracle on the same blocks
    L_h = L.to_scipy().tocsr()
    gt = s.mask.numpy().ravel().astype(np.float64)
    b = A_h @ gt
    it_o, x_o, h_o = O.pcg(A_h, b, O.spai_operator(L_h, ws.epsilon), rtol=1e-8, max_iter=25, dot="exact")
    it, _, xg, h = _solve(A, L, b, ws.epsilon, 1e-8, max_iter=25)
    assert it == it_o == 25
    np.testing.assert_allclose(h, h_o, rtol=1e-12, atol=0)
    assert np.linalg.norm(xg - x_o) / np.linalg.norm(x_o) <= 1e-12


def test_c5_heat_batch8_counts(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = synthetic_dataset("heat_batch8")
    assert len(samples) == 8
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=samples[0].edge_attr.shape[1],
                                  seed=0)
    for s in samples:
        ds = s.to("cuda")
        L, _ = ws.inference_step(ds)
        A = ws.system_matrix(ds)
        A_h, L_h = _csr(A), _csr(L)
        b = A_h @ s.mask.numpy().ravel().astype(np.float64)
        it_o = O.pcg(A_h, b, O.spai_operator(L_h, ws.epsilon), rtol=1e-6, dot="exact")[0]
        it, conv, _, _ = _solve(A, L, b, ws.epsilon, 1e-6)
        assert conv and it == it_o, (A.n, it, it_o)


def test_bench_system_views_bitwise(gpu_ctx, monkeypatch):
    """The headline system (kuhn101: 1,030,301 rows, SELL-DIA views, GNN-inferred L, ext_spai to
    1e-8) at full size through size-independent properties: the count, every ‖r_k‖ and the iterate
    are bit-identical on SELL-DIA views (split group reductions and last-arriver reductions) and
    on the staged CSR views (LSPCG_NO_SELL=1, scipy's row order by construction), and the true
    residual ‖b - A x‖ / ‖b‖ is below the requested rtol (within the recurrence's drift)."""
    A_raw, mask, _, _, _ = P.workload("kuhn101")
    s, ws, A, L = _system(A_raw, mask)
    assert A.n == 1030301
    gt = s.mask.to("cuda").reshape(-1).to(torch.float64)
    b = A.matvec(gt).cpu().numpy()
    out = []
    for env in ({"LSPCG_NO_SELL": "0", "LSPCG_SPLIT_REDUCE": "1"}, {"LSPCG_NO_SELL": "0", "LSPCG_SPLIT_REDUCE": "0"},
                {"LSPCG_NO_SELL": "1", "LSPCG_SPLIT_REDUCE": "1"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out.append(_solve(A, L, b, ws.epsilon, 1e-8))
    it, conv, x, h = out[0]
    assert conv and it == 212, it
    for o in out[1:]:
        assert o[0] == it and np.array_equal(o[2], x) and np.array_equal(o[3], h)
    A_h = _csr(A)
    assert np.linalg.norm(b - A_h @ x) / np.linalg.norm(b) <= 2e-8
