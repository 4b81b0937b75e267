"""GPU parity: HIP GNN forward (lspcg_gnn_forward) vs the oracle's torch-CPU restatement,
fp32 within 1e-5 (BASELINE.json north_star), plus the end-to-end inference_step -> PCG."""
import numpy as np
import pytest
import torch

from oracle import gnn as OG
from oracle import linalg as O
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _pair(node_in, edge_in, bs, seed=0):
    from learningsparsepreconditioner4gpu_amd.nn import build_gnn

    ref = OG.build(node_in, edge_in, bs, seed=seed)
    gpu = build_gnn(node_in, edge_in, bs, seed=seed)
    return ref, gpu


def _close(a, b, tol=1e-5):
    scale = max(1.0, float(np.abs(b).max()))
    err = float(np.abs(a - b).max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("case", ["poisson", "synthetic", "elast"])
def test_gnn_forward_matches_oracle(gpu_ctx, case):
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    if case == "poisson":
        A, mask, _ = P.poisson2d_grid(23, 19)
        s = make_sample(A, mask)
        bs = 1
    elif case == "synthetic":
        A = P.generate_spd_sparse_matrix(1500, 4e-3, 1e-5, np.random.RandomState(1))
        s = make_sample(A, None, use_edge_features_as_node_feature="mean")
        bs = 1
    else:
        A, mask, nodes = P.elasticity_box(7, 4, 4)
        s = make_sample(A, mask, node_features=np.concatenate([nodes, nodes * 0.5], 1), block_size=3)
        bs = 3
    ref, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], bs, seed=3)
    with torch.no_grad():
        _, want = ref(s.x, s.edge_index, s.edge_attr)
    _, got = gpu(s.x.cuda(), s.edge_index.cuda(), s.edge_attr.cuda())
    _close(got.cpu().numpy(), want.numpy())


@pytest.mark.parametrize("case", ["poisson", "elast"])
@pytest.mark.parametrize("scale", [1e-9, 1e-4, 1e6, 1e12])
def test_gnn_edge_feature_magnitudes(gpu_ctx, case, scale):
    """Raw edge features far outside f16's range (normalize_matrix="none", data.py:247-267): the
    fused encoder's per-edge power-of-two input scale and its hidden-layer overflow guard keep the
    split-f16 forward at fp32 accuracy -- no inf from inputs >= 65520, no lost bits below 2^-14."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    if case == "poisson":
        A, mask, _ = P.poisson2d_grid(23, 19)
        s = make_sample(A, mask)
        bs = 1
    else:
        A, mask, nodes = P.elasticity_box(7, 4, 4)
        s = make_sample(A, mask, node_features=nodes, block_size=3)
        bs = 3
    ea = s.edge_attr * scale
    ref, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], bs, seed=5)
    with torch.no_grad():
        _, want = ref(s.x, s.edge_index, ea)
    _, got = gpu(s.x.cuda(), s.edge_index.cuda(), ea.cuda())
    got = got.cpu().numpy()
    assert np.isfinite(got).all()
    _close(got, want.numpy())


def test_gnn_weights_past_f16_range_run_fp32(gpu_ctx):
    """MLP weights whose LayerNorm-fed hidden activations could reach 2^15 (the split-f16 GEMMs'
    limit; f16 holds 65504) run: lspcg_gnn_create selects the fp32-MFMA kernels for them, and the
    forward matches the oracle at 1e-5 (no runtime refusal)."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A, mask, _ = P.poisson2d_grid(10, 10)
    s = make_sample(A, mask)
    ref, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], 1, seed=2)
    _, got = gpu(s.x.cuda(), s.edge_index.cuda(), s.edge_attr.cuda())  # as initialised: split-f16
    p0 = gpu.precision()
    assert not p0["f32"] and p0["hidden_bound"] < 2 ** 15, p0
    with torch.no_grad():
        for m in (gpu, ref):
            for p in m.parameters():
                p.mul_(1e3)
        _, want = ref(s.x, s.edge_index, s.edge_attr)
    _, got = gpu(s.x.cuda(), s.edge_index.cuda(), s.edge_attr.cuda())
    p1 = gpu.precision()
    assert p1["f32"] and p1["hidden_bound"] >= 2 ** 15, p1
    got = got.cpu().numpy()
    assert np.isfinite(got).all()
    _close(got, want.numpy())


def test_gnn_tiny_last_layer_weights_run_fp32(gpu_ctx):
    """the split-f16 kernels carry a layer's output scaled by 2^s (max |W| 2^s in
    [2^10, 2^11)) and sum the messages still scaled; a message MLP with tiny last-layer weights
    (x 1e-30) beside O(1) biases has 2^s ~ 2^110, so its scaled messages could overflow fp32.
    lspcg_gnn_create runs such weights on the fp32-MFMA kernels (no scaling): a finite forward within
    1e-5 of the oracle."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A, mask, _ = P.poisson2d_grid(10, 10)
    s = make_sample(A, mask)
    ref, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], 1, seed=3)
    with torch.no_grad():
        for m in (gpu, ref):
            for name, p in m.named_parameters():
                if "msg_mlp.proj" in name and name.endswith("weight"):
                    p.mul_(1e-30)
        _, want = ref(s.x, s.edge_index, s.edge_attr)
    _, got = gpu(s.x.cuda(), s.edge_index.cuda(), s.edge_attr.cuda())
    p1 = gpu.precision()
    assert p1["f32"] and p1["hidden_bound"] < 2 ** 15, p1  # chosen for the scaled range, not the f16 bound
    got = got.cpu().numpy()
    assert np.isfinite(got).all()
    _close(got, want.numpy())


@pytest.mark.parametrize("case", ["poisson", "synthetic", "bunny", "elast"])
def test_gnn_forced_fp32_kernels_match_reference_fixture(gpu_ctx, monkeypatch, case):
    """The fp32-MFMA kernels (LSPCG_GNN_F32=1 forces them at create) on the reference's own
    forward fixtures: within 1e-5, like the default split-f16 kernels."""
    from learningsparsepreconditioner4gpu_amd.nn import build_gnn
    from tests.test_oracle_golden import _load, gnn_fixture

    monkeypatch.setenv("LSPCG_GNN_F32", "1")
    x, ei, ea, bs, seed, sd, want = gnn_fixture(_load("gnn_forward.npz"), case)
    gpu = build_gnn(x.shape[1], ea.shape[1], bs, seed=None)
    gpu.load_state_dict(sd, strict=True)
    _, got = gpu(x.cuda(), ei.cuda(), ea.cuda())
    assert gpu.precision()["f32"]
    _close(got.cpu().numpy(), want)


def test_gnn_decoder_guard_is_per_edge(gpu_ctx):
    """edges of 1e12 and of O(1) magnitude in the same 16-edge tile.  The decoder's
    hidden-layer overflow guard scales per edge, so every small edge keeps fp32 accuracy relative
    to ITS OWN output (a wave-wide factor would flush its f16 low halves)."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A, mask, _ = P.poisson2d_grid(23, 19)
    s = make_sample(A, mask)
    rng = np.random.default_rng(4)
    big = torch.from_numpy(rng.random(s.edge_attr.shape[0]) < 0.3)
    ea = s.edge_attr.clone()
    ea[big] *= 1e12
    ref, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], 1, seed=5)
    with torch.no_grad():
        _, want = ref(s.x, s.edge_index, ea)
    _, got = gpu(s.x.cuda(), s.edge_index.cuda(), ea.cuda())
    got, want = got.cpu().numpy().reshape(len(ea), -1), want.numpy().reshape(len(ea), -1)
    assert np.isfinite(got).all()
    small = ~big.numpy()
    # per edge, relative to the edge's own output; a floor at 1e-3 of the small edges' median
    # magnitude keeps an output that cancels to ~0 from dividing by nothing
    mag = np.abs(want).max(1)
    floor = 1e-3 * np.median(mag[small])
    rel = np.abs(got - want).max(1) / np.maximum(mag, floor)
    assert float(rel[small].max()) <= 1e-5, float(rel[small].max())
    assert float(rel[~small].max()) <= 1e-5, float(rel[~small].max())


def test_gnn_deterministic(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A, mask, _ = P.poisson2d_grid(30, 30)
    s = make_sample(A, mask).to("cuda")
    _, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], 1, seed=1)
    a = gpu(s.x, s.edge_index, s.edge_attr)[1]
    b = gpu(s.x, s.edge_index, s.edge_attr)[1]
    assert torch.equal(a, b)


def test_gnn_invalidate_graph_after_untracked_edit(gpu_ctx):
    """edge_index edited in place through .data (no version bump) keeps the cached CSC;
    invalidate_graph() makes the next forward re-analyse -- equal to a forward on a fresh copy."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A, mask, _ = P.poisson2d_grid(20, 17)
    s = make_sample(A, mask).to("cuda")
    _, gpu = _pair(s.x.shape[1], s.edge_attr.shape[1], 1, seed=2)
    ei = s.edge_index.clone()
    gpu(s.x, ei, s.edge_attr)
    ei.data.copy_(s.edge_index.flip(0))  # the transposed graph: a different CSC, same tensor
    gpu.invalidate_graph()
    got = gpu(s.x, ei, s.edge_attr)[1]
    want = gpu(s.x, s.edge_index.flip(0).contiguous(), s.edge_attr)[1]
    assert torch.equal(got, want)


def test_inference_step_and_pcg_end_to_end(gpu_ctx):
    """GNN -> device assembly of L (masked) -> ext_spai PCG vs oracle on the same L."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace
    from learningsparsepreconditioner4gpu_amd.validate import get_pcg_iter_time

    A, mask, _ = P.poisson2d_grid(26, 21)
    s = make_sample(A, mask)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], seed=0)
    L_dev, dt = ws.inference_step(s)
    assert dt > 0
    # oracle: same GNN weights on CPU, then to_csr restatement
    ref = OG.build(s.x.shape[1], s.edge_attr.shape[1], 1, seed=0)
    with torch.no_grad():
        boo = ref(s.x, s.edge_index, s.edge_attr)[1].reshape(-1, 1, 1).numpy()
    n = A.shape[0]
    L_ref = O.to_csr(s.edge_index.numpy(), boo, n, s.mask.numpy())
    L_got = L_dev.to_scipy()
    assert np.array_equal(L_got.indptr, L_ref.indptr) and np.array_equal(L_got.indices, L_ref.indices)
    _close(L_got.data, L_ref.data)
    # the solve (A assembled on device from the scaled fp32 matrix values, infer.py:282)
    A_dev = ws.system_matrix(s)
    A_ref = O.to_csr(s.edge_index.numpy(), s.matrix_values.numpy(), n, s.mask.numpy())
    assert abs(A_dev.to_scipy() - A_ref).max() == 0
    gt = s.mask.numpy().ravel().astype(np.float64)
    it, prec, solve = get_pcg_iter_time(A_dev, gt, L_dev, ws.epsilon, rtol=1e-8, device="cuda")
    it_o, _, _ = O.pcg(A_ref, A_ref @ gt, O.spai_operator(L_got, ws.epsilon), rtol=1e-8, dot="exact")
    assert it == it_o


@pytest.mark.parametrize("graph", ["asymmetric", "unsorted", "isolated"])
def test_gnn_generic_graphs(gpu_ctx, graph):
    """Edge lists outside the CSR fast path (asymmetric pattern, unsorted order, nodes without
    edges) go through the generic CSC build; results equal the oracle."""
    rng = np.random.default_rng(7)
    N, E = 300, 2400
    src = rng.integers(0, N - 10, E)  # the last 10 nodes have no out-edges
    dst = rng.integers(0, N - 10, E)
    ei = np.unique(np.stack([src, dst]), axis=1)  # row-major sorted, duplicate free, asymmetric
    if graph == "unsorted":
        ei = ei[:, rng.permutation(ei.shape[1])]
    elif graph == "isolated":
        ei = ei[:, ei[0] < N // 2]
    x = torch.from_numpy(rng.normal(size=(N, 3)).astype(np.float32))
    ea = torch.from_numpy(rng.normal(size=(ei.shape[1], 1)).astype(np.float32))
    eit = torch.from_numpy(ei.astype(np.int64))
    ref, gpu = _pair(3, 1, 1, seed=11)
    with torch.no_grad():
        _, want = ref(x, eit, ea)
    _, got = gpu(x.cuda(), eit.cuda(), ea.cuda())
    _close(got.cpu().numpy(), want.numpy())


def test_inference_step_batch_equals_single_forwards(gpu_ctx):
    """One GNN forward over a window's disjoint union of graphs (workspace.inference_step_batch)
    gives every system the L of its own forward, bit for bit (C5 heat systems of 900-30 k nodes)."""
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = [s.to("cuda") for s in synthetic_dataset("heat_batch8")[:5]]
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=samples[0].edge_attr.shape[1],
                                  seed=0)
    Ls, dt = ws.inference_step_batch(samples)
    assert dt > 0 and len(Ls) == len(samples)
    for s, Lb in zip(samples, Ls):
        L1, _ = ws.inference_step(s)
        a, b = L1.to_scipy().tocsr(), Lb.to_scipy().tocsr()
        assert np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
        assert np.array_equal(a.data, b.data)


@pytest.mark.parametrize("case", ["poisson", "synthetic", "bunny", "elast"])
def test_gnn_forward_matches_reference_fixture(gpu_ctx, case):
    """HIP forward vs the REFERENCE's own NodeEdgeProcessing.forward output (gnn_forward.npz,
    made by tests/golden/make_golden.py from gnns.py / basic_layers.py over PyG's dispatch), with
    the reference's parameters loaded through state_dict: fp32 within 1e-5."""
    from learningsparsepreconditioner4gpu_amd.nn import build_gnn
    from tests.test_oracle_golden import _load, gnn_fixture

    x, ei, ea, bs, seed, sd, want = gnn_fixture(_load("gnn_forward.npz"), case)
    gpu = build_gnn(x.shape[1], ea.shape[1], bs, seed=None)
    gpu.load_state_dict(sd, strict=True)
    _, got = gpu(x.cuda(), ei.cuda(), ea.cuda())
    _close(got.cpu().numpy(), want)
