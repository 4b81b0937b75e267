"""GPU PCG vs the REFERENCE's own run at FULL bench size (tests/golden/traj_<workload>.npz).

The fixtures hold what the reference's infer path computed on the bench's own systems: A from
``to_csr_cpu(edge_index, matrix_values, n, mask)`` (infer.py:282), L from ``to_csr_cpu`` of the
bench's GNN output (the HIP forward's ``boo``, dumped on the GPU box, sha256 stored), and
``get_pcg_iter_time_scipy(A, mask, L, 3e-3, rtol=1e-8)`` (validate.py:163-201) recorded at 1 / 2 /
4 / 8 OpenBLAS threads (tests/golden/make_golden.py ``headline``).  Workloads: the headline
kuhn101 (n = 1,030,301, bench.py's default) and C4, the elasticity box in BSR 3×3 (n = 315,900,
the full 2,458-iteration solve).

Each test first rebuilds the inputs on the box (problems.workload, data.make_sample, the seeded
workspace, the HIP GNN forward) and checks boo, A and L against the recorded sha256, so the
comparison is on the very system the reference solved.  Then:
  * parity mode (``dot_order="openblas"``, 1 and 8 threads): count, every ‖r_k‖ and
    sha256(x) EQUAL to the recorded run;
  * default (compensated) mode, the schedule bench.py times: count inside the reference's
    1/2/4/8-thread spread and the true residual below rtol.

End to end on the REFERENCE's GNN (tests/golden/traj_<workload>_refgnn.npz, make_golden.py
``refgnn``: the reference's seeded NodeEdgeProcessing forward run on the same inputs, its L, its
get_pcg_iter_time_scipy at 1 / 2 / 4 / 8 OpenBLAS threads):
  * the HIP forward's output at every stride-th edge within 1e-5 · max|reference output| of the
    reference's (the full-size GNN pin);
  * the HIP pipeline's count (HIP GNN -> HIP assembly -> HIP PCG, default and parity mode)
    inside the reference-GNN-L counts' spread.
"""
import hashlib

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

WORKLOADS = ["kuhn101", "elast"]


def _sha(*arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _scalar_csr(M):
    """The reference's scalar CSR of a device matrix (to_csr_cpu expands 3x3 blocks and its
    masking addition drops explicit zeros: validate.py:51, data.py:159-170)."""
    import scipy.sparse as sp

    C = sp.csr_matrix(M.to_scipy())
    if M.block_size > 1:
        C.eliminate_zeros()
    C.sort_indices()
    return C


_CACHE = {}


def _system(workload):
    """Inputs of bench.py's setup: (fixture, A, L, b, block size, shas of boo / A / L and the
    boo sample at the reference-GNN fixture's stride).  The tests compare the shas themselves."""
    if workload in _CACHE:
        return _CACHE[workload]
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    z = np.load(GOLDEN / f"traj_{workload}.npz")
    A_raw, mask, feats, bs, e2n = P.workload(workload)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs,
                                  epsilon=float(z["eps"]), seed=0)
    d = s.to("cuda")
    boo = ws.forward(d.x, d.edge_index, d.edge_attr)
    torch.cuda.synchronize()
    booh = boo.cpu().numpy()
    L = ws._assemble(d, boo, None)
    A = ws.system_matrix(d)
    Ah, Lh = _scalar_csr(A), _scalar_csr(L)
    zr = np.load(GOLDEN / f"traj_{workload}_refgnn.npz")
    info = {"boo": _sha(booh), "A": _sha(Ah.indptr, Ah.indices, Ah.data), "L": _sha(Lh.indptr, Lh.indices, Lh.data),
            "boo_sample": booh[:: int(zr["stride"])].copy()}
    gt = d.mask.reshape(-1).to(torch.float64)
    b = A.matvec(gt)
    _CACHE.clear()  # one full-size system resident at a time
    _CACHE[workload] = (z, A, L, b, bs, info)
    return _CACHE[workload]


def _same_system(z, info):
    """The fixture's run was on this very system: boo, A and L have the recorded sha256."""
    assert info["A"] == str(z["A_sha256"])
    assert info["boo"] == str(z["boo_sha256"]), "GNN output differs from the recorded bench L"
    assert info["L"] == str(z["L_sha256"])


def _solve(A, L, b, bs, eps, rtol, **kw):
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", **kw)
    s.set_spai(L, eps, block_size=bs)
    x = torch.zeros_like(b)
    it, conv, _t, h = s.solve(b, x, rtol=rtol, return_history=True)
    return it, conv, x, h


@pytest.mark.parametrize("threads", [1, 8])
@pytest.mark.parametrize("workload", WORKLOADS)
def test_full_size_parity_mode_equals_reference_run(gpu_ctx, workload, threads):
    z, A, L, b, bs, info = _system(workload)
    _same_system(z, info)
    it, conv, x, h = _solve(A, L, b, bs, float(z["eps"]), float(z["rtol"]), dot_order="openblas",
                            dot_threads=threads)
    want = int(z[f"t{threads}__count"])
    xs = x.cpu().numpy()
    rec = {"workload": workload, "threads": threads, "gpu_iters": it, "ref_iters": want}
    assert it == want and conv, rec
    assert np.array_equal(h[:want], z[f"t{threads}__hist"]), rec
    assert np.array_equal(xs[:: int(z["x_stride"])], z[f"t{threads}__x_sample"]), rec
    assert _sha(xs) == str(z[f"t{threads}__x_sha256"]), rec


@pytest.mark.parametrize("workload", WORKLOADS)
def test_full_size_default_mode_within_reference_spread(gpu_ctx, workload):
    z, A, L, b, bs, info = _system(workload)
    _same_system(z, info)
    rtol = float(z["rtol"])
    it, conv, x, _h = _solve(A, L, b, bs, float(z["eps"]), rtol)
    counts = [int(c) for c in z["ref_counts"]]
    rec = {"workload": workload, "gpu_iters": it, "ref_counts_1_2_4_8": counts,
           "oracle_exact_count": int(z["oracle_exact_count"])}
    assert conv and min(counts) <= it <= max(counts), rec
    r = b - A.matvec(x)
    tres = float(torch.linalg.vector_norm(r) / torch.linalg.vector_norm(b))
    assert tres < rtol, (rec, tres)


@pytest.mark.parametrize("workload", WORKLOADS)
def test_full_size_gnn_matches_reference_forward(gpu_ctx, workload):
    """The HIP GNN at full size against the reference's own forward on the same inputs and
    seeded weights: every stride-th edge's outputs within 1e-5 · max|reference output| (fp32,
    the north_star's tolerance).  The fixture also records the all-edge error of the HIP output
    it was compared with in the container (``max_abs_err``)."""
    zr = np.load(GOLDEN / f"traj_{workload}_refgnn.npz")
    *_, info = _system(workload)
    got = info["boo_sample"].astype(np.float64)
    want = zr["ref_sample"].astype(np.float64)
    assert got.shape == want.shape, (got.shape, want.shape)
    err = float(np.abs(got - want).max())
    mref = float(zr["max_abs_ref"])
    rec = {"workload": workload, "sampled_max_abs_err": err, "max_abs_ref": mref,
           "container_all_edge_err": float(zr["max_abs_err"]), "edges_compared": int(got.shape[0])}
    assert err <= 1e-5 * mref, rec
    assert float(zr["max_abs_err"]) <= 1e-5 * mref, rec


@pytest.mark.parametrize("mode", ["compensated", "openblas1", "openblas8"])
@pytest.mark.parametrize("workload", WORKLOADS)
def test_end_to_end_count_within_reference_gnn_spread(gpu_ctx, workload, mode):
    """HIP GNN -> HIP assembly -> HIP PCG (what bench.py times) against the reference end to end
    (its GNN's L, its scipy PCG at 1 / 2 / 4 / 8 OpenBLAS threads): the count lies in that spread
    and the solution's true residual is below rtol."""
    zr = np.load(GOLDEN / f"traj_{workload}_refgnn.npz")
    z, A, L, b, bs, _info = _system(workload)
    assert _info["A"] == str(zr["A_sha256"])
    rtol = float(zr["rtol"])
    kw = {} if mode == "compensated" else {"dot_order": "openblas", "dot_threads": int(mode[len("openblas"):])}
    it, conv, x, _h = _solve(A, L, b, bs, float(zr["eps"]), rtol, **kw)
    counts = [int(c) for c in zr["refL_counts"]]
    rec = {"workload": workload, "mode": mode, "gpu_iters": it, "reference_gnn_counts_1_2_4_8": counts,
           "reference_gnn_oracle_exact": int(zr["oracle_exact_count"])}
    assert conv and min(counts) <= it <= max(counts), rec
    r = b - A.matvec(x)
    assert float(torch.linalg.vector_norm(r) / torch.linalg.vector_norm(b)) < rtol, rec
