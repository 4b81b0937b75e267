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
    """Inputs of bench.py's setup, checked against the fixture's sha256 of boo, A and L."""
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
    assert _sha(boo.cpu().numpy()) == str(z["boo_sha256"]), "GNN output differs from the recorded bench L"
    L = ws._assemble(d, boo, None)
    A = ws.system_matrix(d)
    Ah, Lh = _scalar_csr(A), _scalar_csr(L)
    assert _sha(Ah.indptr, Ah.indices, Ah.data) == str(z["A_sha256"])
    assert _sha(Lh.indptr, Lh.indices, Lh.data) == str(z["L_sha256"])
    gt = d.mask.reshape(-1).to(torch.float64)
    b = A.matvec(gt)
    _CACHE.clear()  # one full-size system resident at a time
    _CACHE[workload] = (z, A, L, b, bs)
    return _CACHE[workload]


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
    z, A, L, b, bs = _system(workload)
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
    z, A, L, b, bs = _system(workload)
    rtol = float(z["rtol"])
    it, conv, x, _h = _solve(A, L, b, bs, float(z["eps"]), rtol)
    counts = [int(c) for c in z["ref_counts"]]
    rec = {"workload": workload, "gpu_iters": it, "ref_counts_1_2_4_8": counts,
           "oracle_exact_count": int(z["oracle_exact_count"])}
    assert conv and min(counts) <= it <= max(counts), rec
    r = b - A.matvec(x)
    tres = float(torch.linalg.vector_norm(r) / torch.linalg.vector_norm(b))
    assert tres < rtol, (rec, tres)
