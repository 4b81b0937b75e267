"""GPU parity: device to_csr_cpu (lspcg_assemble) vs the oracle restatement of
validate.py:22-51 / data.py:134-170 -- bit-exact CSR (indptr, indices, data)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu


def _graph(A, bs):
    g = P.to_block_graph(A, bs)
    return g.edge_index, g.block_values, g.num_nodes


def _inputs(which):
    rng = np.random.default_rng(7)
    if which == "poisson":
        A, mask, _ = P.poisson2d_grid(17, 15)
        ei, vals, nb = _graph(A, 1)
        return ei, vals.astype(np.float32), 1, mask
    if which == "poisson-nomask":
        A, mask, _ = P.poisson2d_grid(9, 8)
        ei, vals, nb = _graph(A, 1)
        return ei, vals, 1, None
    if which == "elast":
        A, mask, _ = P.elasticity_box(6, 4, 3)
        ei, vals, nb = _graph(A, 3)
        vals = vals.copy()
        vals[rng.random(vals.shape) < 0.1] = 0.0  # explicit zeros inside blocks are dropped
        return ei, vals.astype(np.float32), 3, mask
    if which == "missing-diag":
        A = P.kuhn_laplacian(5)
        A = sp.csr_matrix(A - sp.diags(A.diagonal()))
        A.eliminate_zeros()
        ei, vals, nb = _graph(A, 1)
        mask = (rng.random((A.shape[0], 1)) > 0.3).astype(np.float64)
        return ei, vals, 1, mask
    if which == "missing-diag-wide":  # ~40 entries per row: the diagonal lands in a later 16-entry chunk
        B = sp.random(300, 300, density=0.07, random_state=11, format="csr")
        A = sp.csr_matrix(B + B.T)
        A.setdiag(0.0)
        A.eliminate_zeros()
        A.sort_indices()
        ei, vals, nb = _graph(A, 1)
        mask = (rng.random((A.shape[0], 1)) > 0.2).astype(np.float64)
        return ei, vals, 1, mask
    raise KeyError(which)


@pytest.mark.parametrize("which", ["poisson", "poisson-nomask", "elast", "missing-diag", "missing-diag-wide"])
@pytest.mark.parametrize("out_dtype", [np.float64, np.float32])
def test_to_csr_bitwise(gpu_ctx, which, out_dtype):
    from learningsparsepreconditioner4gpu_amd.validate import to_csr_cpu

    ei, vals, bs, mask = _inputs(which)
    n = (ei.max() + 1) * bs
    ref = O.to_csr(ei, vals, n, mask, dtype=out_dtype)
    got = to_csr_cpu(torch.from_numpy(ei), torch.from_numpy(vals), n,
                     None if mask is None else torch.from_numpy(mask), dtype=out_dtype)
    assert got.dtype == ref.dtype
    assert np.array_equal(got.indptr, ref.indptr)
    assert np.array_equal(got.indices, ref.indices)
    assert np.array_equal(got.data, ref.data)


def test_bsr_output_matches_scalar(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.validate import to_csr_device

    ei, vals, bs, mask = _inputs("elast")
    n = (ei.max() + 1) * bs
    B = to_csr_device(torch.from_numpy(ei), torch.from_numpy(vals), n, torch.from_numpy(mask),
                      block_output=True).to_scipy()
    ref = O.to_csr(ei, vals, n, mask)
    assert abs(B.tocsr() - ref).max() == 0


def test_unsorted_edges_rejected(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd import _lib
    from learningsparsepreconditioner4gpu_amd.validate import to_csr_cpu

    ei = np.array([[1, 0], [0, 1]], dtype=np.int64)
    with pytest.raises(_lib.LspcgError, match="sorted"):
        to_csr_cpu(torch.from_numpy(ei), torch.ones(2, dtype=torch.float64), 2, None)
