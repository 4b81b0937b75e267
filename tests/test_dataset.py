"""CPU: the on-disk dataset reader (dataset.FolderDataset, data.py:339-640 + make_data :218-336)
against the reference's own FolderDataset outputs on the committed folders (tests/golden/folder_*,
fixture made by tests/golden/make_golden.py)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from tests.conftest import GOLDEN
from learningsparsepreconditioner4gpu_amd.dataset import FolderDataset, make_data, RawData, to_bcoo_components

CONFIGS = {
    "free": dict(is_fixed_topology=False, load_into_memory=True, block_size=1, has_shared_features=False,
                 use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                 use_node_features_as_edge_feature=False, use_edge_features_as_node_feature="disable",
                 use_random_rhs=False, normalize_matrix="mean", prefix="folder_free"),
    "fixed": dict(is_fixed_topology=True, load_into_memory=False, block_size=3, has_shared_features=True,
                  use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                  use_node_features_as_edge_feature=True, use_edge_features_as_node_feature="disable",
                  use_random_rhs=True, normalize_matrix="frob", prefix="folder_fixed"),
    "free_l1": dict(is_fixed_topology=False, load_into_memory=False, block_size=1, has_shared_features=False,
                    use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=False,
                    use_node_features_as_edge_feature=True, use_edge_features_as_node_feature="disable",
                    use_random_rhs=False, normalize_matrix="l1", prefix="folder_free"),
}
KEYS = ("x", "edge_index", "edge_attr", "mask", "matrix_values", "diagonal", "inv_diag", "rsqrt_diag", "gt",
        "residual")


@pytest.mark.parametrize("name", list(CONFIGS))
def test_folder_dataset_matches_reference(name):
    g = np.load(GOLDEN / "folder.npz", allow_pickle=False)
    cfg = dict(CONFIGS[name])
    cfg["prefix"] = str(GOLDEN / cfg["prefix"])
    ds = FolderDataset(**cfg)
    assert ds.len() == int(g[f"{name}__len"]) == len(ds)
    assert ds.num_node_features == int(g[f"{name}__nnf"])
    assert ds.num_edge_features == int(g[f"{name}__nef"])
    for i in range(ds.len()):
        torch.manual_seed(100 + i)
        d = ds.get(i)
        for k in KEYS:
            ref = g.get(f"{name}__{i}__{k}")
            got = getattr(d, k)
            if ref is None:
                assert got is None, (name, i, k)
                continue
            np.testing.assert_array_equal(got.numpy(), ref, err_msg=f"{name}[{i}].{k}")


def test_bcoo_first_appearance_order():
    # block (0,1) only touched by scalar row 1, after block (0,0) row 0 and before (1,0)
    A = sp.coo_matrix(([1.0, 2.0, 3.0, 4.0], ([0, 1, 1, 2], [0, 3, 0, 1])), shape=(4, 4))
    vals, r, c = to_bcoo_components(A, 2)
    assert list(zip(r, c)) == [(0, 0), (0, 1), (1, 0)]
    assert vals[0, 0, 0] == 1.0 and vals[0, 1, 0] == 3.0 and vals[1, 1, 1] == 2.0 and vals[2, 0, 1] == 4.0


@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
def test_edge_to_node_aggregation(reduce):
    """PyG scatter semantics (parity unpinned: PyG is not installed): nodes without incoming
    edges get 0; checked against a per-node loop."""
    rng = np.random.default_rng(0)
    n = 7
    ei = np.stack([rng.integers(0, n, 30), rng.integers(0, n - 1, 30)])  # node n-1 has no in-edges
    vals = rng.normal(size=(30, 1, 1))
    raw = RawData(vals, None, ei, None, None, None, np.ones((n, 1)), n, 1)
    d = make_data(raw, use_mask_as_node_feature=False, use_edge_features_as_node_feature=reduce,
                  normalize_matrix="none")
    ea = d.edge_attr.numpy()
    exp = np.zeros((n, 1), np.float32)
    for v in range(n):
        sel = ea[ei[1] == v]
        if len(sel):
            exp[v] = {"sum": sel.sum(0), "mean": sel.mean(0), "max": sel.max(0), "min": sel.min(0)}[reduce]
    np.testing.assert_allclose(d.x.numpy(), exp, rtol=1e-6, atol=1e-7)


def test_infer_folder_samples_equal_reference_infer_inputs():
    """infer.folder_dataset (the --folder input of python -m ...infer) yields the GNN / solver inputs
    the reference's own FolderDataset.get gave when infer_folder_free.npz was recorded."""
    from learningsparsepreconditioner4gpu_amd.infer import folder_dataset

    z = np.load(GOLDEN / "infer_folder_free.npz")
    samples = folder_dataset(str(GOLDEN / "folder_free"))
    assert len(samples) == int(z["len"])
    for i, s in enumerate(samples):
        for key in ("x", "edge_index", "edge_attr", "matrix_values", "mask"):
            got = getattr(s, key).numpy()
            ref = z[f"{i}__{key}"]
            assert got.shape == ref.shape and np.array_equal(got, ref), (i, key)
