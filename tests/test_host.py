"""CPU: host-side logic -- generators, byte models, weight packing, sample building."""
from pathlib import Path

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from learningsparsepreconditioner4gpu_amd import problems as P

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_kuhn_roofline_target_sizes():
    # 101^3 -> N = 1,030,301, nnz = 15,210,901 (formula check at small n)
    for n in (3, 5, 8):
        A = P.kuhn_laplacian(n)
        m = n - 1
        want = n ** 3 + 2 * (3 * m * n * n + 3 * m * m * n + m ** 3)
        assert A.nnz == want
        assert (A != A.T).nnz == 0
        assert np.all(np.linalg.eigvalsh(A.toarray()) > 0)


def test_elasticity_is_spd_block3():
    A, mask, nodes = P.elasticity_box(5, 3, 3)
    assert A.shape[0] == 3 * nodes.shape[0]
    assert abs(A - A.T).max() < 1e-6 * abs(A).max()
    assert mask.shape == (nodes.shape[0], 3) and (mask == 0).any()
    ev = np.linalg.eigvalsh(A.toarray())
    assert ev.min() > 0


def test_poisson_masking_semantics():
    A, mask, _ = P.poisson2d_grid(12, 10)
    m = mask.ravel()
    dead = np.where(m == 0)[0]
    assert len(dead) > 0
    for i in dead:
        row = A.getrow(i)
        assert row.nnz == 1 and row[0, i] == 1.0
        assert A.getcol(i).nnz == 1


def test_bench_byte_model():
    import bench

    n, nnz = 1030301, 15210901
    assert bench.spmv_bytes(n, nnz) == 12 * nnz + 20 * n + 4 == 203136836
    assert bench.pcg_bytes_per_iter(n, nnz, nnz) == 3 * 203136836 + 80 * n
    # BSR 3x3: C4's 105,300 block rows, 1,516,846 blocks -> 120.8 MB
    assert bench.bsr3_bytes(105300, 1516846) == 76 * 1516846 + 4 * 105301 + 48 * 105300 == 120755900
    # GNN forward: per edge 2 (1·16 + 256 + 256) + 4·2·2 (48·16 + 256 + 256) + 2 (48·16 + 256 + 16)
    per_edge = 2 * (16 + 256 + 256) + 8 * 2 * (768 + 512) + 2 * (768 + 256 + 16)
    per_node = 2 * (2 * 16 + 512) + 4 * 2 * (256 + 512)
    assert bench.gnn_flops(10, 100, 2, 1, 1) == 100 * per_edge + 10 * per_node


def test_pack_weights_layout():
    from learningsparsepreconditioner4gpu_amd.nn import build_gnn

    H = 16
    ff = lambda i, o: H * i + H + H * H + H + o * H + o
    for node_in, edge_in, bs in [(2, 1, 1), (4, 1, 1), (9, 9, 3)]:
        g = build_gnn(node_in, edge_in, bs, seed=0)
        blob = g.pack_weights()
        want = ff(node_in, H) + ff(edge_in, H) + 4 * ((2 * H + ff(H, H)) + 2 * (6 * H + ff(3 * H, H))) \
            + ff(3 * H, bs * bs)
        assert blob.numel() == want and blob.dtype == torch.float32
        # first block = node encoder lift weight, row-major [16, node_in]
        assert torch.equal(blob[: H * node_in], g.node_enc.lift[0].weight.detach().reshape(-1))


def test_make_sample_edge_mean_feature():
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A = P.generate_spd_sparse_matrix(300, 2e-2, 1e-3, np.random.RandomState(0))
    s = make_sample(A, None, use_edge_features_as_node_feature="mean")
    assert s.x.shape == (300, 2)  # mask + mean edge feature (training/synthetic.sh)
    ei = s.edge_index.numpy()
    tgt = 17
    sel = ei[1] == tgt
    assert np.isclose(s.x[tgt, 1].item(), s.edge_attr.numpy()[sel, 0].astype(np.float64).mean(), rtol=1e-6)


def test_timestat_csv_schema(tmp_path):
    from learningsparsepreconditioner4gpu_amd.infer import Timestat

    st = Timestat()
    st.put("Neural+CUDA", 0.010, 0.002, 113, 6276)
    st.put("Neural+CUDA", 0.020, 0.004, 115, 6300)
    df = st.timestat_to_dataframe()
    assert list(df.columns) == ["Key", "Total Time (ms)", "Solve Time (ms)", "Precond Time (ms)", "#Iteration"]
    assert df.iloc[0]["Total Time (ms)"] == 18.0 and df.iloc[0]["#Iteration"] == 114.0
    al = st.all_time_stat()
    assert list(al.columns) == ["Key", "Solve Time (ms)", "Precond Time (ms)", "#Iteration", "Matrix Size"]
    assert len(al) == 2


# the rows misc/tab_to_latex.py:79-126 and misc/plot_bars.py:54-55 read from an infer CSV (the
# reference's own consumers of infer.py:372-384); `read_csv_data` restates tab_to_latex.py:45-55
TAB_TO_LATEX_KEYS = ("PCG-ic-cpu", "PCG-ainv-cpu", "PCG-diagonal-cpu", "Neural", "PCG-ic-cuda", "PCG-ainv-cuda",
                     "PCG-diagonal-cuda", "Neural+CUDA")


def _read_csv_data(path):
    import csv

    data = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            data[row["Key"]] = {"total": float(row["Total Time (ms)"]), "iter": float(row["#Iteration"]),
                                "construction": float(row["Precond Time (ms)"])}
    return data


def test_infer_csv_reads_with_reference_consumer_keys(tmp_path):
    """The infer CSV carries the row keys the reference's table / plot scripts key on: the GPU rows
    (PCG-{diagonal,ic,ainv}-cuda, Neural+CUDA) from the device path, the host rows Neural and
    PCG-diagonal-cpu from --cpu-rows (PCG-{ic,ainv}-cpu need pymathprim / ilupp, absent)."""
    from learningsparsepreconditioner4gpu_amd import infer

    assert "Neural+CUDA" in infer.__doc__ and "--hip-key" in infer.__doc__
    st = infer.Timestat()
    rows = {"PCG-none-cuda": 474, "PCG-diagonal-cuda": 265, "PCG-ainv-cuda": 172, "PCG-ic-cuda": 100,
            "Neural+CUDA": 113, "Neural": 113, "PCG-none-cpu": 474, "PCG-diagonal-cpu": 265}
    for k, it in rows.items():
        st.put(k, 0.02, 0.001, it, 6276)
    f = tmp_path / "infer_heat_8.csv"
    st.timestat_to_dataframe().to_csv(f, index=False)
    data = _read_csv_data(f)
    gpu = [k for k in TAB_TO_LATEX_KEYS if k.endswith("cuda") or k == "Neural+CUDA"]
    for k in gpu + ["Neural", "PCG-diagonal-cpu"]:
        assert data[k]["iter"] == rows[k] and data[k]["total"] == 21.0 and data[k]["construction"] == 1.0


def test_cpu_rows_restate_reference_scipy_counts():
    """cpu_rows (the --cpu-rows host rows) = the reference's scipy restatements: the recorded
    counts of pcg_counts.npz (validate.py get_*_scipy run by make_golden.py)."""
    import scipy.sparse as sp

    from learningsparsepreconditioner4gpu_amd import cpu_rows

    z = np.load(GOLDEN / "pcg_counts.npz")
    for name in ("synthetic600", "poisson16", "kuhn7"):
        A = sp.csr_matrix((z[f"{name}__data"], z[f"{name}__indices"], z[f"{name}__indptr"]))
        L = A.copy()
        L.data = z[f"{name}__L_data"]
        gt, eps = z[f"{name}__gt"], float(z[f"{name}__eps"])
        for rtol in (1e-6, 1e-8):
            tag = f"{name}__rtol{int(-np.log10(rtol))}"
            assert cpu_rows.get_cg_iter_time_scipy(A, gt, rtol=rtol) == int(z[f"{tag}__none"])
            assert cpu_rows.get_pcg_diagonal_iter_time_scipy(A, gt, rtol=rtol) == int(z[f"{tag}__diagonal"])
            assert cpu_rows.get_pcg_iter_time_scipy(A, gt, L, eps, rtol=rtol) == int(z[f"{tag}__ext_spai"])
            assert cpu_rows.get_pcg_scaled_iter_time_scipy(A, gt, L, eps, rtol=rtol) == int(z[f"{tag}__ext_spai_scaled"])


def test_heat_bunny_c3_stand_in():
    """C3 stand-in (heat.py:22-96 on the voxelised bunny_low_res.obj): ~6.3 k vertices like the
    reference's tetgen mesh (heat.yaml:1 says 6276), SPD, κ in [0.01, 1) as heat.py:83-86, the
    Dirichlet rows masked, and make_data's node input [field, x, y, z, mask]: F_in = 5."""
    from learningsparsepreconditioner4gpu_amd.data import make_sample

    A, mask, feats = P.heat_bunny()
    n = A.shape[0]
    assert 6000 <= n <= 6600 and feats.shape == (n, 4)
    assert abs(A - A.T).max() <= 1e-15 * abs(A).max()
    assert (A.diagonal() > 0).all()
    assert 0.01 - 1e-12 <= feats[:, 0].min() and feats[:, 0].max() < 1.0
    assert 0 < (mask == 0).sum() < 0.1 * n
    s = make_sample(A, mask, node_features=feats)
    assert s.x.shape == (n, 5)
    assert torch.equal(s.x[:, 4], torch.from_numpy(mask[:, 0]).float())
    # the hot path's assembly masks the Dirichlet rows: identity there
    from oracle import linalg as O

    Am = O.to_csr(s.edge_index.numpy(), s.matrix_values.numpy(), n, s.mask.numpy())
    d = np.flatnonzero(mask[:, 0] == 0)
    assert np.array_equal(Am[d].toarray(), np.eye(n)[d])
    # same seed, same system
    A2, _, f2 = P.heat_bunny()
    assert (A != A2).nnz == 0 and np.array_equal(feats, f2)


@pytest.mark.parametrize("order", ["rcm", "rand"])
def test_renumbered_workloads_are_the_same_system(order):
    """problems.workload('kuhn<N>rcm' / 'kuhn<N>rand'): P A Pᵀ and P mask of the structured system
    (same nnz, same spectrum-defining entries), seeded, and -- for rcm -- banded with many more
    distinct row-relative offsets per 64-row slice than the structured ordering (SELL-DIA's 16)."""
    import bench

    A0, m0, _, _, _ = P.workload("kuhn17")
    A1, m1, f, bs, e2n = P.workload(f"kuhn17{order}")
    A2, _, _, _, _ = P.workload(f"kuhn17{order}")
    assert (A1 != A2).nnz == 0 and bs == 1 and f is None
    assert A1.nnz == A0.nnz and A1.shape == A0.shape and m1.sum() == m0.sum()
    assert np.allclose(np.sort(A1.diagonal()), np.sort(A0.diagonal()))
    assert np.array_equal(np.sort(A1.data), np.sort(A0.data))
    assert np.array_equal(np.sort(np.diff(A1.indptr)), np.sort(np.diff(A0.indptr)))
    d0 = bench.dia_counts(A0.indptr, A0.indices)
    d1 = bench.dia_counts(A1.indptr, A1.indices)
    assert d0.max() <= 16 and d1.mean() > d0.mean()
    rows = np.repeat(np.arange(A1.shape[0]), np.diff(A1.indptr))
    bw1 = np.abs(A1.indices - rows).max()
    if order == "rcm":
        assert bw1 < A1.shape[0] // 4


def test_sell_format_model_matches_layouts():
    """bench.sell_kind / sell_format_bytes restate the SELL-64 build's choice and bytes
    (csrc/lspcg_sell.hpp): the Kuhn grid takes SELL-DIA (<= 16 offsets per slice; 64 value slots
    per distinct offset + 128 B of row masks + a 64-B dictionary per slice), its RCM renumbering
    16-bit offsets (4-entry groups, value + 2-B column per slot), a random renumbering int32."""
    import bench

    A, _, _, _, _ = P.workload("kuhn17")
    ns = (A.shape[0] + 63) // 64
    assert bench.sell_kind(A.indptr, A.indices) == 1
    d = bench.dia_counts(A.indptr, A.indices)
    assert bench.sell_format_bytes(A.indptr, A.indices, 1, 4) == 64 * int(d.sum()) * 4 + ns * (128 + 64)
    R, _, _, _, _ = P.workload("kuhn41rcm")  # SELL-64 pads 1.11 x nnz: 16-bit offsets
    assert bench.sell_kind(R.indptr, R.indices) == 16
    assert bench.sell_format_bytes(R.indptr, R.indices, 16, 4) == bench.sell_slots(R.indptr) * 6
    J, _, _, _, _ = P.workload("kuhn17rcm")  # pads 1.17 x nnz: the jagged layout (x-staged only from 2^18 rows)
    assert bench.sell_kind(J.indptr, J.indices) == 17
    nsj = (J.shape[0] + 63) // 64
    assert bench.sell_format_bytes(J.indptr, J.indices, 17, 4) == bench.jag_elems(J.indptr) * 6 + nsj * 80
    assert bench.jag_elems(J.indptr) < bench.sell_slots(J.indptr)
    xb = bench.xs_blocks(J.indptr, J.indices)
    assert xb.max() <= bench.XS_MAX and bench.sell_format_bytes(J.indptr, J.indices, 18, 4) == (
        bench.jag_elems(J.indptr) * 6 + nsj * 80 + 4 * int(xb.sum()) + 4 * xb.size)
    X, _, _, _, _ = P.workload("kuhn41rand")
    assert bench.sell_kind(X.indptr, X.indices) == 32


def test_delaunay_heat_generator_pinned():
    """problems.delaunay_heat (qhull tets of a seeded uniform point cloud, P1 Laplacian + lumped mass,
    heat_tetmesh.py:17-56): this host builds the recorded matrix bits (tests/golden/delaunay_sha.json,
    written by make_golden.py delaunay), an unstructured pattern (rows of 4 to ~31 entries, no
    stencil: >16 distinct offsets per 64-row slice), SPD with a Dirichlet face."""
    import json

    import bench

    fx = json.loads((Path(__file__).parent / "golden" / "delaunay_sha.json").read_text())["delaunay20k"]
    A, m, nodes, bs, _ = P.workload("delaunay20k")
    assert bs == 1 and nodes.shape == (A.shape[0], 3)
    assert (A.shape[0], A.nnz) == (fx["n"], fx["nnz"]) and P.matrix_sha256(A) == fx["A_sha256"]
    assert int((m == 0).sum()) == fx["dirichlet"]
    lens = np.diff(A.indptr)
    assert lens.min() >= 4 and lens.max() > 2 * lens.min() and abs(A - A.T).max() == 0
    assert bench.dia_counts(A.indptr, A.indices).min() > 16 and bench.sell_kind(A.indptr, A.indices) == 17
    assert np.all(A.diagonal() > 0)
    B = P.apply_dbc_masking(A, m)
    assert np.linalg.eigvalsh(B[:400, :400].toarray()).min() > 0
