"""GPU vs the reference's own outputs (tests/golden, produced by tests/golden/make_golden.py):
device to_csr_cpu bit-exact; PCG iteration counts for every preconditioner and both tolerances:
in the reference's dot order (parity mode) equal on every system, in the default compensated
order equal on the well-conditioned ones and equal to the correctly-rounded-dot count on the
ill-conditioned synthetic one."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import linalg as O
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu
WELL_CONDITIONED = ("poisson16", "kuhn7")


def _load(name):
    return np.load(GOLDEN / name, allow_pickle=False)


def test_device_to_csr_matches_reference(gpu_ctx):
    from learningsparsepreconditioner4gpu_amd.validate import to_csr_cpu

    z = _load("to_csr.npz")
    for c in sorted({k.split("__")[0] for k in z.files}):
        m = z[f"{c}__mask"]
        got = to_csr_cpu(torch.from_numpy(z[f"{c}__edge_index"]), torch.from_numpy(z[f"{c}__edge_attr"]),
                         int(z[f"{c}__n"]), None if m.size == 0 else torch.from_numpy(m))
        assert np.array_equal(got.indptr, z[f"{c}__indptr"]), c
        assert np.array_equal(got.indices, z[f"{c}__indices"]), c
        assert np.array_equal(got.data, z[f"{c}__data"]), c


@pytest.mark.parametrize("small_n", ["0", None])
@pytest.mark.parametrize("method", ["none", "diagonal", "ext_spai", "ext_spai_scaled"])
def test_pcg_counts_match_reference(gpu_ctx, method, small_n, monkeypatch):
    """small_n None: the default (these n <= 600 systems take the one-workgroup solve); "0": the
    multi-kernel schedule the bench times."""
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    if small_n is not None:
        monkeypatch.setenv("LSPCG_SMALL_N", small_n)
    else:
        monkeypatch.delenv("LSPCG_SMALL_N", raising=False)

    z = _load("pcg_counts.npz")
    for name in sorted({k.split("__")[0] for k in z.files}):
        ip, ix, d = z[f"{name}__indptr"], z[f"{name}__indices"], z[f"{name}__data"]
        n = ip.size - 1
        A = sp.csr_matrix((d, ix, ip), shape=(n, n))
        L = sp.csr_matrix((z[f"{name}__L_data"], ix, ip), shape=(n, n))
        gt, eps = z[f"{name}__gt"], float(z[f"{name}__eps"])
        b = A @ gt
        for rtol in (6, 8):
            want = int(z[f"{name}__rtol{rtol}__{method}"])
            s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=method)
            x = np.zeros(n)
            it, _, _ = s(b, x, 10.0 ** -rtol, 0, ext_spai=(L, eps) if method.startswith("ext") else None)
            if name in WELL_CONDITIONED:
                assert it == want, (name, rtol, method, it, want)
            else:  # ill-conditioned: the count of the correctly rounded dots (the default's contract)
                ps = {"none": None, "diagonal": O.diagonal_operator(A), "ext_spai": O.spai_operator(L, eps),
                      "ext_spai_scaled": O.spai_scaled_operator(A, L, eps)}[method]
                it_o = O.pcg(A, b, ps, rtol=10.0 ** -rtol, dot="exact")[0]
                assert it == it_o, (name, rtol, method, it, it_o, want)
            # parity mode: the reference's own dot order -> the reference's count, every system
            s.set_dot_order("openblas", 1)
            x = np.zeros(n)
            it, _, _ = s(b, x, 10.0 ** -rtol, 0, ext_spai=(L, eps) if method.startswith("ext") else None)
            assert it == want, ("openblas", name, rtol, method, it, want)


def test_infer_driver_end_to_end(gpu_ctx, tmp_path):
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import Timestat, run
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = [make_sample(*P.poisson2d_grid(20 + 3 * i, 17)[:2]) for i in range(3)]
    ws = SimpleInferenceWorkspace(node_features=1, edge_features=1, seed=0)
    recs = run(samples, ws, rtol=1e-8, warmup=1)
    assert [r.index for r in recs] == [0, 1, 2]
    st = Timestat()
    for r, s in zip(recs, samples):
        assert r.iters > 0 and r.converged
        # the gathered record carries the true ‖b − A x‖/‖b‖ of the solution: below rtol (up to the
        # recurrence/true residual gap) and equal to the oracle's (same trajectory) to 1e-12
        d = s.to("cuda")
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d).to_scipy()
        b = A @ s.mask.numpy().reshape(-1).astype(np.float64)
        it_o, x_o, _ = O.pcg(A, b, O.spai_operator(L.to_scipy(), ws.epsilon), rtol=1e-8, dot="exact")
        rel_o = np.linalg.norm(b - A @ x_o) / np.linalg.norm(b)
        assert r.iters == it_o
        assert r.rel_res <= 1.05e-8 and abs(r.rel_res - rel_o) <= 1e-12, (r.rel_res, rel_o)
        st.put("Neural+CUDA", r.t_solve, r.t_prec, r.iters, r.n)
    df = st.timestat_to_dataframe()
    assert list(df.columns) == ["Key", "Total Time (ms)", "Solve Time (ms)", "Precond Time (ms)", "#Iteration"]


def test_infer_concurrent_solves_match_sequential(gpu_ctx):
    """run(..., concurrency=4): several solves in flight on one GPU give the records of the
    sequential loop (counts, true residuals bit for bit) on the C5 heat batch."""
    from learningsparsepreconditioner4gpu_amd.infer import run, synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = synthetic_dataset("heat_batch8")
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=1, seed=0)
    seq = run(samples, ws, rtol=1e-8, warmup=1)
    con = run(samples, ws, rtol=1e-8, warmup=1, concurrency=4)
    assert [r.index for r in con] == list(range(len(samples)))
    for a, b in zip(seq, con):
        assert a.converged and b.converged
        assert (a.iters, a.rel_res, a.n, a.nnz) == (b.iters, b.rel_res, b.n, b.nnz)


def test_infer_batched_solves_match_sequential(gpu_ctx):
    """run(..., batch=K): the rank's systems solved K at a time in one lockstep batch give the
    records of the sequential loop (counts, convergence, true residuals) on the C5 heat batch."""
    from learningsparsepreconditioner4gpu_amd.infer import run, synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = synthetic_dataset("heat_batch8")
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=1, seed=0)
    seq = run(samples, ws, rtol=1e-8, warmup=1)
    for k in (3, 8):
        bat = run(samples, ws, rtol=1e-8, warmup=1, batch=k)
        assert [r.index for r in bat] == list(range(len(samples)))
        for a, b in zip(seq, bat):
            assert a.converged and b.converged
            assert (a.iters, a.n, a.nnz) == (b.iters, b.n, b.nnz)
            assert abs(a.rel_res - b.rel_res) <= 1e-12 and b.rel_res <= 1e-8


@pytest.mark.parametrize("rhs", ["mask", "neighbour"])
def test_folder_dataset_through_hot_path(gpu_ctx, rhs):
    """On-disk dataset (reference folder format, golden folder_free) -> GNN -> L -> PCG through
    the infer driver; iteration counts equal the oracle's on the same A, L, rhs."""
    import numpy as np

    from learningsparsepreconditioner4gpu_amd.infer import folder_dataset, rhs_for, run
    from learningsparsepreconditioner4gpu_amd.validate import to_csr_cpu
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = folder_dataset(str(GOLDEN / "folder_free"))
    assert len(samples) == 4  # 2 matrices x 2 rhs columns
    s0 = samples[0]
    ws = SimpleInferenceWorkspace(node_features=s0.x.shape[1], edge_features=s0.edge_attr.shape[1], seed=0)
    recs = run(samples, ws, rtol=1e-8, warmup=1, rhs=rhs)
    for rec, s in zip(recs, samples):
        d = s.to("cuda")
        L, _ = ws.inference_step(d)
        A = to_csr_cpu(d.edge_index, d.matrix_values, s.num_nodes, d.mask)
        r = rhs_for(rhs, s.mask.numpy(), d)
        it_o, _, _ = O.pcg(A, A @ r, O.spai_operator(L.to_scipy(), ws.epsilon), rtol=1e-8, dot="exact")
        assert rec.iters == it_o, (rec.index, rec.iters, it_o)  # (tiny systems may need n iterations)


def test_infer_main_parity_mode_reference_counts(gpu_ctx, tmp_path):
    """python -m ...infer --dot-order openblas on folder_free: every row's count equals the count the
    REFERENCE's infer rows recorded on the same samples (infer_folder_free.npz: its FolderDataset,
    seeded GNN, to_csr_cpu and scipy PCG): PCG-none-cuda / PCG-diagonal-cuda and Neural+CUDA per
    sample and as the CSV's #Iteration mean.  (The GNN-L of Neural+CUDA is the HIP forward, within
    1e-7 of the reference's: on these 30- / 35-row systems both take the same count.)"""
    import pandas as pd

    from learningsparsepreconditioner4gpu_amd.infer import main

    z = np.load(GOLDEN / "infer_folder_free.npz")
    k = int(z["len"])
    recs = main(["--folder", str(GOLDEN / "folder_free"), "--rtol", "1e-8", "--warmup", "1", "--out-dir",
                 str(tmp_path), "--dot-order", "openblas", "--dot-threads", "1", "--baselines", "none,diagonal"])
    assert [r.iters for r in sorted(recs, key=lambda r: r.index)] == [int(z[f"{i}__ext_spai"]) for i in range(k)]
    df = pd.read_csv(tmp_path / "infer_folder_free_8.csv").set_index("Key")
    for key, col in (("Neural+CUDA", "ext_spai"), ("PCG-none-cuda", "none"), ("PCG-diagonal-cuda", "diagonal")):
        assert df.loc[key, "#Iteration"] == pytest.approx(np.mean([int(z[f"{i}__{col}"]) for i in range(k)]), abs=1e-9)
    alls = pd.read_csv(tmp_path / "all_infer_folder_free_8.csv")
    for key, col in (("PCG-none-cuda", "none"), ("PCG-diagonal-cuda", "diagonal")):
        got = alls[alls["Key"] == key]["#Iteration"].tolist()
        assert got == [float(z[f"{i}__{col}"]) for i in range(k)], key


def test_infer_main_cpu_rows_reference_counts(gpu_ctx, tmp_path):
    """--cpu-rows: the reference's host rows (Neural, PCG-none-cpu, PCG-diagonal-cpu; scipy
    restatement on the host copies of the device-assembled A and L) beside the GPU rows, with the
    counts the reference's own infer rows recorded on folder_free (infer_folder_free.npz)."""
    import pandas as pd

    from learningsparsepreconditioner4gpu_amd.infer import main

    z = np.load(GOLDEN / "infer_folder_free.npz")
    k = int(z["len"])
    main(["--folder", str(GOLDEN / "folder_free"), "--rtol", "1e-8", "--warmup", "1", "--out-dir", str(tmp_path),
          "--baselines", "none,diagonal", "--cpu-rows"])
    alls = pd.read_csv(tmp_path / "all_infer_folder_free_8.csv")
    for key, col in (("Neural", "ext_spai"), ("PCG-none-cpu", "none"), ("PCG-diagonal-cpu", "diagonal")):
        got = alls[alls["Key"] == key]["#Iteration"].tolist()
        assert got == [float(z[f"{i}__{col}"]) for i in range(k)], key
    keys = set(pd.read_csv(tmp_path / "infer_folder_free_8.csv")["Key"])
    assert {"Neural", "Neural+CUDA", "PCG-none-cpu", "PCG-diagonal-cpu", "PCG-none-cuda", "PCG-diagonal-cuda"} <= keys


@pytest.mark.parametrize("batch", ["1", "4"])
def test_infer_main_writes_baseline_rows(gpu_ctx, tmp_path, batch):
    """infer CLI on an on-disk dataset: Neural+CUDA and PCG-{none,diagonal,ainv,ic}-cuda rows (the
    Neural rows solved one by one or, --batch 4, as one lockstep batch)."""
    import pandas as pd

    from learningsparsepreconditioner4gpu_amd.infer import main

    recs = main(["--folder", str(GOLDEN / "folder_free"), "--rtol", "1e-8", "--warmup", "1", "--out-dir", str(tmp_path),
                 "--batch", batch])
    assert len(recs) == 4 and all(r.iters == r.iters for r in recs)
    df = pd.read_csv(tmp_path / "infer_folder_free_8.csv")
    keys = set(df["Key"])  # (a row whose every solve hit max_iter = n is left out, like the reference)
    assert {"Neural+CUDA", "PCG-ainv-cuda", "PCG-ic-cuda"} <= keys
    assert keys <= {"Neural+CUDA", "PCG-none-cuda", "PCG-diagonal-cuda", "PCG-ainv-cuda", "PCG-ic-cuda"}
    alls = pd.read_csv(tmp_path / "all_infer_folder_free_8.csv")
    assert list(alls.columns) == ["Key", "Solve Time (ms)", "Precond Time (ms)", "#Iteration", "Matrix Size"]
