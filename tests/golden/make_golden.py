"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only in the development container, where /root/reference exists (never on the GPU
box; the committed .npz files are what travels).  The reference targets Python 3.12 with
loguru / torch_geometric / lightning, so a few import shims are installed first
(SURVEY.md 8(c)): ``typing.override`` and stub modules for loguru and torch_geometric.  The
torch_geometric stub carries PyG 2.6.1's ``MessagePassing`` dispatch (collect x_i / x_j by
``flow``, sum-aggregate at i with dim_size = N, then ``update``; ``edge_updater``) and
``utils.scatter`` (sum / mean) restated -- the only PyG code the reference's modules call --
so the GNN / GraphSpmv / AATPE fixtures run the reference's own forward code.

Fixtures (inputs and the reference's outputs, data only):
  to_csr.npz       -- neural_cg/utils/validate.py:22-51 to_csr_cpu on 4 masked/unmasked
                      scalar and 3x3-block COO inputs
  pcg_counts.npz   -- validate.py get_cg_iter_time_scipy / get_pcg_iter_time_scipy /
                      get_pcg_diagonal_iter_time_scipy / get_pcg_scaled_iter_time_scipy
                      iteration counts on small systems (A, L, gt stored)
  synthetic.npz    -- datagen/synthetic.py generate_spd_sparse_matrix(512, 3e-3, 1e-5, RandomState(7))
  gnn_init.npz     -- state_dict of neural_cg.nn.gnns.NodeEdgeProcessing (config/gnn.yaml)
                      constructed after torch.manual_seed(0)
  make_data.npz    -- neural_cg/data.py make_data outputs for one masked block matrix
  pcg_traj.npz     -- the bench-sized trajectories (n = 4,096 / 19,683 / 65,536 and the
                      synthetic C1 system, n = 10,240): the reference's scipy entry points run
                      with scipy's ``cg`` wrapped (``rval.cg``) so that every ‖r_k‖ scipy tests
                      (the argument of each preconditioner call) and the returned x are kept,
                      at 1 / 2 / 4 / 8 OpenBLAS threads (counts of all; history and x of the 1-
                      and 8-thread runs; the BLAS build in ``blas_info``); beside them, labelled
                      ``oracle_exact_*`` (not the reference), the oracle's correctly-rounded-dot
                      trajectory
  gnn_forward.npz  -- the reference's NodeEdgeProcessing.forward (seeded) on make_data inputs of
                      the BASELINE configs' layouts (F_in 1 / 2 / 5 / 9), with its state_dict
  graph_spmv.npz   -- the reference's GraphSpmv / AATPE / LLT on random edge lists (fp32, fp64)
  ic_traj.npz      -- the reference's get_pcg_iter_time_scipy_ichol on the oracle's IC(0) factor
  traj_kuhn101.npz, traj_elast.npz
                   -- the reference's get_pcg_iter_time_scipy at FULL bench size (the headline
                      kuhn101 system, n = 1,030,301, and the C4 elasticity box, n = 315,900) with
                      the bench's own L (the HIP GNN's output, dumped on the GPU box by
                      tools/dump_gnn_l.py; its sha256 is stored and re-checked by the GPU tests):
                      counts at 1 / 2 / 4 / 8 OpenBLAS threads, every ‖r_k‖ and sha256(x) + a
                      sample of x at 1 and 8 threads
  infer_folder_free.npz
                   -- the reference's infer rows (PCG-none / PCG-diagonal / Neural counts, mask
                      rhs, rtol 1e-8) on folder_free, its FolderDataset samples and its seeded GNN
  ../../learningsparsepreconditioner4gpu_amd/meshes/bunny_grid.npz
                   -- voxelised interior of data/objs/bunny_low_res.obj (winding numbers of a
                      regular grid's vertices), input of the C3 heat stand-in (problems.heat_bunny);
                      it lives with the package because bench.py / infer load it as a workload
  folder_free/, folder_fixed/ + folder.npz
                   -- two on-disk datasets in the datagen_helper.py folder format (written by
                      dataset.FolderWriter: .mtx + features/mask/rhs/lhs; fixed-topology 3x3
                      blocks with demo.mtx + value vectors + shared features) and the outputs of
                      the reference's FolderDataset.get(i) for every sample

    python tests/golden/make_golden.py            # every fixture
    python tests/golden/make_golden.py traj       # pcg_traj.npz only
    python tests/golden/make_golden.py gnn        # gnn_forward.npz + graph_spmv.npz only
    python tests/golden/make_golden.py ichol      # ic_traj.npz only
    python tests/golden/make_golden.py infer      # infer_folder_free.npz only
    python tests/golden/make_golden.py headline kuhn101 gpurun_out/.../kuhn101.npy   # traj_kuhn101.npz
    python tests/golden/make_golden.py batch delaunay_batch8 gpurun_out/...         # traj_delaunay_batch8.npz
    python tests/golden/make_golden.py delaunay   # delaunay_sha.json
    python tests/golden/make_golden.py bunny      # bunny_grid.npz only
"""
from __future__ import annotations

import inspect
import os
import sys
import types
import typing
from pathlib import Path

import numpy as np
import scipy.sparse as sp
import torch
from torch import nn

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
ROOT = OUT.parents[1]
MESHES = ROOT / "learningsparsepreconditioner4gpu_amd" / "meshes"


def install_shims():
    typing.override = lambda f: f
    lg = types.ModuleType("loguru")

    class _L:
        def __getattr__(self, _):
            return lambda *a, **k: None

    lg.logger = _L()
    sys.modules["loguru"] = lg
    tg = types.ModuleType("torch_geometric")
    tgd = types.ModuleType("torch_geometric.data")
    tgu = types.ModuleType("torch_geometric.utils")
    tgn = types.ModuleType("torch_geometric.nn")

    class Data:
        def __init__(self, **kw):
            self.__dict__.update(kw)

        def to_dict(self):
            return dict(self.__dict__)

    class Dataset:  # PyG Dataset: len() / get() hooks behind __len__ / __getitem__
        def __init__(self, *a, **k):
            pass

        def __len__(self):
            return self.len()

        def __getitem__(self, i):
            return self.get(i)

    class MessagePassing(nn.Module):
        """PyG 2.6.1's MessagePassing dispatch (torch_geometric/nn/conv/message_passing.py:
        _collect / propagate / edge_updater; SumAggregation -> utils.scatter(reduce="sum")),
        restated for a plain [2, E] edge_index -- the only part of PyG the reference's modules
        call.  Everything the reference computes (message / edge_update / update bodies, the
        MLPs, the residuals) runs from the reference's own source."""

        def __init__(self, aggr="add", flow="source_to_target", node_dim=-2, **kw):
            super().__init__()
            assert aggr in ("add", "sum"), aggr  # the reference uses aggr='add' only (config/gnn.yaml)
            assert flow in ("source_to_target", "target_to_source"), flow
            self.aggr, self.flow, self.node_dim = aggr, flow, node_dim

        def _collect(self, fn, edge_index, kwargs):
            # _collect: i, j = (1, 0) for source_to_target else (0, 1); '<name>_i' / '<name>_j'
            # args are kwargs[name] lifted by index_select(node_dim, edge_index[dim]); the
            # sizes are recorded per side; index = edge_index[i], dim_size = size[i] or size[j]
            assert edge_index.dtype == torch.long and edge_index.dim() == 2 and edge_index.size(0) == 2
            i, j = (1, 0) if self.flow == "source_to_target" else (0, 1)
            size = [None, None]
            out = {}
            for arg in inspect.signature(fn).parameters:
                if arg[-2:] in ("_i", "_j"):
                    dim = j if arg[-2:] == "_j" else i
                    data = kwargs[arg[:-2]]
                    n = data.size(self.node_dim)
                    assert size[dim] in (None, n), "node counts differ"
                    size[dim] = n
                    out[arg] = data.index_select(self.node_dim, edge_index[dim])
                elif arg in kwargs:
                    out[arg] = kwargs[arg]
            return out, edge_index[i], size[i] if size[i] is not None else size[j]

        def propagate(self, edge_index, size=None, **kwargs):
            assert size is None
            msg_kw, index, dim_size = self._collect(self.message, edge_index, kwargs)
            msg = self.message(**msg_kw)
            # SumAggregation: scatter(msg, index, dim=node_dim, dim_size, reduce="sum") =
            # msg.new_zeros(size).scatter_add_(dim, broadcast(index), msg)
            dim = msg.dim() + self.node_dim if self.node_dim < 0 else self.node_dim
            shape = list(msg.shape)
            shape[dim] = dim_size
            idx = index.view([-1 if d == dim else 1 for d in range(msg.dim())]).expand_as(msg)
            aggr = msg.new_zeros(shape).scatter_add_(dim, idx, msg)
            upd = {k: kwargs[k] for k in list(inspect.signature(self.update).parameters)[1:] if k in kwargs}
            return self.update(aggr, **upd)

        def update(self, inputs):  # PyG's default update
            return inputs

        def edge_updater(self, edge_index, size=None, **kwargs):
            kw, _, _ = self._collect(self.edge_update, edge_index, kwargs)
            return self.edge_update(**kw)

    class MessageNorm(nn.Module):  # parameter holder with PyG's state (scale = 1)
        def __init__(self, learn_scale=False):
            super().__init__()
            self.scale = nn.Parameter(torch.empty(1), requires_grad=learn_scale)
            self.reset_parameters()

        def reset_parameters(self):
            self.scale.data.fill_(1.0)

    def scatter(src, index, dim=0, dim_size=None, reduce="sum"):
        """torch_geometric.utils.scatter (PyG 2.6.1) for reduce sum / mean: broadcast index,
        new_zeros(...).scatter_add_; mean divides by the per-node count clamped to >= 1."""
        dim = src.dim() + dim if dim < 0 else dim
        if dim_size is None:
            dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
        shape = list(src.shape)
        shape[dim] = dim_size
        idx = index.view([-1 if d == dim else 1 for d in range(src.dim())]).expand_as(src)
        out = src.new_zeros(shape).scatter_add_(dim, idx, src)
        if reduce in ("sum", "add"):
            return out
        assert reduce == "mean", reduce
        count = src.new_zeros(dim_size).scatter_add_(0, index, src.new_ones(src.size(dim))).clamp(min=1)
        return out / count.view([-1 if d == dim else 1 for d in range(out.dim())])

    tgd.Data, tgd.Dataset = Data, Dataset
    for name in ("coalesce", "remove_self_loops", "to_torch_coo_tensor", "to_edge_index"):
        setattr(tgu, name, None)
    tgu.scatter = scatter
    tgn.MessagePassing, tgn.MessageNorm = MessagePassing, MessageNorm
    sys.modules.update({"torch_geometric": tg, "torch_geometric.data": tgd, "torch_geometric.utils": tgu,
                        "torch_geometric.nn": tgn})
    sys.path.insert(0, str(REF))


def reference_synthetic():
    """datagen/synthetic.py:10-27 executed from the reference's source file."""
    src = (REF / "datagen" / "synthetic.py").read_text()
    body = src.split("class SyntheticDatagen")[0]
    body = "\n".join(l for l in body.splitlines() if not l.startswith(("from typing", "import hydra",
                                                                         "from neural_cg")))
    ns = {}
    exec(compile(body, str(REF / "datagen" / "synthetic.py"), "exec"), ns)
    return ns["generate_spd_sparse_matrix"]


def spai_factor(A, seed=5):
    """Deterministic stand-in for the GNN's L on A's pattern (fp32-representable values, like
    the GNN output): diagonal 1/sqrt(d), off-diagonal N(0, 0.05²)/sqrt(d_row)."""
    n = A.shape[0]
    rng = np.random.default_rng(seed)
    L = A.copy()
    rows = np.repeat(np.arange(n), np.diff(A.indptr))
    d = np.abs(A.diagonal()) + 1e-12
    L.data = rng.normal(size=A.nnz) * 0.05 / np.sqrt(d[rows])
    dg = rows == A.indices
    L.data[dg] = 1.0 / np.sqrt(d[rows[dg]])
    L.data = L.data.astype(np.float32).astype(np.float64)
    return L


class RecordingCG:
    """Stands in for the ``cg`` name inside the reference's validate module: calls scipy's cg
    with the same arguments, recording ‖r_k‖ (np.linalg.norm of the vector scipy hands to the
    preconditioner -- the value it has just compared with atol) and the returned x.  With M=None
    the recorder is the identity that returns its argument itself, like scipy's
    IdentityOperator, so the arithmetic is untouched."""

    def __init__(self):
        from scipy.sparse.linalg import LinearOperator, cg

        self._cg, self._LO = cg, LinearOperator
        self.hist, self.x, self.count = [], None, 0

    def __call__(self, A, b, M=None, callback=None, **kw):
        hist = self.hist = []
        inner = M
        rec = self

        class Rec(self._LO):
            def __init__(self):
                super().__init__(np.dtype(np.float64), A.shape)

            def _matvec(self, v):
                hist.append(float(np.linalg.norm(v)))
                return v if inner is None else inner.matvec(v)

        def cb(xk):
            rec.count += 1
            if callback is not None:
                callback(xk)

        self.count = 0
        x, info = self._cg(A, b, M=Rec(), callback=cb, **kw)
        self.x = np.array(x, dtype=np.float64)
        return x, info


TRAJ_THREADS = (1, 2, 4, 8)  # OpenBLAS thread counts the reference is run at (8 = nproc here)


def blas_info() -> str:
    """numpy / scipy / BLAS build of the process that ran the reference (stored in the fixture)."""
    import json

    import scipy
    import threadpoolctl

    return json.dumps({"numpy": np.__version__, "scipy": scipy.__version__,
                       "threadpool_info": threadpoolctl.threadpool_info()})


def traj_fixtures(rval):
    """pcg_traj.npz.  Every system / method is run through the reference's scipy entry point at
    each OpenBLAS thread count in TRAJ_THREADS (threadpoolctl): numpy's ddot splits vectors of
    n > 10,000 over the threads, so the reference's own rounding -- and on ill-conditioned
    systems its count -- moves with the thread count.  Stored: every run's count; the 1- and
    8-thread runs' ‖r_k‖ history and x; the reference's own spread (x and true residual between
    thread counts); and, labelled ``oracle_exact_*``, the oracle's correctly-rounded-dot
    trajectory (the HIP default's contract)."""
    import threadpoolctl

    from learningsparsepreconditioner4gpu_amd import problems as P
    from oracle import linalg as O

    rec = RecordingCG()
    rval.cg = rec
    systems = {
        "poisson64": P.poisson2d_grid(64, 64)[:2],
        "kuhn27": (P.kuhn_laplacian(27), None),
        "poisson256": P.poisson2d_grid(256, 256)[:2],
        "synthetic10240": (P.synthetic_c1(), None),  # BASELINE config 1 (unpreconditioned only)
    }
    out = {"blas_info": np.array(blas_info()), "ref_threads": np.array(TRAJ_THREADS)}
    for name, (A, mask) in systems.items():
        A = sp.csr_matrix(A)
        A.sort_indices()
        n = A.shape[0]
        gt = np.ones(n) if mask is None else mask.ravel().astype(np.float64)
        L = spai_factor(A)
        eps = 3e-3
        rtol = 1e-8
        out[f"{name}__indptr"], out[f"{name}__indices"], out[f"{name}__data"] = A.indptr, A.indices, A.data
        out[f"{name}__gt"], out[f"{name}__eps"], out[f"{name}__rtol"] = gt, np.array(eps), np.array(rtol)
        methods = ("none",) if name.startswith("synthetic") else ("none", "diagonal", "ext_spai", "ext_spai_scaled")
        if len(methods) > 1:
            out[f"{name}__L_data"] = L.data
        b = A @ gt
        nb = np.linalg.norm(b)
        for m in methods:
            t = f"{name}__{m}"
            runs = {}
            for th in TRAJ_THREADS:
                with threadpoolctl.threadpool_limits(th):
                    if m == "none":
                        cnt = rval.get_cg_iter_time_scipy(A, gt, rtol=rtol)
                    elif m == "diagonal":
                        cnt = rval.get_pcg_diagonal_iter_time_scipy(A, gt, rtol=rtol)
                    elif m == "ext_spai":
                        cnt = rval.get_pcg_iter_time_scipy(A, gt, L, eps, rtol=rtol)
                    else:
                        cnt = rval.get_pcg_scaled_iter_time_scipy(A, gt, L, eps, rtol=rtol)
                assert cnt == rec.count and len(rec.hist) == cnt
                runs[th] = (cnt, rec.x.copy(), np.array(rec.hist))
                if th in (1, 8):
                    out[f"{t}__t{th}__count"] = np.array(cnt)
                    out[f"{t}__t{th}__x"] = rec.x.copy()
                    out[f"{t}__t{th}__hist"] = np.array(rec.hist)  # ‖r_k‖, k = 0 .. count-1
                    out[f"{t}__t{th}__true_res"] = np.array(np.linalg.norm(b - A @ rec.x) / nb)
            counts = [runs[th][0] for th in TRAJ_THREADS]
            out[f"{t}__ref_counts"] = np.array(counts)
            x1 = runs[1][1]
            out[f"{t}__ref_x_spread"] = np.array(max(np.linalg.norm(r[1] - x1) / np.linalg.norm(x1) for r in runs.values()))
            tr = [np.linalg.norm(b - A @ r[1]) / nb for r in runs.values()]
            out[f"{t}__ref_true_res_spread"] = np.array(max(tr) - min(tr))
            ps = {"none": None, "diagonal": O.diagonal_operator(A), "ext_spai": O.spai_operator(L, eps),
                  "ext_spai_scaled": O.spai_scaled_operator(A, L, eps)}[m]
            # the oracle's OpenBLAS restatement reproduces every recorded run bit for bit
            for th in (1, 8):
                it_b, x_b, h_b = O.pcg(A, b, ps, rtol=rtol, dot=f"blas{th}")
                assert it_b == runs[th][0] and np.array_equal(x_b, runs[th][1]), (name, m, th)
                assert np.array_equal(np.asarray(h_b[:it_b]), runs[th][2]), (name, m, th)
            ex = O.pcg(A, b, ps, rtol=rtol, dot="exact")
            out[f"{t}__oracle_exact_count"] = np.array(ex[0])
            out[f"{t}__oracle_exact_x"] = ex[1]
            out[f"{t}__oracle_exact_hist"] = np.asarray(ex[2])
            print(name, m, "reference counts", dict(zip(TRAJ_THREADS, counts)), "exact-dot", ex[0],
                  "ref x spread %.1e" % float(out[f"{t}__ref_x_spread"]), flush=True)
    np.savez_compressed(OUT / "pcg_traj.npz", **out)


def ichol_fixtures(rval):
    """ic_traj.npz: the reference's PCG-IC entry point get_pcg_iter_time_scipy_ichol
    (validate.py:372-419: IncompleteCholeskyPreconditioner(L), two spsolve_triangular calls per
    apply) on the oracle's IC(0) factor (ilupp, the reference's own factorization, is absent:
    the factor arithmetic stays parity-unpinned, the apply and the loop are pinned), recording
    count, every ‖r_k‖ and x at 1 OpenBLAS thread."""
    import threadpoolctl

    from learningsparsepreconditioner4gpu_amd import problems as P
    from oracle import linalg as O
    from oracle import precond as OP

    rec = RecordingCG()
    rval.cg = rec

    def masked(A, m):
        M = O.apply_dbc_masking(sp.csr_matrix(A), m).tocsr()
        M.eliminate_zeros()
        M.sort_indices()
        return M

    A1, m1, _ = P.poisson2d_grid(16, 16)
    A3, m3, _ = P.poisson2d_grid(64, 64)
    systems = {"poisson16": (masked(A1, m1), m1.ravel()), "kuhn7": (sp.csr_matrix(P.kuhn_laplacian(7)), None),
               "poisson64": (masked(A3, m3), m3.ravel())}
    out = {"blas_info": np.array(blas_info())}
    for name, (A, m) in systems.items():
        A.sort_indices()
        gt = np.ones(A.shape[0]) if m is None else m.astype(np.float64)
        L = OP.ic0(A)
        out[f"{name}__indptr"], out[f"{name}__indices"], out[f"{name}__data"] = A.indptr, A.indices, A.data
        out[f"{name}__L_indptr"], out[f"{name}__L_indices"], out[f"{name}__L_data"] = L.indptr, L.indices, L.data
        out[f"{name}__gt"] = gt
        for rtol in (1e-6, 1e-8):
            with threadpoolctl.threadpool_limits(1):
                cnt = rval.get_pcg_iter_time_scipy_ichol(A, L, gt, rtol=rtol)
            assert cnt == rec.count and len(rec.hist) == cnt
            t = f"{name}__rtol{int(-np.log10(rtol))}"
            out[f"{t}__count"] = np.array(cnt)
            out[f"{t}__hist"] = np.array(rec.hist)
            out[f"{t}__x"] = rec.x.copy()
            print("ichol", name, rtol, cnt, flush=True)
    np.savez_compressed(OUT / "ic_traj.npz", **out)


def _sha(*arrs) -> str:
    import hashlib

    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


HEADLINE_THREADS = (1, 2, 4, 8)
X_STRIDE = 997  # sampled iterate entries stored beside the iterate's sha256


def headline_fixtures(rval, workload: str, boo_path: str):
    """traj_<workload>.npz: the reference's own ext_spai PCG on a bench workload at full size.

    Inputs: the bench's system (problems.workload -> data.make_sample, pinned bit-equal to the
    reference's make_data) and the HIP GNN's own output ``boo`` on it (tools/dump_gnn_l.py on the
    GPU box: seeded init, the bench's forward), so the fixture's L is the bench's L.  The
    reference then runs exactly its infer path: ``to_csr_cpu(edge_index, matrix_values, n, mask)``
    for A (infer.py:282), ``to_csr_cpu(edge_index, boo, n, mask, float64)`` for L
    (workspace.py:195-205), and ``get_pcg_iter_time_scipy(A, mask, L, eps, rtol=1e-8)``
    (validate.py:163-201) through RecordingCG at 1 / 2 / 4 / 8 OpenBLAS threads.  Stored: every
    count and true residual; for 1 and 8 threads every ‖r_k‖ and sha256(x) with every 997th entry
    of x; sha256 of boo, A and L (the GPU test checks its inputs against them); labelled
    ``oracle_exact_*``, the oracle's correctly-rounded-dot run.  A is not stored."""
    import json

    import threadpoolctl

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from oracle import linalg as O

    meta = json.load(open(boo_path[:-4] + ".json"))
    boo = np.load(boo_path)
    assert boo.dtype == np.float32 and _sha(boo) == meta["sha256"], "boo file does not match its sha256"
    A_raw, mask, feats, bs, e2n = P.workload(workload)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    n = s.num_nodes * bs
    assert boo.shape == (s.edge_index.shape[1], bs, bs), boo.shape
    A = rval.to_csr_cpu(s.edge_index, s.matrix_values, n, s.mask)
    L = rval.to_csr_cpu(s.edge_index, torch.from_numpy(boo), n, s.mask, dtype=np.float64)
    gt = s.mask.numpy().reshape(-1).astype(np.float64)
    eps, rtol = 3e-3, 1e-8
    rec = RecordingCG()
    rval.cg = rec
    out = {"blas_info": np.array(blas_info()), "ref_threads": np.array(HEADLINE_THREADS),
           "workload": np.array(workload), "n": np.array(n), "nnz_A": np.array(A.nnz), "nnz_L": np.array(L.nnz),
           "block_size": np.array(bs), "eps": np.array(eps), "rtol": np.array(rtol),
           "boo_sha256": np.array(meta["sha256"]), "A_sha256": np.array(_sha(A.indptr, A.indices, A.data)),
           "L_sha256": np.array(_sha(L.indptr, L.indices, L.data)), "x_stride": np.array(X_STRIDE)}
    b = A @ gt
    nb = np.linalg.norm(b)
    runs = {}
    for th in HEADLINE_THREADS:
        with threadpoolctl.threadpool_limits(th):
            cnt = rval.get_pcg_iter_time_scipy(A, gt, L, eps, rtol=rtol)
        assert cnt == rec.count and len(rec.hist) == cnt
        runs[th] = (cnt, rec.x.copy(), np.array(rec.hist))
        out[f"t{th}__count"] = np.array(cnt)
        out[f"t{th}__true_res"] = np.array(np.linalg.norm(b - A @ rec.x) / nb)
        if th in (1, 8):
            out[f"t{th}__hist"] = np.array(rec.hist)
            out[f"t{th}__x_sha256"] = np.array(_sha(rec.x))
            out[f"t{th}__x_sample"] = rec.x[::X_STRIDE].copy()
        print(workload, "threads", th, "count", cnt, "true res %.3e" % float(out[f"t{th}__true_res"]), flush=True)
    out["ref_counts"] = np.array([runs[t][0] for t in HEADLINE_THREADS])
    ps = O.spai_operator(L, eps)
    # the oracle's OpenBLAS restatement reproduces the recorded runs bit for bit (GOLDEN_SKIP_BLAS_CHECK=1
    # skips this self-check for long solves -- delaunay1m: 16 k iterations at 1 M rows, ~30 min a run)
    checked = os.environ.get("GOLDEN_SKIP_BLAS_CHECK", "0") != "1"
    out["oracle_blas_checked"] = np.array(checked)
    for th in (1, 8) if checked else ():
        it_b, x_b, h_b = O.pcg(A, b, ps, rtol=rtol, dot=f"blas{th}")
        assert it_b == runs[th][0] and np.array_equal(x_b, runs[th][1]), (workload, th)
        assert np.array_equal(np.asarray(h_b[:it_b]), runs[th][2]), (workload, th)
    ex = O.pcg(A, b, ps, rtol=rtol, dot="exact")
    out["oracle_exact_count"] = np.array(ex[0])
    out["oracle_exact_hist"] = np.asarray(ex[2])
    out["oracle_exact_x_sha256"] = np.array(_sha(ex[1]))
    print(workload, "reference counts", out["ref_counts"].tolist(), "exact-dot", ex[0], flush=True)
    np.savez_compressed(OUT / f"traj_{workload}.npz", **out)


def batch_fixtures(rval, dataset: str, boo_dir: str):
    """traj_<dataset>.npz: the reference's ext_spai PCG on every system of a C5-style dataset
    (infer.synthetic_dataset, e.g. delaunay_batch8: 8 unstructured Delaunay heat systems of
    400-32 k vertices) with the bench's own L per system (the HIP GNN's output, dumped on the GPU
    box by ``tools/dump_gnn_l.py --dataset``; one workspace for the batch, as bench.c5_rows):
    ``to_csr_cpu`` of A and L and ``get_pcg_iter_time_scipy(A, mask, L, 3e-3, rtol=1e-8)`` through
    RecordingCG at 1 / 2 / 4 / 8 OpenBLAS threads.  Stored per system k: counts, the 1- and
    8-thread ‖r_k‖ histories and sha256(x), sha256 of boo, A and L, the oracle's correctly
    rounded-dot count."""
    import json

    import threadpoolctl

    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from oracle import linalg as O

    samples = synthetic_dataset(dataset)
    eps, rtol = 3e-3, 1e-8
    out = {"dataset": np.array(dataset), "count": np.array(len(samples)), "eps": np.array(eps),
           "rtol": np.array(rtol), "ref_threads": np.array(HEADLINE_THREADS), "blas_info": np.array(blas_info())}
    rec = RecordingCG()
    rval.cg = rec
    for k, smp in enumerate(samples):
        path = f"{boo_dir}/{dataset}_{k}.npy"
        meta = json.load(open(path[:-4] + ".json"))
        boo = np.load(path)
        assert boo.dtype == np.float32 and _sha(boo) == meta["sha256"]
        n = smp.num_nodes
        A = rval.to_csr_cpu(smp.edge_index, smp.matrix_values, n, smp.mask)
        L = rval.to_csr_cpu(smp.edge_index, torch.from_numpy(boo), n, smp.mask, dtype=np.float64)
        gt = smp.mask.numpy().reshape(-1).astype(np.float64)
        out[f"{k}__n"] = np.array(n)
        out[f"{k}__boo_sha256"] = np.array(meta["sha256"])
        out[f"{k}__A_sha256"] = np.array(_sha(A.indptr, A.indices, A.data))
        out[f"{k}__L_sha256"] = np.array(_sha(L.indptr, L.indices, L.data))
        counts = []
        for th in HEADLINE_THREADS:
            with threadpoolctl.threadpool_limits(th):
                cnt = rval.get_pcg_iter_time_scipy(A, gt, L, eps, rtol=rtol)
            assert cnt == rec.count and len(rec.hist) == cnt
            counts.append(cnt)
            if th in (1, 8):
                out[f"{k}__t{th}__hist"] = np.array(rec.hist)
                out[f"{k}__t{th}__x_sha256"] = np.array(_sha(rec.x))
        out[f"{k}__ref_counts"] = np.array(counts)
        b = A @ gt
        out[f"{k}__oracle_exact_count"] = np.array(O.pcg(A, b, O.spai_operator(L, eps), rtol=rtol, dot="exact")[0])
        print(dataset, k, "n", n, "reference counts", counts, "exact-dot", int(out[f"{k}__oracle_exact_count"]),
              flush=True)
    np.savez_compressed(OUT / f"traj_{dataset}.npz", **out)


REFGNN_STRIDE = 127  # every 127th edge's reference output is stored (the GPU test compares there)


def headline_refgnn_fixtures(rdata, rgnn, rval, workload: str, boo_path: str):
    """traj_<workload>_refgnn.npz: the headline end to end on the REFERENCE's own GNN.

    The reference's infer path for one sample (infer.py:278-325) with every stage its own code:
    ``make_data`` (data.py:218-336) on the bench's system, the seeded ``NodeEdgeProcessing``
    (torch.manual_seed(0), config/gnn.yaml -- what SimpleInferenceWorkspace(seed=0) builds;
    gnns.py:77-97 over the PyG dispatch above) run on this container's CPU in fp32,
    ``to_csr_cpu`` of its output (workspace.py:195-205) and ``get_pcg_iter_time_scipy(A, mask,
    L_ref, 3e-3, rtol=1e-8)`` at 1 / 2 / 4 / 8 OpenBLAS threads.  Beside it, the HIP forward's
    output on the same inputs (tools/dump_gnn_l.py on the GPU box, ``boo_path``) is compared with
    the reference's edge by edge.  Stored: the error statistics (max |HIP - ref|, max |ref|, the
    worst per-edge relative error), every REFGNN_STRIDE-th edge of the reference's output (the
    GPU test recomputes the HIP forward and compares there at 1e-5 * max |ref|), the reference-L
    counts / true residuals at every thread count and the 1-thread ‖r_k‖ history, and the
    oracle's correctly-rounded-dot count on the reference L."""
    import json

    import threadpoolctl

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.nn import NodeEdgeProcessing as OurNet
    from oracle import linalg as O

    meta = json.load(open(boo_path[:-4] + ".json"))
    boo = np.load(boo_path)
    assert boo.dtype == np.float32 and _sha(boo) == meta["sha256"], "boo file does not match its sha256"
    A_raw, mask, feats, bs, e2n = P.workload(workload)
    A_raw = sp.csr_matrix(A_raw)
    g = P.to_block_graph(A_raw, bs)
    nn_ = g.num_nodes
    m = np.ones((nn_, bs)) if mask is None else np.asarray(mask, dtype=np.float64).reshape(nn_, bs)
    raw = rdata.RawData(block_values=g.block_values, diagonals=A_raw.diagonal().reshape(-1, bs),
                        edge_index=g.edge_index, node_features=feats, lhs=None, rhs=None, mask=m,
                        num_nodes=nn_, block_size=bs)
    d = rdata.make_data(raw, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                        use_node_features_as_edge_feature=False, use_edge_features_as_node_feature=e2n,
                        use_random_rhs=True, normalize_matrix="mean", is_inference=True)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    for key in ("x", "edge_index", "edge_attr", "matrix_values", "mask"):  # the bench's inputs ARE make_data's
        assert torch.equal(getattr(d, key), getattr(s, key)), key
    torch.manual_seed(0)
    net = rgnn.NodeEdgeProcessing(node_in_features=d.x.shape[1], node_out_features=None,
                                  edge_in_features=d.edge_attr.shape[1], edge_out_features=bs * bs, **_gnn_cfg())
    net.eval()
    torch.manual_seed(0)
    ours = OurNet(node_in_features=d.x.shape[1], node_out_features=None, edge_in_features=d.edge_attr.shape[1],
                  edge_out_features=bs * bs, **_gnn_cfg())
    osd = ours.state_dict()
    for k, v in net.state_dict().items():  # the bench's seeded weights are the reference's
        assert torch.equal(v, osd[k].to(v.dtype).reshape(v.shape)), k
    with torch.no_grad():
        ref = net(d.x, d.edge_index, d.edge_attr)[1].reshape(-1, bs, bs).numpy()
    del net
    assert ref.shape == boo.shape, (ref.shape, boo.shape)
    err = np.abs(boo.astype(np.float64) - ref.astype(np.float64))
    mref = float(np.abs(ref).max())
    e_edge = err.reshape(len(ref), -1).max(1)
    r_edge = np.abs(ref).reshape(len(ref), -1).max(1)
    rel_edge = e_edge / np.maximum(r_edge, 1e-30)
    out = {"workload": np.array(workload), "n": np.array(nn_ * bs), "block_size": np.array(bs),
           "E": np.array(len(ref)), "boo_sha256": np.array(meta["sha256"]),
           "ref_boo_sha256": np.array(_sha(ref)), "max_abs_err": np.array(float(err.max())),
           "max_abs_ref": np.array(mref), "rel_err_vs_max": np.array(float(err.max()) / mref),
           "max_edge_rel_err": np.array(float(rel_edge.max())),
           "p99_edge_rel_err": np.array(float(np.quantile(rel_edge, 0.99))),
           "mean_abs_err": np.array(float(err.mean())), "stride": np.array(REFGNN_STRIDE),
           "ref_sample": ref[::REFGNN_STRIDE].copy(), "blas_info": np.array(blas_info()),
           "torch_threads": np.array(torch.get_num_threads())}
    print(workload, "GNN: max|HIP-ref| %.3e  max|ref| %.3e  rel %.3e  worst edge rel %.3e" % (
        float(err.max()), mref, float(err.max()) / mref, float(rel_edge.max())), flush=True)
    del err, e_edge, r_edge, rel_edge
    n = nn_ * bs
    A = rval.to_csr_cpu(d.edge_index, d.matrix_values, n, d.mask)
    L = rval.to_csr_cpu(d.edge_index, torch.from_numpy(ref), n, d.mask, dtype=np.float64)
    gt = d.mask.numpy().reshape(-1).astype(np.float64)
    eps, rtol = 3e-3, 1e-8
    out.update({"eps": np.array(eps), "rtol": np.array(rtol), "ref_threads": np.array(HEADLINE_THREADS),
                "A_sha256": np.array(_sha(A.indptr, A.indices, A.data)),
                "Lref_sha256": np.array(_sha(L.indptr, L.indices, L.data))})
    rec = RecordingCG()
    rval.cg = rec
    b = A @ gt
    nb = np.linalg.norm(b)
    counts = []
    for th in HEADLINE_THREADS:
        with threadpoolctl.threadpool_limits(th):
            cnt = rval.get_pcg_iter_time_scipy(A, gt, L, eps, rtol=rtol)
        assert cnt == rec.count and len(rec.hist) == cnt
        counts.append(cnt)
        out[f"t{th}__count"] = np.array(cnt)
        out[f"t{th}__true_res"] = np.array(np.linalg.norm(b - A @ rec.x) / nb)
        if th == 1:
            out["t1__hist"] = np.array(rec.hist)
        print(workload, "reference GNN L, threads", th, "count", cnt, "true res %.3e" % float(out[f"t{th}__true_res"]),
              flush=True)
    out["refL_counts"] = np.array(counts)
    ex = O.pcg(A, b, O.spai_operator(L, eps), rtol=rtol, dot="exact")
    out["oracle_exact_count"] = np.array(ex[0])
    print(workload, "reference-GNN-L counts", counts, "exact-dot", ex[0], flush=True)
    np.savez_compressed(OUT / f"traj_{workload}_refgnn.npz", **out)


def _gnn_cfg():
    ff = lambda norm: {"pre_norm": norm, "hidden_channels": 16, "num_layers": 2}
    return dict(node_encoder=ff("none"), edge_encoder=ff("none"), node_decoder=ff("none"), edge_decoder=ff("none"),
                num_mp_layers=4, node_residual=True, edge_residual=True, node_features=16, edge_features=16,
                node_mlp=ff("layer"), edge_mlp=ff("layer"), msg_mlp=ff("layer"), msg_norm=True, aggr="add")


def infer_fixtures(rdata, rgnn, rval):
    """infer_folder_free.npz: the reference's infer.py rows (:278-331) on the on-disk folder_free
    dataset, run from the reference's own modules: FolderDataset(**infer config).get(i), the seeded
    NodeEdgeProcessing (torch.manual_seed(0), config/gnn.yaml -- what infer's
    SimpleInferenceWorkspace(seed=0) builds), A = to_csr_cpu(edge_index, matrix_values, n, mask)
    (:282), L = to_csr_cpu(edge_index, forward(...), n, mask) (workspace.py:195-205), r = mask
    (:297-299), and the PCG-none / PCG-diagonal / Neural counts from get_cg_iter_time_scipy /
    get_pcg_diagonal_iter_time_scipy / get_pcg_iter_time_scipy (the reference's CPU stand-ins,
    validate.py:163-333) at 1 OpenBLAS thread, rtol 1e-8."""
    import threadpoolctl

    cfg = dict(is_fixed_topology=False, load_into_memory=False, block_size=1, has_shared_features=False,
               use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
               use_node_features_as_edge_feature=False, use_edge_features_as_node_feature="disable",
               use_random_rhs=True, normalize_matrix="mean", prefix=str(OUT / "folder_free"))
    ds = rdata.FolderDataset(**cfg)
    out = {"rtol": np.array(1e-8), "eps": np.array(3e-3), "len": np.array(ds.len())}
    for i in range(ds.len()):
        torch.manual_seed(100 + i)
        d = ds.get(i)
        n = d.x.shape[0]
        torch.manual_seed(0)
        net = rgnn.NodeEdgeProcessing(node_in_features=d.x.shape[1], node_out_features=None,
                                      edge_in_features=d.edge_attr.shape[1], edge_out_features=1, **_gnn_cfg())
        net.eval()
        with torch.no_grad():
            boo = net(d.x, d.edge_index, d.edge_attr)[1].reshape(-1, 1, 1)
        A = rval.to_csr_cpu(d.edge_index, d.matrix_values, n, d.mask)
        L = rval.to_csr_cpu(d.edge_index, boo, n, d.mask, dtype=np.float64)
        r = d.mask.numpy().reshape(-1).astype(np.float64)
        with threadpoolctl.threadpool_limits(1):
            out[f"{i}__none"] = np.array(rval.get_cg_iter_time_scipy(A, r, rtol=1e-8))
            out[f"{i}__diagonal"] = np.array(rval.get_pcg_diagonal_iter_time_scipy(A, r, rtol=1e-8))
            out[f"{i}__ext_spai"] = np.array(rval.get_pcg_iter_time_scipy(A, r, L, 3e-3, rtol=1e-8))
        out[f"{i}__n"] = np.array(n)
        for key in ("x", "edge_index", "edge_attr", "matrix_values", "mask"):
            out[f"{i}__{key}"] = getattr(d, key).numpy()
        print("infer folder_free", i, "n", n, {k: int(out[f"{i}__{k}"]) for k in ("none", "diagonal", "ext_spai")},
              flush=True)
    np.savez_compressed(OUT / "infer_folder_free.npz", **out)


def gnn_forward_fixtures(rdata, rgnn):
    """gnn_forward.npz: the REFERENCE's NodeEdgeProcessing.forward (gnns.py:77-97, MPLayer
    basic_layers.py:193-225 over the PyG dispatch above) on inputs built by the reference's own
    make_data (data.py:218-336), seeded construction (torch.manual_seed(seed), config/gnn.yaml).
    Cases: the BASELINE configs' input layouts -- Poisson (F_in 1), synthetic with the mean edge
    feature (F_in 2), the heat bunny (field + xyz + mask, F_in 5), elasticity b = 3 (xyz + deform
    + mask, F_in 9, 9 edge features)."""
    from learningsparsepreconditioner4gpu_amd import problems as P

    gen = reference_synthetic()
    cases = {}
    A, m, _ = P.poisson2d_grid(23, 19)
    cases["poisson"] = (A, m, None, 1, "disable", 3)
    A = gen(1500, 4e-3, 1e-5, np.random.RandomState(1))
    cases["synthetic"] = (A, None, None, 1, "mean", 4)
    A, m, f = P.heat_bunny()
    cases["bunny"] = (A, m, f, 1, "disable", 5)
    A, m, nodes = P.elasticity_box(7, 4, 4)
    cases["elast"] = (A, m, np.concatenate([nodes, nodes * 0.5], 1), 3, "disable", 6)
    out = {}
    for name, (A, m, feats, bs, e2n, seed) in cases.items():
        A = sp.csr_matrix(A)
        A.sort_indices()
        g = P.to_block_graph(A, bs)
        if m is None:
            m = np.ones((g.num_nodes, bs))
        raw = rdata.RawData(block_values=g.block_values, diagonals=A.diagonal().reshape(-1, bs),
                            edge_index=g.edge_index, node_features=feats, lhs=None, rhs=None,
                            mask=np.asarray(m, dtype=np.float64).reshape(g.num_nodes, bs), num_nodes=g.num_nodes,
                            block_size=bs)
        d = rdata.make_data(raw, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                            use_node_features_as_edge_feature=False, use_edge_features_as_node_feature=e2n,
                            use_random_rhs=True, normalize_matrix="mean", is_inference=True)
        torch.manual_seed(seed)
        net = rgnn.NodeEdgeProcessing(node_in_features=d.x.shape[1], node_out_features=None,
                                      edge_in_features=d.edge_attr.shape[1], edge_out_features=bs * bs, **_gnn_cfg())
        net.eval()
        with torch.no_grad():
            node_out, edge_out = net(d.x, d.edge_index, d.edge_attr)
        out[f"{name}__x"] = d.x.numpy()
        out[f"{name}__edge_index"] = d.edge_index.numpy()
        out[f"{name}__edge_attr"] = d.edge_attr.numpy()
        out[f"{name}__mask"] = d.mask.numpy()
        out[f"{name}__block_size"] = np.array(bs)
        out[f"{name}__seed"] = np.array(seed)
        out[f"{name}__edge_out"] = edge_out.numpy()
        out[f"{name}__node_out"] = node_out.numpy()
        for k, v in net.state_dict().items():
            out[f"{name}__sd__{k}"] = v.numpy()
        print("gnn", name, "N", d.x.shape, "E", d.edge_attr.shape, "out |max|", float(edge_out.abs().max()), flush=True)
    np.savez_compressed(OUT / "gnn_forward.npz", **out)


def graph_spmv_fixtures(rbl):
    """graph_spmv.npz: the REFERENCE's GraphSpmv(use_transpose) (basic_layers.py:112-142), AATPE(ε)
    (:228-261, with mask and with mask + diag) and LLT (:264-275) over the PyG dispatch above, on
    random edge lists (unsorted, with duplicated (row, col) pairs), b = 1 and b = 3, fp32 and fp64."""
    out = {}
    for bs in (1, 3):
        g = torch.Generator().manual_seed(40 + bs)
        N, E = 700, 5000
        ei = torch.randint(0, N, (2, E), generator=g)
        ei[:, : E // 10] = ei[:, E // 2: E // 2 + E // 10]
        A = torch.randn(E, bs, bs, generator=g, dtype=torch.float64)
        X = torch.randn(N, bs, generator=g, dtype=torch.float64)
        mask = (torch.rand(N, bs, generator=g) > 0.2).to(torch.float64)
        diag = torch.rand(N, bs, generator=g, dtype=torch.float64) + 0.5
        t = f"b{bs}"
        out[f"{t}__edge_index"], out[f"{t}__A"], out[f"{t}__X"] = ei.numpy(), A.numpy(), X.numpy()
        out[f"{t}__mask"], out[f"{t}__diag"] = mask.numpy(), diag.numpy()
        for dt, dn in ((torch.float64, "f64"), (torch.float32, "f32")):
            Ad, Xd, md, dd = A.to(dt), X.to(dt), mask.to(dt), diag.to(dt)
            with torch.no_grad():
                for tr in (False, True):
                    op = rbl.GraphSpmv(use_transpose=tr)
                    out[f"{t}__{dn}__spmv_t{int(tr)}"] = op(Xd, ei, Ad).numpy()
                    out[f"{t}__{dn}__spmv_t{int(tr)}_mask"] = op(Xd, ei, Ad, md).numpy()
                op = rbl.AATPE(3e-3)
                out[f"{t}__{dn}__aatpe_mask"] = op(Xd, ei, Ad, md).numpy()
                out[f"{t}__{dn}__aatpe_mask_diag"] = op(Xd, ei, Ad, md, dd).numpy()
                out[f"{t}__{dn}__aatpe"] = op(Xd, ei, Ad).numpy()
                out[f"{t}__{dn}__llt_mask"] = rbl.LLT()(Xd, ei, Ad, md).numpy()
    out["epsilon"] = np.array(3e-3)
    np.savez_compressed(OUT / "graph_spmv.npz", **out)
    print("graph_spmv fixtures", len(out))


def bunny_grid():
    """bunny_grid.npz: which vertices of a regular grid over data/objs/bunny_low_res.obj's bounding
    box lie inside the surface (generalised winding number > 1/2) -- the voxelised interior from
    which problems.heat_bunny builds the C3 stand-in (tetgen is absent).  The obj
    is parsed as plain text (v / f records); nothing of the reference is imported."""
    V, F = [], []
    for line in (REF / "data" / "objs" / "bunny_low_res.obj").read_text().splitlines():
        if line.startswith("v "):
            V.append([float(t) for t in line.split()[1:4]])
        elif line.startswith("f "):
            F.append([int(t.split("/")[0]) - 1 for t in line.split()[1:4]])
    V, F = np.asarray(V), np.asarray(F)
    lo, hi = V.min(0), V.max(0)
    h = float((hi - lo).max() / 32.0)
    shape = (np.ceil((hi - lo) / h).astype(int) + 1)
    P = np.stack(np.meshgrid(*[lo[k] + h * np.arange(shape[k]) for k in range(3)], indexing="ij"), -1).reshape(-1, 3)
    a, b, c = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    wn = np.zeros(len(P))
    for i in range(0, len(P), 1024):  # Van Oosterom-Strackee solid angles / 4 pi
        p = P[i:i + 1024, None, :]
        A, B, C = a[None] - p, b[None] - p, c[None] - p
        la, lb, lc = (np.linalg.norm(X, axis=2) for X in (A, B, C))
        det = np.einsum("ijk,ijk->ij", A, np.cross(B, C))
        den = (la * lb * lc + np.einsum("ijk,ijk->ij", A, B) * lc + np.einsum("ijk,ijk->ij", B, C) * la
               + np.einsum("ijk,ijk->ij", C, A) * lb)
        wn[i:i + 1024] = np.arctan2(det, den).sum(1) / (2 * np.pi)
    inside = (wn > 0.5).reshape(tuple(shape))
    MESHES.mkdir(exist_ok=True)
    np.savez_compressed(MESHES / "bunny_grid.npz", lo=lo, h=np.array(h), shape=shape, inside=inside,
                        surface_vertices=np.array(len(V)), surface_faces=np.array(len(F)))
    print("bunny grid", tuple(shape), "inside vertices", int(inside.sum()))


def delaunay_sha():
    """delaunay_sha.json: sha256 of the unstructured Delaunay systems' A (problems.delaunay_heat: qhull
    + elementwise numpy only) as this container builds them, so a GPU box whose qhull / numpy gave a
    different mesh or different bits fails loudly instead of comparing against the wrong system."""
    import json

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset

    out = {}
    for name in ("delaunay20k", "delaunay1m"):
        A, mask, _, _, _ = P.workload(name)
        lens = np.diff(A.indptr)
        out[name] = {"n": int(A.shape[0]), "nnz": int(A.nnz), "A_sha256": P.matrix_sha256(A),
                     "dirichlet": int((np.asarray(mask) == 0).sum()),
                     "row_entries": [int(lens.min()), float(lens.mean()), int(lens.max())]}
        print(name, out[name], flush=True)
    rows = []
    for smp in synthetic_dataset("delaunay_batch8"):
        rows.append({"n": int(smp.num_nodes), "E": int(smp.edge_index.shape[1]),
                     "values_sha256": _sha(smp.matrix_values.numpy(), smp.edge_index.numpy())})
    out["delaunay_batch8"] = rows
    print("delaunay_batch8", [r["n"] for r in rows], flush=True)
    (OUT / "delaunay_sha.json").write_text(json.dumps(out, indent=1) + "\n")


def main():
    install_shims()
    if sys.argv[1:] == ["bunny"]:
        bunny_grid()
        return
    if sys.argv[1:] == ["delaunay"]:
        sys.path.insert(0, str(ROOT))
        delaunay_sha()
        return
    if sys.argv[1:] == ["traj"]:
        from neural_cg.utils import validate as rval

        sys.path.insert(0, str(ROOT))
        traj_fixtures(rval)
        return
    if sys.argv[1:2] == ["headline"]:  # headline <workload> <boo .npy from tools/dump_gnn_l.py>
        from neural_cg.utils import validate as rval

        sys.path.insert(0, str(ROOT))
        headline_fixtures(rval, sys.argv[2], sys.argv[3])
        return
    if sys.argv[1:2] == ["batch"]:  # batch <dataset> <dir of tools/dump_gnn_l.py --dataset output>
        from neural_cg.utils import validate as rval

        sys.path.insert(0, str(ROOT))
        batch_fixtures(rval, sys.argv[2], sys.argv[3])
        return
    if sys.argv[1:2] == ["refgnn"]:  # refgnn <workload> <boo .npy from tools/dump_gnn_l.py>
        from neural_cg import data as rdata
        from neural_cg.nn import gnns as rgnn
        from neural_cg.utils import validate as rval

        sys.path.insert(0, str(ROOT))
        headline_refgnn_fixtures(rdata, rgnn, rval, sys.argv[2], sys.argv[3])
        return
    if sys.argv[1:] == ["infer"]:
        from neural_cg import data as rdata
        from neural_cg.nn import gnns as rgnn
        from neural_cg.utils import validate as rval

        sys.path.insert(0, str(ROOT))
        infer_fixtures(rdata, rgnn, rval)
        return
    if sys.argv[1:] == ["ichol"]:
        from neural_cg.utils import validate as rval

        sys.path.insert(0, str(ROOT))
        ichol_fixtures(rval)
        return
    if sys.argv[1:] == ["gnn"]:
        from neural_cg import data as rdata
        from neural_cg.nn import basic_layers as rbl
        from neural_cg.nn import gnns as rgnn

        sys.path.insert(0, str(ROOT))
        gnn_forward_fixtures(rdata, rgnn)
        graph_spmv_fixtures(rbl)
        return
    from neural_cg import data as rdata
    from neural_cg.nn import gnns as rgnn
    from neural_cg.utils import validate as rval

    sys.path.insert(0, str(ROOT))
    from learningsparsepreconditioner4gpu_amd import problems as P

    rng = np.random.default_rng(2024)
    # ---------------- to_csr_cpu
    cases = {}
    A, mask, _ = P.poisson2d_grid(9, 7)
    g = P.to_block_graph(A, 1)
    cases["poisson_masked_f32in"] = (g.edge_index, g.block_values.astype(np.float32), A.shape[0], mask)
    cases["poisson_nomask"] = (g.edge_index, g.block_values, A.shape[0], None)
    Ae, me, _ = P.elasticity_box(4, 3, 3)
    ge = P.to_block_graph(Ae, 3)
    vals = ge.block_values.copy()
    vals[rng.random(vals.shape) < 0.1] = 0.0
    cases["elast_b3_masked"] = (ge.edge_index, vals.astype(np.float32), Ae.shape[0], me)
    K = P.kuhn_laplacian(4)
    K = sp.csr_matrix(K - sp.diags(K.diagonal()))
    K.eliminate_zeros()
    gk = P.to_block_graph(K, 1)
    mk = (rng.random((K.shape[0], 1)) > 0.3).astype(np.float64)
    cases["kuhn_nodiag_masked"] = (gk.edge_index, gk.block_values, K.shape[0], mk)
    out = {}
    for name, (ei, ea, n, m) in cases.items():
        csr = rval.to_csr_cpu(torch.from_numpy(ei), torch.from_numpy(ea), n,
                              None if m is None else torch.from_numpy(m), dtype=np.float64)
        out[f"{name}__edge_index"] = ei
        out[f"{name}__edge_attr"] = ea
        out[f"{name}__n"] = np.array(n)
        out[f"{name}__mask"] = np.zeros(0) if m is None else m
        out[f"{name}__indptr"] = csr.indptr
        out[f"{name}__indices"] = csr.indices
        out[f"{name}__data"] = csr.data
    np.savez_compressed(OUT / "to_csr.npz", **out)

    # ---------------- synthetic generator
    gen = reference_synthetic()
    S = sp.csr_matrix(gen(512, 3e-3, 1e-5, np.random.RandomState(7)))
    S.sort_indices()
    np.savez_compressed(OUT / "synthetic.npz", indptr=S.indptr, indices=S.indices, data=S.data, n=512,
                        sparsity=3e-3, amp=1e-5, seed=7)

    # ---------------- PCG iteration counts (scipy restatements in validate.py)
    pc = {}
    systems = {
        "synthetic600": (sp.csr_matrix(gen(600, 8e-3, 1e-3, np.random.RandomState(11))), None),
        "poisson16": P.poisson2d_grid(16, 16)[:2],
        "kuhn7": (P.kuhn_laplacian(7), None),
    }
    for name, (A, mask) in systems.items():
        A = sp.csr_matrix(A)
        A.sort_indices()
        n = A.shape[0]
        gt = np.ones(n) if mask is None else mask.ravel().astype(np.float64)
        Lr = np.random.default_rng(5)
        L = A.copy()
        rows = np.repeat(np.arange(n), np.diff(A.indptr))
        d = np.abs(A.diagonal()) + 1e-12
        L.data = Lr.normal(size=A.nnz) * 0.05 / np.sqrt(d[rows])
        dg = rows == A.indices
        L.data[dg] = 1.0 / np.sqrt(d[rows[dg]])
        eps = 3e-3
        pc[f"{name}__indptr"], pc[f"{name}__indices"], pc[f"{name}__data"] = A.indptr, A.indices, A.data
        pc[f"{name}__L_data"] = L.data
        pc[f"{name}__gt"] = gt
        pc[f"{name}__eps"] = np.array(eps)
        for rtol in (1e-6, 1e-8):
            tag = f"{name}__rtol{int(-np.log10(rtol))}"
            pc[f"{tag}__none"] = np.array(rval.get_cg_iter_time_scipy(A, gt, rtol=rtol))
            pc[f"{tag}__diagonal"] = np.array(rval.get_pcg_diagonal_iter_time_scipy(A, gt, rtol=rtol))
            pc[f"{tag}__ext_spai"] = np.array(rval.get_pcg_iter_time_scipy(A, gt, L, eps, rtol=rtol))
            pc[f"{tag}__ext_spai_scaled"] = np.array(rval.get_pcg_scaled_iter_time_scipy(A, gt, L, eps, rtol=rtol))
    np.savez_compressed(OUT / "pcg_counts.npz", **pc)

    # ---------------- GNN construction / seeded init (config/gnn.yaml)
    ff = lambda norm: {"pre_norm": norm, "hidden_channels": 16, "num_layers": 2}
    cfg = dict(node_encoder=ff("none"), edge_encoder=ff("none"), node_decoder=ff("none"), edge_decoder=ff("none"),
               num_mp_layers=4, node_residual=True, edge_residual=True, node_features=16, edge_features=16,
               node_mlp=ff("layer"), edge_mlp=ff("layer"), msg_mlp=ff("layer"), msg_norm=True, aggr="add")
    torch.manual_seed(0)
    net = rgnn.NodeEdgeProcessing(node_in_features=4, node_out_features=None, edge_in_features=9,
                                  edge_out_features=9, **cfg)
    np.savez_compressed(OUT / "gnn_init.npz", **{k: v.detach().numpy() for k, v in net.state_dict().items()})

    # ---------------- make_data (data.py:218-336), 'disable' edge->node aggregation
    Ab, mb, nodes = P.elasticity_box(4, 3, 3)
    gb = P.to_block_graph(Ab, 3)
    raw = rdata.RawData(block_values=gb.block_values, diagonals=Ab.diagonal().reshape(-1, 3),
                        edge_index=gb.edge_index, node_features=nodes, lhs=None, rhs=None, mask=mb,
                        num_nodes=gb.num_nodes, block_size=3)
    dd = rdata.make_data(raw, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                         use_node_features_as_edge_feature=False, use_edge_features_as_node_feature="disable",
                         use_random_rhs=True, normalize_matrix="mean", is_inference=True)
    np.savez_compressed(OUT / "make_data.npz", A_indptr=Ab.indptr, A_indices=Ab.indices, A_data=Ab.data, mask=mb,
                        nodes=nodes, x=dd.x.numpy(), edge_index=dd.edge_index.numpy(), edge_attr=dd.edge_attr.numpy(),
                        matrix_values=dd.matrix_values.numpy(), rsqrt_diag=dd.rsqrt_diag.numpy(),
                        inv_diag=dd.inv_diag.numpy(), mask_out=dd.mask.numpy())
    # ---------------- FolderDataset (data.py:339-640) on two folders written in the datagen format
    import shutil

    from learningsparsepreconditioner4gpu_amd.dataset import FolderWriter

    fx = {}
    free, fixed = OUT / "folder_free", OUT / "folder_fixed"
    for d in (free, fixed):
        shutil.rmtree(d, ignore_errors=True)
    w = FolderWriter(str(free), block_size=1, save_rhs=2, save_lhs=True, seed=3)
    for k in range(2):
        Af, mf, _ = P.poisson2d_grid(6 + k, 5)
        w.append(Af * (1.0 + k), mf, rng.random((Af.shape[0], 2)))
    Ab, mb, nodes = P.elasticity_box(3, 2, 2)
    # (bs > 1: the reference's rhs files hold one entry per block row and no lhs can be solved
    # for them -- datagen_helper.py:300-321 -- so this folder samples a random rhs instead)
    w = FolderWriter(str(fixed), block_size=3, is_fixed_topology=True, save_rhs=1, save_lhs=False, seed=4)
    w.write_topology(Ab)
    w.write_shared(nodes)
    for k in range(2):
        Ak = sp.csr_matrix(Ab * (1.0 + 0.5 * k))
        w.append(Ak, mb, rng.random((Ab.shape[0] // 3, 2)), rhs=rng.standard_normal(Ab.shape[0] // 3))
    configs = {
        "free": dict(is_fixed_topology=False, load_into_memory=True, block_size=1, has_shared_features=False,
                     use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                     use_node_features_as_edge_feature=False, use_edge_features_as_node_feature="disable",
                     use_random_rhs=False, normalize_matrix="mean", prefix=str(free)),
        "fixed": dict(is_fixed_topology=True, load_into_memory=False, block_size=3, has_shared_features=True,
                      use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                      use_node_features_as_edge_feature=True, use_edge_features_as_node_feature="disable",
                      use_random_rhs=True, normalize_matrix="frob", prefix=str(fixed)),
        "free_l1": dict(is_fixed_topology=False, load_into_memory=False, block_size=1, has_shared_features=False,
                        use_node_features=True, use_matrix_as_edge_feature=True, use_mask_as_node_feature=False,
                        use_node_features_as_edge_feature=True, use_edge_features_as_node_feature="disable",
                        use_random_rhs=False, normalize_matrix="l1", prefix=str(free)),
    }
    for name, cfg in configs.items():
        ds = rdata.FolderDataset(**cfg)
        fx[f"{name}__len"] = np.array(ds.len())
        fx[f"{name}__nnf"] = np.array(ds.num_node_features)
        fx[f"{name}__nef"] = np.array(ds.num_edge_features)
        for i in range(ds.len()):
            torch.manual_seed(100 + i)  # the random rhs (data.py:318) draws from torch's generator
            dd = ds.get(i)
            for key in ("x", "edge_index", "edge_attr", "mask", "matrix_values", "diagonal", "inv_diag",
                        "rsqrt_diag", "gt", "residual"):
                if hasattr(dd, key):
                    fx[f"{name}__{i}__{key}"] = getattr(dd, key).numpy()
    np.savez_compressed(OUT / "folder.npz", **fx)

    from neural_cg.nn import basic_layers as rbl

    gnn_forward_fixtures(rdata, rgnn)
    graph_spmv_fixtures(rbl)
    ichol_fixtures(rval)
    infer_fixtures(rdata, rgnn, rval)

    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
