"""Inference driver: GNN -> SPAI -> PCG per sample, Timestat + CSVs (infer.py of the reference).

Mirrors ``/root/reference/infer.py``: warm-up of the GNN (:270-275), per sample the
preconditioner time averaged over ``repeat`` inference steps (:288-293), rhs = mask /
random / neighbour (:297-307), the Neural PCG row (:322-331) and the two CSVs with the
reference schema (:372-384: ``Key, Total Time (ms), Solve Time (ms), Precond Time (ms),
#Iteration`` and the per-sample ``all_*`` file with ``Matrix Size``), with the reference's row
keys: the GPU PCG row is ``Neural+CUDA`` (:331; the reference's consumers key on it,
misc/plot_bars.py:54-55, misc/tab_to_latex.py:79-126; ``--hip-key`` writes ``Neural+HIP``
instead) and the GPU baselines are ``PCG-{none,diagonal,ainv,ic}-cuda`` (:310-321).  The host
rows ``Neural`` (:330) and ``PCG-{none,diagonal}-cpu`` come with ``--cpu-rows`` from the
reference's own scipy restatement (cpu_rows.py; pymathprim's CPU backend is absent, and so
are ``PCG-{ainv,ic}-cpu``).  Differences kept on purpose: ``Neural+CUDA`` carries the GPU
solve's own count (the reference copies the CPU run's, :330-331) and ``Precond Time`` is the
GNN time (the reference overwrites it with the last baseline's setup time).
``--dot-order openblas --dot-threads T`` runs every GPU row in parity mode (the reference's
recorded scipy trajectories, T OpenBLAS threads).  Samples are sharded one-per-GPU under
torchrun (``distributed.run_sharded``) with a single all-gather at the end.

    python -m learningsparsepreconditioner4gpu_amd.infer --dataset heat_batch8 --rtol 1e-8
    torchrun --nproc-per-node 8 -m learningsparsepreconditioner4gpu_amd.infer --dataset heat_batch8
"""
from __future__ import annotations

import argparse
import math
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import problems as P
from .data import GraphSample, make_sample
from .distributed import SolveRecord, run_sharded, run_sharded_batched, run_sharded_concurrent
from .validate import get_cg_iter_time, get_pcg_iter_time, get_pcg_iter_time_batch, get_pcg_scaled_iter_time
from .workspace import ScaledInferenceWorkspace, SimpleInferenceWorkspace


@dataclass
class InferenceTimestat:
    all_solve_time: List[float] = field(default_factory=list)
    all_prec_time: List[float] = field(default_factory=list)
    all_iteration: List[float] = field(default_factory=list)
    all_matrix_size: List[int] = field(default_factory=list)


class Timestat:
    """infer.py:38-151 (same keys, same CSV columns)."""

    def __init__(self):
        self.stat_dict: Dict[str, InferenceTimestat] = {}

    def put(self, key: str, solve_time: float, prec_time: float, iteration: float, matrix_size: int):
        s = self.stat_dict.setdefault(key, InferenceTimestat())
        s.all_solve_time.append(solve_time)
        s.all_prec_time.append(prec_time)
        s.all_iteration.append(iteration)
        s.all_matrix_size.append(matrix_size)

    def timestat_to_dataframe(self):
        import pandas as pd

        rows = []
        for key, st in self.stat_dict.items():
            sol = np.mean(st.all_solve_time) * 1000
            pre = np.mean(st.all_prec_time) * 1000
            rows.append({"Key": key, "Total Time (ms)": sol + pre, "Solve Time (ms)": sol, "Precond Time (ms)": pre,
                         "#Iteration": np.mean(st.all_iteration)})
        df = pd.DataFrame(rows)
        cols = ["Total Time (ms)", "Solve Time (ms)", "Precond Time (ms)", "#Iteration"]
        if len(df):
            df[cols] = df[cols].round(4)
        return df

    def all_time_stat(self):
        import pandas as pd

        rows = []
        for key, st in self.stat_dict.items():
            for s, p, i, m in zip(st.all_solve_time, st.all_prec_time, st.all_iteration, st.all_matrix_size):
                rows.append({"Key": key, "Solve Time (ms)": s * 1000, "Precond Time (ms)": p * 1000, "#Iteration": i,
                             "Matrix Size": m})
        df = pd.DataFrame(rows)
        cols = ["Solve Time (ms)", "Precond Time (ms)", "#Iteration", "Matrix Size"]
        if len(df):
            df[cols] = df[cols].round(4)
        return df

    def print(self):
        for key, st in self.stat_dict.items():
            print(f"{key}: solve {np.mean(st.all_solve_time) * 1e3:.2f} ms, precond "
                  f"{np.mean(st.all_prec_time) * 1e3:.2f} ms, {np.mean(st.all_iteration):.4f} it/sample")


def synthetic_dataset(name: str) -> List[GraphSample]:
    """Stand-in datasets; the reference's generated/ folders are absent."""
    if name == "heat_batch8":  # C5: 8 heat-tet systems, 400-32000 vertices, seeds 0-7
        rng = np.random.default_rng(0)
        out = []
        for s in range(8):
            nv = int(rng.integers(400, 32000))
            k = max(4, int(round(nv ** (1 / 3))))
            A, mask, feats = P.heat_tet(k, k, max(4, nv // (k * k)), rho=float(rng.uniform(1e-4, 5e-4)), seed=s)
            out.append(make_sample(A, mask, node_features=feats))
        return out
    if name == "delaunay_batch8":  # C5 on unstructured Delaunay tet meshes: 8 systems, 400-32000 vertices
        rng = np.random.default_rng(0)
        out = []
        for s in range(8):
            A, mask, nodes = P.delaunay_heat(int(rng.integers(400, 32000)), seed=s)
            out.append(make_sample(A, mask, node_features=nodes))
        return out
    if name == "heat_bunny":  # C3: heat on the voxelised bunny, F_in = 5 (field, xyz, mask)
        A, mask, feats = P.heat_bunny()
        return [make_sample(A, mask, node_features=feats)]
    if name.startswith("poisson"):
        A, mask, _ = P.poisson2d_grid(256, 256)
        return [make_sample(A, mask)]
    if name.startswith("synthetic"):
        return [make_sample(P.synthetic_c1(), None, use_edge_features_as_node_feature="mean")]
    if name.startswith("kuhn"):
        A, mask = P.kuhn_dirichlet(int(name[4:] or 101))
        return [make_sample(A, mask)]
    raise KeyError(name)


def folder_dataset(prefix: str, block_size: int = 1, fixed_topology: bool = False, shared_features: bool = False,
                   node_features: bool = True, edge_to_node: str = "disable", normalize="mean") -> List[GraphSample]:
    """Samples of an on-disk dataset (dataset.FolderDataset, data.py:339-640; config/data.yaml
    defaults), one per rhs column like the reference's dataloader."""
    from .dataset import FolderDataset

    ds = FolderDataset(is_fixed_topology=fixed_topology, load_into_memory=False, block_size=block_size,
                       has_shared_features=shared_features, use_node_features=node_features,
                       use_matrix_as_edge_feature=True, use_mask_as_node_feature=True,
                       use_node_features_as_edge_feature=False, use_edge_features_as_node_feature=edge_to_node,
                       use_random_rhs=True, normalize_matrix=normalize, prefix=prefix)
    return [ds.get(i, is_inference=True) for i in range(ds.len())]


def rhs_for(rhs: str, mask: np.ndarray, sample: Optional[GraphSample] = None,
            rng: Optional[np.random.Generator] = None) -> np.ndarray:
    """infer.py:297-309: mask / ones, random (masked), neighbour (A_full (1-m) + 0.1 m, masked).
    ``random`` draws from ``rng`` when given (main passes one seeded per sample, so every rank
    draws the same vector for a sample), else from numpy's global generator like the reference."""
    m = mask.reshape(-1).astype(np.float64)
    if rhs in ("mask", "ones"):
        return m
    if rhs == "random":
        return (rng.standard_normal(m.size) if rng is not None else np.random.randn(m.size)) * m
    if rhs == "neighbour":
        from .validate import to_csr_cpu

        n = m.size
        A_full = to_csr_cpu(sample.edge_index, sample.matrix_values, n, None)
        A_full.data.fill(1.0)
        return (A_full @ (1 - m) + 0.1 * m) * m
    raise ValueError(f"Unknown rhs type: {rhs}")


def _rhs(rhs: str, i: int, s: GraphSample, rhs_vectors: Optional[Dict[int, np.ndarray]]) -> np.ndarray:
    """Sample i's right-hand side: the shared one when given (infer.py:296-307 builds r once per
    sample and solves every row with it), else rhs_for."""
    if rhs_vectors is not None:
        return rhs_vectors[i]
    return rhs_for(rhs, s.mask.cpu().numpy(), s)


def run(samples: Sequence[GraphSample], ws: SimpleInferenceWorkspace, rtol: float = 1e-6, repeat: int = 1,
        rhs: str = "mask", warmup: int = 20, concurrency: int = 1, batch: int = 1, dot_order: str = "compensated",
        dot_threads: int = 1, rhs_vectors: Optional[Dict[int, np.ndarray]] = None) -> List[SolveRecord]:
    """The ``Neural+CUDA`` row of infer.py:278-331 (GNN -> L, A; ext_spai PCG).  ``concurrency``
    > 1 keeps that many solves of this rank in flight at once (run_sharded_concurrent): the same
    iterates and counts, a higher batch throughput on the reference's mid-size systems.  ``batch``
    > 1 (ext_spai, not the scaled variant) solves this rank's systems in lockstep windows of that
    many (run_sharded_batched, validate.get_pcg_iter_time_batch) after ONE GNN forward over the
    window's graphs (workspace.inference_step_batch): the same L, counts and iterates, every launch
    covering the whole window; a record's t_prec / t_solve are its shares of the window's forward
    / device solve time.  ``dot_order`` / ``dot_threads``: the loop's dot order (``"openblas"`` =
    parity mode; not with ``batch`` > 1, whose lockstep schedule has the compensated order only)."""
    if batch > 1 and dot_order != "compensated":
        raise ValueError("batch > 1 runs the compensated dot order only; use batch=1 for dot_order='openblas'")
    pcg = get_pcg_scaled_iter_time if isinstance(ws, ScaledInferenceWorkspace) else get_pcg_iter_time
    dev = torch.device("cuda", torch.cuda.current_device())
    warmed = set()

    def prepare(i: int):
        s = samples[i].to(dev)
        if not warmed:
            for _ in range(warmup):
                ws.inference_step(s)
            warmed.add(True)
        prec = 0.0
        for _ in range(repeat):
            _, dt = ws.inference_step(s)
            prec += dt
        prec /= repeat
        L, _ = ws.inference_step(s)
        A = ws.system_matrix(s)
        r = _rhs(rhs, i, s, rhs_vectors)
        return i, A, L, r, prec

    def finish(job) -> SolveRecord:
        i, A, L, r, prec = job
        info = {}
        it, _, sol = pcg(A, r, L, ws.epsilon, rtol=rtol, repeat=repeat, device="cuda", info=info,
                         dot_order=dot_order, dot_threads=dot_threads)
        # the true ‖b − A x‖/‖b‖ of the solution (one device SpMV) and the solver's own verdict
        return SolveRecord(index=i, iters=it, rel_res=info["rel_res"], t_prec=prec, t_solve=sol, n=A.n, nnz=A.nnz,
                           converged=info["converged"])

    def finish_batch(jobs) -> List[SolveRecord]:
        infos = [{} for _ in jobs]
        out = get_pcg_iter_time_batch([j[1] for j in jobs], [j[3] for j in jobs], [j[2] for j in jobs], ws.epsilon,
                                      rtol=rtol, infos=infos, repeat=repeat)
        return [SolveRecord(index=j[0], iters=it, rel_res=info["rel_res"], t_prec=j[4], t_solve=sol, n=j[1].n,
                            nnz=j[1].nnz, converged=info["converged"]) for j, (it, _, sol), info in zip(jobs, out, infos)]

    def prepare_batch(items):
        # one GNN forward over the window's graphs (inference_step_batch: the same L bits); each
        # record's t_prec is its share of the window's forward
        ss = [samples[i].to(dev) for i in items]
        if not warmed:
            for _ in range(warmup):
                ws.inference_step_batch(ss)
            warmed.add(True)
        prec = 0.0
        for _ in range(repeat):
            _, dt = ws.inference_step_batch(ss)
            prec += dt
        prec /= repeat * len(items)
        Ls, _ = ws.inference_step_batch(ss)
        return [(i, ws.system_matrix(s), L, _rhs(rhs, i, s, rhs_vectors), prec)
                for i, s, L in zip(items, ss, Ls)]

    weights = [float(s.edge_index.shape[1]) for s in samples]
    if batch > 1 and not isinstance(ws, ScaledInferenceWorkspace):
        return run_sharded_batched(len(samples), weights, prepare, finish_batch, batch, prepare_batch=prepare_batch)
    if concurrency > 1:
        return run_sharded_concurrent(len(samples), weights, prepare, finish, concurrency)
    return run_sharded(len(samples), weights, lambda i: finish(prepare(i)))


def run_baseline(samples: Sequence[GraphSample], ws: SimpleInferenceWorkspace, method: str, rtol: float = 1e-6,
                 repeat: int = 1, rhs: str = "mask", dot_order: str = "compensated",
                 dot_threads: int = 1, rhs_vectors: Optional[Dict[int, np.ndarray]] = None) -> List[SolveRecord]:
    """The ``PCG-{method}-cuda`` rows (infer.py:310-321: get_cg_iter_time with method none /
    diagonal / ainv / ic on the same A and rhs).  A non-converged solve raises RuntimeError in
    the reference (caught at :363); here its row is NaN and left out of the statistics."""
    dev = torch.device("cuda", torch.cuda.current_device())

    def solve(i: int) -> SolveRecord:
        s = samples[i].to(dev)
        A = ws.system_matrix(s)
        r = _rhs(rhs, i, s, rhs_vectors)
        info = {}
        try:
            it, prec, sol = get_cg_iter_time(A, r, rtol=rtol, repeat=repeat, method=method, device="cuda",
                                             info=info, dot_order=dot_order, dot_threads=dot_threads)
        except RuntimeError:
            return SolveRecord(index=i, iters=float("nan"), rel_res=float("nan"), t_prec=float("nan"),
                               t_solve=float("nan"), n=A.n, nnz=A.nnz, converged=False)
        return SolveRecord(index=i, iters=it, rel_res=info["rel_res"], t_prec=prec, t_solve=sol, n=A.n, nnz=A.nnz,
                           converged=info["converged"])

    weights = [float(s.edge_index.shape[1]) for s in samples]
    return run_sharded(len(samples), weights, solve)


def run_cpu_rows(samples: Sequence[GraphSample], ws: SimpleInferenceWorkspace, rtol: float = 1e-6, repeat: int = 1,
                 rhs: str = "mask", methods: Sequence[str] = ("none", "diagonal"),
                 threads: Optional[int] = None,
                 rhs_vectors: Optional[Dict[int, np.ndarray]] = None) -> Dict[str, List[SolveRecord]]:
    """The reference's host rows (infer.py:310-330 with device="cpu"): ``Neural`` (ext_spai or its
    scaled variant on the host copies of A and of the GNN's L) and ``PCG-{method}-cpu`` for
    ``methods`` (none / diagonal), each from cpu_rows (the reference's scipy restatement; its
    pymathprim CPU backend is absent).  The GNN and the assembly run on the GPU as for the GPU
    rows; ``Precond Time`` is the GNN time for ``Neural`` and 0 for the baselines (no setup).
    A baseline that reaches max_iter is left out, as the reference's RuntimeError does (:363)."""
    from . import cpu_rows

    dev = torch.device("cuda", torch.cuda.current_device())
    scaled = isinstance(ws, ScaledInferenceWorkspace)

    def solve(i: int):
        s = samples[i].to(dev)
        prec = 0.0
        for _ in range(repeat):
            _, dt = ws.inference_step(s)
            prec += dt
        prec /= repeat
        L, _ = ws.inference_step(s)
        A = ws.system_matrix(s)
        Ah, Lh = A.to_scipy().tocsr(), L.to_scipy().tocsr()
        r = _rhs(rhs, i, s, rhs_vectors)
        it, sol = cpu_rows.neural_row(Ah, r, Lh, ws.epsilon, rtol, scaled=scaled, repeat=repeat, threads=threads)
        recs = [SolveRecord(index=i, iters=it, rel_res=float("nan"), t_prec=prec, t_solve=sol, n=A.n, nnz=A.nnz,
                            converged=it < A.n)]
        for m in methods:
            try:
                it, sol = cpu_rows.baseline_row(Ah, r, m, rtol, repeat=repeat, threads=threads)
                recs.append(SolveRecord(index=i, iters=it, rel_res=float("nan"), t_prec=0.0, t_solve=sol, n=A.n,
                                        nnz=A.nnz, converged=True))
            except RuntimeError:
                recs.append(SolveRecord(index=i, iters=float("nan"), rel_res=float("nan"), t_prec=float("nan"),
                                        t_solve=float("nan"), n=A.n, nnz=A.nnz, converged=False))
        return recs

    per = {}
    for i in range(len(samples)):  # host rows: the rank-0 process's host, one sample at a time
        per[i] = solve(i)
    out = {"Neural": [per[i][0] for i in sorted(per)]}
    for k, m in enumerate(methods):
        out[f"PCG-{m}-cpu"] = [per[i][k + 1] for i in sorted(per)]
    return out


def reference_quirks(rows: Dict[str, List[SolveRecord]], neural_key: str, baselines: Sequence[str]):
    """The reference's row bookkeeping, bit for bit (opt-in ``--reference-quirks``).  In
    infer.py:310-331 the name ``prec`` is rebound by every baseline call, so both Neural rows are
    put with the LAST baseline's setup time (``PCG-ic-cuda`` in its row order), not the GNN time of
    :287-291; and ``Neural+CUDA`` is put with ``it`` of the CPU ``Neural`` row (:330-331), not its
    own count.  By default this package records each row's own values."""
    from dataclasses import replace

    out = dict(rows)
    last = out.get(f"PCG-{baselines[-1]}-cuda") if baselines else None
    prec = {r.index: r.t_prec for r in last} if last else {}
    host = {r.index: r.iters for r in out.get("Neural", [])}
    for k in (neural_key, "Neural"):
        if k in out:
            out[k] = [replace(r, t_prec=prec.get(r.index, r.t_prec),
                              iters=host.get(r.index, r.iters) if k == neural_key else r.iters) for r in out[k]]
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="heat_batch8")
    ap.add_argument("--folder", default="", help="on-disk dataset (datagen folder format); overrides --dataset")
    ap.add_argument("--block-size", type=int, default=1)
    ap.add_argument("--fixed-topology", action="store_true")
    ap.add_argument("--shared-features", action="store_true")
    ap.add_argument("--no-node-features", action="store_true")
    ap.add_argument("--edge-to-node", default="disable", choices=["disable", "sum", "mean", "max", "min"])
    ap.add_argument("--normalize", default="mean")
    ap.add_argument("--exp-name", default=None)
    ap.add_argument("--rtol", type=float, default=1e-6)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--rhs", default="mask")
    ap.add_argument("--rhs-seed", type=int, default=0, help="rhs=random: sample i draws from default_rng(seed + i)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workspace", default="simple", choices=["simple", "scaled"])
    ap.add_argument("--pretrained", default="")
    ap.add_argument("--epsilon", type=float, default=3e-3)
    ap.add_argument("--out-dir", default="output")
    ap.add_argument("--infer-prefix", default="")
    ap.add_argument("--concurrency", type=int, default=1,
                    help="solves in flight at once per GPU (run_sharded_concurrent); 1 = the reference's sequential loop")
    ap.add_argument("--batch", type=int, default=1,
                    help="systems per lockstep batch per GPU (run_sharded_batched); 1 = one solve at a time")
    ap.add_argument("--baselines", default="none,diagonal,ainv,ic",
                    help="comma list of PCG-{method}-cuda rows (infer.py:310-321); '' for none")
    ap.add_argument("--dot-order", default="compensated", choices=["compensated", "openblas"],
                    help="dot order of every GPU row: openblas = parity mode (the reference's scipy trajectories)")
    ap.add_argument("--dot-threads", type=int, default=1,
                    help="OpenBLAS threads of the parity order (numpy splits dots of n > 10,000 over them)")
    ap.add_argument("--hip-key", action="store_true", help="key the GPU PCG row Neural+HIP instead of Neural+CUDA")
    ap.add_argument("--cpu-rows", action="store_true",
                    help="also write the reference's host rows Neural and PCG-{none,diagonal}-cpu (scipy restatement)")
    ap.add_argument("--cpu-threads", type=int, default=None, help="BLAS threads of the host rows (default: process)")
    ap.add_argument("--reference-quirks", action="store_true",
                    help="reproduce infer.py:318,330-331 in the CSVs: the Neural rows' Precond Time is the last "
                         "baseline row's setup time and Neural+CUDA carries the host Neural row's count")
    args = ap.parse_args(argv)

    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per local rank; more ranks than GPUs (a gloo rehearsal on one GPU) share them
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        # RCCL over xGMI; LSPCG_DIST_BACKEND=gloo rehearses several ranks on ONE GPU (RCCL refuses that)
        backend = os.environ.get("LSPCG_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": torch.device("cuda", local)} if backend == "nccl" else {}))
    if args.folder:
        samples = folder_dataset(args.folder, args.block_size, args.fixed_topology, args.shared_features,
                                 not args.no_node_features, args.edge_to_node, args.normalize)
    else:
        samples = synthetic_dataset(args.dataset)
    cls = ScaledInferenceWorkspace if args.workspace == "scaled" else SimpleInferenceWorkspace
    if args.pretrained:
        ws = cls.load_from_checkpoint(args.pretrained)
    else:
        s0 = samples[0]
        ws = cls(node_features=s0.x.shape[1], edge_features=s0.edge_attr.shape[1], block_size=s0.block_size,
                 epsilon=args.epsilon, seed=0)
    rows = {}
    dots = dict(dot_order=args.dot_order, dot_threads=args.dot_threads)
    # one right-hand side per sample, shared by every row (infer.py:296-307); only "random" draws,
    # from a generator seeded by the sample index: under torchrun the owning rank's GPU rows and
    # rank 0's host rows then solve the SAME vector for a sample
    rhs_vectors = ({i: rhs_for(args.rhs, s.mask.numpy(), s, rng=np.random.default_rng(args.rhs_seed + i))
                    for i, s in enumerate(samples)} if args.rhs == "random" else None)
    for m in [b for b in args.baselines.split(",") if b]:
        rows[f"PCG-{m}-cuda"] = run_baseline(samples, ws, m, rtol=args.rtol, repeat=args.repeat, rhs=args.rhs,
                                             rhs_vectors=rhs_vectors, **dots)
    key = "Neural+HIP" if args.hip_key else "Neural+CUDA"
    rows[key] = run(samples, ws, rtol=args.rtol, repeat=args.repeat, rhs=args.rhs, warmup=args.warmup,
                    concurrency=args.concurrency, batch=args.batch, rhs_vectors=rhs_vectors, **dots)
    recs = rows[key]
    if args.cpu_rows and (not dist.is_initialized() or dist.get_rank() == 0):
        rows.update(run_cpu_rows(samples, ws, rtol=args.rtol, repeat=args.repeat, rhs=args.rhs,
                                 threads=args.cpu_threads, rhs_vectors=rhs_vectors))
    if args.reference_quirks:
        rows = reference_quirks(rows, key, [b for b in args.baselines.split(",") if b])
    if not dist.is_initialized() or dist.get_rank() == 0:
        stats = Timestat()
        for key, rs in rows.items():
            for r in rs:
                if r.iters == r.iters:  # NaN = not converged (reference: RuntimeError, row skipped)
                    stats.put(key, r.t_solve, r.t_prec, r.iters, r.n)
        stats.print()
        out = Path(args.out_dir)
        out.mkdir(parents=True, exist_ok=True)
        exp = args.exp_name or (Path(args.folder).name if args.folder else args.dataset)
        log_rtol = -int(math.log10(args.rtol))
        stats.timestat_to_dataframe().to_csv(out / f"infer_{args.infer_prefix}{exp}_{log_rtol}.csv", index=False)
        stats.all_time_stat().to_csv(out / f"all_infer_{args.infer_prefix}{exp}_{log_rtol}.csv", index=False)
    if dist.is_initialized():
        dist.destroy_process_group()
    return recs


if __name__ == "__main__":
    main()
