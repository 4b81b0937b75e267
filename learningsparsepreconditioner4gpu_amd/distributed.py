"""Independent systems sharded one-per-GPU.

Each rank (one process per GPU, torchrun) solves its own subset of a batch of independent
systems -- there is no data-path collective.  At the end ONE all-gather of a small fixed
record per system (RCCL over xGMI with backend "nccl", or gloo on CPU for tests) brings
every rank's results to every rank.  Assignment is longest-processing-time-first by a work
estimate (nnz), so unequal systems (the heat-tetmesh dataset: 400-32000 vertices) balance.
"""
from __future__ import annotations

import heapq
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

FIELDS = ("index", "iters", "rel_res", "t_prec", "t_solve", "n", "nnz", "converged")


@dataclass
class SolveRecord:
    index: int
    iters: float
    rel_res: float
    t_prec: float
    t_solve: float
    n: int
    nnz: int
    converged: bool = True

    def as_list(self):
        return [float(self.index), float(self.iters), float(self.rel_res), float(self.t_prec), float(self.t_solve),
                float(self.n), float(self.nnz), float(self.converged)]

    @classmethod
    def from_list(cls, v):
        return cls(int(v[0]), float(v[1]), float(v[2]), float(v[3]), float(v[4]), int(v[5]), int(v[6]), bool(v[7]))


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def lpt_assign(weights: Sequence[float], world: int) -> List[List[int]]:
    """Longest-processing-time-first: heaviest item to the least loaded rank (ties -> lower rank)."""
    order = sorted(range(len(weights)), key=lambda i: (-float(weights[i]), i))
    heap = [(0.0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + float(weights[i]), r))
    return [sorted(v) for v in out]


def my_items(weights: Sequence[float], rank: int, world: int) -> List[int]:
    return lpt_assign(weights, world)[rank]


def gather_records(local: List[SolveRecord], n_total: int, device: Optional[torch.device] = None,
                   group=None) -> List[SolveRecord]:
    """All-gather fixed-size per-system records; returns all systems sorted by index.

    Every rank contributes an ``[n_total, len(FIELDS)]`` fp64 tensor with NaN in rows it did
    not solve; the gathered rows are combined with a max-plus-fill (exactly one rank owns a row).
    """
    if not dist.is_available() or not dist.is_initialized():
        return sorted(local, key=lambda r: r.index)
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
            else torch.device("cpu")
    t = torch.full((n_total, len(FIELDS)), float("nan"), dtype=torch.float64, device=device)
    for r in local:
        t[r.index] = torch.tensor(r.as_list(), dtype=torch.float64)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    merged = parts[0].clone()
    for p in parts[1:]:
        fill = torch.isnan(merged[:, 0]) & ~torch.isnan(p[:, 0])
        merged[fill] = p[fill]
    merged = merged.cpu()
    return [SolveRecord.from_list(merged[i].tolist()) for i in range(n_total) if not torch.isnan(merged[i, 0])]


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def run_sharded(n_items: int, weights: Sequence[float], solve: Callable[[int], SolveRecord],
                device: Optional[torch.device] = None) -> List[SolveRecord]:
    """Solve this rank's share of the batch, then gather every record (collective at the end only)."""
    rank, world = _rank_world()
    mine = my_items(weights, rank, world)
    local = [solve(i) for i in mine]
    return gather_records(local, n_items, device)


def run_sharded_concurrent(n_items: int, weights: Sequence[float], prepare: Callable[[int], object],
                           finish: Callable[[object], SolveRecord], concurrency: int,
                           device: Optional[torch.device] = None) -> List[SolveRecord]:
    """run_sharded with up to ``concurrency`` solves of this rank in flight on its GPU.

    The rank's systems go in windows of ``concurrency``: ``prepare`` (GNN inference + assembly:
    one workspace, so one at a time, each timed on an otherwise idle device) runs for every
    system of the window on this thread, then ``finish`` (the PCG solve: every solver owns a
    non-blocking stream, and the native call releases the GIL) runs for all of them at once on a
    thread pool.  Mid-size systems are latency-bound (a few hundred workgroups per launch, five
    dependent launches per iteration), so concurrent solves fill the chip that one leaves idle.
    Results are those of the sequential path; per-system solve times include the overlap."""
    from concurrent.futures import ThreadPoolExecutor

    rank, world = _rank_world()
    mine = my_items(weights, rank, world)
    k = max(1, int(concurrency))
    local: List[SolveRecord] = []
    # the device this rank selected is per-thread state: the pool's threads select it too
    init, args = (), ()
    if torch.cuda.is_available():
        init, args = torch.cuda.set_device, (torch.cuda.current_device(),)
    with ThreadPoolExecutor(k, initializer=init or None, initargs=args) as ex:
        for w0 in range(0, len(mine), k):
            batch = [prepare(i) for i in mine[w0:w0 + k]]
            local.extend(ex.map(finish, batch))
    return gather_records(local, n_items, device)


def run_sharded_batched(n_items: int, weights: Sequence[float], prepare: Callable[[int], object],
                        finish_batch: Callable[[list], List[SolveRecord]], batch: int,
                        device: Optional[torch.device] = None,
                        prepare_batch: Optional[Callable[[list], list]] = None) -> List[SolveRecord]:
    """run_sharded with this rank's systems solved ``batch`` at a time as ONE batch (``finish_batch``
    over a window of prepared systems: linalg.BatchedConjugateGradient, every launch covering the
    whole window).  ``prepare_batch`` (optional) prepares a whole window at once (one GNN forward
    over the window's graphs) instead of ``prepare`` per system.  The records are gathered once at
    the end, as run_sharded."""
    rank, world = _rank_world()
    mine = my_items(weights, rank, world)
    k = max(1, int(batch))
    local: List[SolveRecord] = []
    for w0 in range(0, len(mine), k):
        window = mine[w0:w0 + k]
        jobs = prepare_batch(window) if prepare_batch is not None else [prepare(i) for i in window]
        local.extend(finish_batch(jobs))
    return gather_records(local, n_items, device)
