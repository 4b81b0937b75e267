"""CPU: the N>1 path (independent systems sharded across ranks + one gather at the end)
with the gloo backend, world_size 2 (and 3), on 127.0.0.1."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from learningsparsepreconditioner4gpu_amd.distributed import (SolveRecord, gather_records, lpt_assign, my_items,
                                                             run_sharded, run_sharded_batched,
                                                             run_sharded_concurrent)


def test_lpt_assignment_balanced_and_complete():
    w = [32000, 400, 12000, 9000, 30000, 700, 15000, 8000]
    parts = lpt_assign(w, 4)
    assert sorted(i for p in parts for i in p) == list(range(len(w)))
    loads = [sum(w[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(w)
    assert lpt_assign(w, 1) == [list(range(len(w)))]
    assert my_items(w, 0, 8) and all(len(p) == 1 for p in lpt_assign(w, 8))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_items, q, concurrency=0, batch=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    weights = [float(10 + (i * 7) % 5) for i in range(n_items)]

    def solve(i):  # deterministic stand-in for the GPU solve of system i
        return SolveRecord(index=i, iters=100 + i, rel_res=1e-9 * (i + 1), t_prec=0.001 * i, t_solve=0.01 * (i + 1),
                           n=1000 + i, nnz=5000 + i, converged=(i % 3 != 2))

    if batch:  # windows of `batch` prepared systems, each window solved by one call
        windows = []

        def finish_batch(jobs):
            assert 1 <= len(jobs) <= batch
            windows.append(list(jobs))
            return [solve(i) for i in jobs]

        recs = run_sharded_batched(n_items, weights, lambda i: i, finish_batch, batch, device=torch.device("cpu"))
        assert [i for w in windows for i in w] == my_items(weights, rank, world)
    elif concurrency:  # prepare on this thread in windows, the solves on a pool
        import threading

        main = threading.get_ident()
        prepared = []

        def prepare(i):
            assert threading.get_ident() == main
            prepared.append(i)
            return i

        recs = run_sharded_concurrent(n_items, weights, prepare, solve, concurrency, device=torch.device("cpu"))
        assert prepared == my_items(weights, rank, world)
    else:
        recs = run_sharded(n_items, weights, solve, device=torch.device("cpu"))
    q.put((rank, [r.as_list() for r in recs], my_items(weights, rank, world)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,concurrency,batch", [(2, 0, 0), (3, 0, 0), (2, 3, 0), (2, 0, 2)])
def test_gloo_sharded_gather(world, concurrency, batch):
    n_items = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, q, concurrency, batch)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = sorted(i for _, _, mine in outs for i in mine)
    assert owned == list(range(n_items))  # every system solved exactly once
    for rank, recs, _ in outs:
        assert [int(r[0]) for r in recs] == list(range(n_items))  # every rank sees all records
        for r in recs:
            i = int(r[0])
            assert r[1] == 100 + i and r[5] == 1000 + i and bool(r[7]) == (i % 3 != 2)


def test_gather_without_process_group_is_local():
    recs = [SolveRecord(2, 1, 0, 0, 0, 1, 1), SolveRecord(0, 1, 0, 0, 0, 1, 1)]
    assert [r.index for r in gather_records(recs, 3)] == [0, 2]


def test_concurrent_runner_without_process_group():
    weights = [5.0, 1.0, 3.0, 2.0, 4.0]
    recs = run_sharded_concurrent(5, weights, lambda i: i, lambda i: SolveRecord(i, 10 * i, 0, 0, 0, 1, 1), 2)
    assert [(r.index, r.iters) for r in recs] == [(i, 10.0 * i) for i in range(5)]


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    elapsed, iters = bench.reduce_timing(0.5 + rank, 212.0 * (rank + 1), torch.device("cpu"))
    q.put((rank, elapsed, iters))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_reduce_timing_max_and_sum(world):
    """bench.py's N>1 aggregation: value = iterations of ALL ranks / MAX-over-ranks wall time."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for _, elapsed, iters in out:
        assert elapsed == 0.5 + world - 1
        assert iters == 212.0 * world * (world + 1) / 2
