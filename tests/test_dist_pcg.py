"""CPU: the host side of the row-partitioned single-system PCG (dist_pcg.py, SURVEY.md §8(f)
rank 4): partition, halo plans, extended local matrices, the compensated cross-rank sum, and the
exchange / gather plumbing over gloo with world sizes 2 and 3 (127.0.0.1), and the plan built
from each rank's own rows by two all-to-alls (build_plan_exchanged) equal to the global one."""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.dist_pcg import (GROUPS, build_plan, build_plan_exchanged, dd_add, exchange,
                                                          gather_rows, local_matrix, partition_rows, sum_groups)


def _mats():
    A, _, _ = P.poisson2d_grid(30, 25)
    A = sp.csr_matrix(A)
    A.sort_indices()
    rng = np.random.default_rng(0)
    L = sp.csr_matrix(A, copy=True)
    L.data = rng.standard_normal(L.nnz)
    return [A, L, L.T.tocsr()]


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_plans_reproduce_global_spmv_in_scipy_order(world):
    mats = _mats()
    n = mats[0].shape[0]
    bounds = partition_rows(mats[0].indptr, world)
    assert bounds[0] == 0 and bounds[-1] == n and all(a <= b for a, b in zip(bounds, bounds[1:]))
    plans = [build_plan(mats, bounds, r) for r in range(world)]
    x = np.random.default_rng(1).standard_normal(n)
    for M in mats:
        y = []
        for r, p in enumerate(plans):
            xe = np.concatenate([x[bounds[r]:bounds[r + 1]], x[p.halo]])
            Ml = local_matrix(M, p)
            # stored order = global column order: the row sums are scipy's, bit for bit
            halo = np.append(p.halo, -1)  # (sentinel: an empty halo still indexes)
            g = np.where(Ml.indices < p.n_own, Ml.indices + bounds[r], halo[np.maximum(Ml.indices - p.n_own, 0)])
            for i in range(p.n_own):
                seg = slice(Ml.indptr[i], Ml.indptr[i + 1])
                assert np.all(np.diff(g[seg]) > 0)
            y.append((Ml @ xe)[:p.n_own])
            assert Ml.shape == (p.n_ext, p.n_ext) and Ml[p.n_own:].nnz == 0
        assert np.array_equal(np.concatenate(y), M @ x)
    for r, p in enumerate(plans):  # what rank s sends to r is r's halo block owned by s, in order
        for s, q in enumerate(plans):
            if s == r:
                continue
            off = sum(q.send_counts[:r])
            sent = q.send_idx[off:off + q.send_counts[r]] + bounds[s]
            got = p.halo[sum(p.recv_counts[:s]):sum(p.recv_counts[:s + 1])]
            assert np.array_equal(sent, got)


def test_sum_groups_is_compensated_and_order_fixed():
    rng = np.random.default_rng(2)
    vals = rng.standard_normal((3, GROUPS)) * 10.0 ** rng.integers(-8, 8, (3, GROUPS))
    buf = np.zeros((3, GROUPS * 2))
    buf[:, 0::2] = vals
    total = sum_groups(buf, 1)[0]
    exact = float(np.sum(np.array(sorted(vals.ravel(), key=abs), dtype=np.longdouble)))
    assert abs(total - exact) <= 2 ** -52 * abs(exact)
    acc = (0.0, 0.0)
    for v in vals.ravel():
        acc = dd_add(acc, (float(v), 0.0))
    assert total == acc[0] + acc[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mats = _mats()
    n = mats[0].shape[0]
    bounds = partition_rows(mats[0].indptr, world)
    p = build_plan(mats, bounds, rank)
    # the same plan from this rank's own rows and two all-to-alls
    r0, r1 = bounds[rank], bounds[rank + 1]
    pe = build_plan_exchanged([M[r0:r1] for M in mats], bounds, rank)
    ok_plan = (np.array_equal(pe.halo, p.halo) and pe.recv_counts == p.recv_counts
               and pe.send_counts == p.send_counts and np.array_equal(pe.send_idx, p.send_idx)
               and all((local_matrix(M[r0:r1], pe) != local_matrix(M, p)).nnz == 0 for M in mats))
    x = np.random.default_rng(3).standard_normal(n)
    own = torch.from_numpy(x[bounds[rank]:bounds[rank + 1]].copy())
    ext = torch.zeros(p.n_ext, dtype=torch.float64)
    ext[:p.n_own] = own
    send = own[torch.from_numpy(p.send_idx.astype(np.int64))]  # the device pack, restated
    exchange(ext[p.n_own:], send, p.recv_counts, p.send_counts)
    ok_halo = bool(torch.equal(ext[p.n_own:], torch.from_numpy(x[p.halo])))
    red = torch.zeros(GROUPS * 2, dtype=torch.float64)
    red[2 * rank] = float(rank + 1)  # group `rank` of this rank's buffer
    tot = sum_groups(gather_rows(red), 1)[0]
    q.put((rank, ok_halo and ok_plan, tot))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_halo_exchange_and_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, ok_halo, tot in outs:
        assert ok_halo, rank
        assert tot == sum(range(1, world + 1))


def test_plan_exchange_uses_device_tensors_on_nccl(monkeypatch):
    """on a nccl (RCCL) group the planning all-to-alls move device tensors (RCCL has no
    CPU backend), on gloo host tensors; the backend check is mocked (no GPU in the CPU suite), the
    gloo path itself runs for real in test_gloo_plan_exchange."""
    from learningsparsepreconditioner4gpu_amd import dist_pcg

    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    monkeypatch.setattr(dist_pcg, "_backend", lambda g: "nccl")
    assert dist_pcg.plan_device() == torch.device("cuda", 3)
    monkeypatch.setattr(dist_pcg, "_backend", lambda g: "gloo")
    assert dist_pcg.plan_device() == torch.device("cpu")
    src = open(dist_pcg.__file__).read().split("def build_plan_exchanged")[1].split("\ndef ")[0]
    assert "dev = plan_device(group)" in src and src.count("device=dev") == 3 and ".to(dev)" in src


def test_from_row_blocks_validates_its_blocks():
    """n and bounds are required, L_rows needs LT_rows, and every block must be
    (own rows) x n -- checked before any device work."""
    from learningsparsepreconditioner4gpu_amd.dist_pcg import DistributedPCG

    A = sp.csr_matrix(P.kuhn_laplacian(4))
    n = A.shape[0]
    with pytest.raises(TypeError):
        DistributedPCG.from_row_blocks(A)  # n / bounds missing
    with pytest.raises(ValueError, match="both L_rows and LT_rows"):
        DistributedPCG.from_row_blocks(A, A, n=n, bounds=[0, n])
    with pytest.raises(ValueError, match="bounds"):
        DistributedPCG.from_row_blocks(A, n=n, bounds=[0, n - 1])
    with pytest.raises(ValueError, match="shape"):
        DistributedPCG.from_row_blocks(A[: n - 3], n=n, bounds=[0, n])


def test_next_chunk_prediction():
    """dist_pcg's chunks follow the residual's decay, not a blind doubling to 16."""
    from learningsparsepreconditioner4gpu_amd.dist_pcg import next_chunk

    c, last = next_chunk(1, 16, 1, 1.0, 1e-4, 1000, None)  # no history yet: double
    assert c == 2 and last == (1, 1.0)
    # rr fell 1.0 -> 1e-2 over 2 iterations (a factor 10 per iteration in ‖r‖²): atol² = 1e-8 needs
    # log(1e-8 / 1e-2) / log(0.1) = 6 more
    c, last = next_chunk(2, 16, 3, 1e-2, 1e-4, 1000, last)
    assert c == 6 and last == (3, 1e-2)
    c, _ = next_chunk(2, 16, 3, 1e-2, 1e-4, 4, (1, 1.0))  # capped by max_iter - k
    assert c == 1
    c, _ = next_chunk(4, 16, 5, 1e-2, 1e-4, 1000, (3, 1e-2))  # no decay: double
    assert c == 8


@pytest.mark.parametrize("world", [2, 3])
def test_split_plans_interior_first(world):
    """Interior-first local numbering (dist_pcg overlap): every interior row's columns are owned, the
    local SpMV over [interior | boundary] rows reproduces scipy's rows bit for bit in global order,
    row_range splits a local matrix into the two launches' halves exactly, and what a rank sends is
    what its neighbours' halos hold."""
    from learningsparsepreconditioner4gpu_amd.dist_pcg import interior_rows, row_range

    mats = _mats()
    n = mats[0].shape[0]
    bounds = partition_rows(mats[0].indptr, world)
    plans = [build_plan(mats, bounds, r, split=True) for r in range(world)]
    x = np.random.default_rng(3).standard_normal(n)
    for M in mats:
        y = np.empty(n)
        for r, p in enumerate(plans):
            r0, r1 = bounds[r], bounds[r + 1]
            assert 0 < p.n_int < p.n_own and sorted(p.order) == list(range(r0, r1))
            ok = interior_rows([m[r0:r1] for m in mats], r0, r1)
            assert np.array_equal(np.sort(p.order[:p.n_int]), np.arange(r0, r1)[ok])
            xe = np.concatenate([x[p.order], x[p.halo]])
            Ml = local_matrix(M, p)
            assert Ml[:p.n_int].indices.max() < p.n_own  # interior rows: own columns only
            lo, hi = row_range(Ml, 0, p.n_int), row_range(Ml, p.n_int, p.n_own)
            assert (lo + hi - Ml).nnz == 0 and lo[p.n_int:].nnz == 0 and hi[:p.n_int].nnz == 0
            y[p.order] = (Ml @ xe)[:p.n_own]
        assert np.array_equal(y, M @ x)
    for r, p in enumerate(plans):
        for s, q in enumerate(plans):
            if s == r:
                continue
            off = sum(q.send_counts[:r])
            sent = q.order[q.send_idx[off:off + q.send_counts[r]]]
            got = p.halo[sum(p.recv_counts[:s]):sum(p.recv_counts[:s + 1])]
            assert np.array_equal(sent, got)


def _agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from learningsparsepreconditioner4gpu_amd.dist_pcg import all_ranks_agree

    A = sp.diags([-np.ones(5), np.full(6, 2.5), -np.ones(5)], [-1, 0, 1], format="csr")
    bounds = [0, 2, 4, 6]
    p = build_plan([A], bounds, rank, split=True)
    q.put((rank, p.n_int, p.n_own, all_ranks_agree(0 < p.n_int < p.n_own), all_ranks_agree(True),
           all_ranks_agree(rank != 2)))
    dist.barrier()
    dist.destroy_process_group()


def test_split_decision_all_ranks_agree():
    """ADVICE r5 (dist_pcg.py): the interior / boundary split changes the reductions' sizes, so it is
    decided by all ranks together: on a 6-row chain over 3 ranks the middle rank has no interior rows
    and every rank turns the split off; a flag true on all ranks stays true, false on one is false
    everywhere (gloo, world 3)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 3, port, q)) for r in range(3)]
    for pr in procs:
        pr.start()
    outs = sorted([q.get(timeout=120) for _ in range(3)])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert [o[1] for o in outs] == [1, 0, 1] and all(o[2] == 2 for o in outs)
    assert all(o[3:] == (False, True, False) for o in outs)


def test_sum_groups_two_halves():
    """Two 64-group halves per rank are summed rank-major, half by half: the same as treating every
    half as a rank (lspcg_part_scalars with world * 2)."""
    rng = np.random.default_rng(5)
    g = rng.standard_normal((3, 2 * GROUPS * 2 * 2))
    a = sum_groups(g, 2)
    b = sum_groups(g.reshape(6, GROUPS * 2 * 2), 2)
    assert a == b
