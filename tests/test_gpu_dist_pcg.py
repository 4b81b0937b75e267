"""GPU parity: ONE system row-partitioned over ranks (dist_pcg.py + csrc/lspcg_part.hip, SURVEY.md
§8(f) rank 4) against the oracle's scipy cg with correctly rounded dots and against the
single-GPU solver: same counts, iterates and residual histories to 1e-12.  World 1 runs in this
process; worlds 2 and 3 run as ranks on the one GPU of the box with gloo (halo and dot buffers
staged through the host) -- the RCCL path differs only in moving device buffers directly."""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp
import torch
import torch.multiprocessing as mp

from oracle import linalg as O
from tests import _cases
from learningsparsepreconditioner4gpu_amd import problems as P

pytestmark = pytest.mark.gpu
EPS = 3e-3


def _system(kind):
    if kind == "chain":  # 6-row 1-D chain over 3 ranks: the middle rank's two rows are both boundary rows
        A = sp.diags([-np.ones(5), np.full(6, 2.5), -np.ones(5)], [-1, 0, 1], format="csr")
        A.sort_indices()
        return A, _cases.spai_like(A), A @ np.ones(6)
    if kind == "kuhn":
        A, mask = P.kuhn_dirichlet(17)
    else:
        A, mask, _ = P.poisson2d_grid(90, 70)
    A = sp.csr_matrix(A)
    A.sort_indices()
    b = A @ np.asarray(mask, dtype=np.float64).reshape(-1)
    return A, _cases.spai_like(A), b


def _oracle(A, L, b, rtol):
    ps = O.spai_operator(L, EPS) if L is not None else None
    return O.pcg(A, b, ps, rtol=rtol, dot="exact")


@pytest.mark.parametrize("kind,precond", [("kuhn", "ext_spai"), ("poisson", "ext_spai"), ("poisson", "none")])
def test_world1_matches_oracle_and_single_gpu(gpu_ctx, kind, precond):
    from learningsparsepreconditioner4gpu_amd.dist_pcg import DistributedPCG
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A, L, b = _system(kind)
    L = L if precond == "ext_spai" else None
    d = DistributedPCG(A, L, EPS)
    it, conv, x, hist = d.solve(b, rtol=1e-8, return_history=True)
    it_h, conv_h, x_h, hist_h = d.solve_host(b, rtol=1e-8, return_history=True)  # round 3's host recurrence
    assert (it_h, conv_h) == (it, conv) and np.array_equal(hist_h, hist) and torch.equal(x_h, x)
    it_o, x_o, h_o = _oracle(A, L, b, 1e-8)
    assert conv and it == it_o
    np.testing.assert_allclose(hist, h_o[: it + 1], rtol=1e-12, atol=0)
    x = d.gather_solution(x)
    assert np.linalg.norm(x - x_o) <= 1e-12 * np.linalg.norm(x_o)
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner=precond)
    if L is not None:
        s.set_spai(L, EPS)
    bt = torch.from_numpy(b).cuda()
    xs = torch.zeros_like(bt)
    it_s, conv_s, _ = s.solve(bt, xs, rtol=1e-8)
    assert it_s == it
    np.testing.assert_allclose(x, xs.cpu().numpy(), rtol=0, atol=1e-12 * np.abs(x_o).max())


def test_world1_fp32(gpu_ctx):
    """fp32 vectors and matrices (the solver's LSPCG_F32 path): the oracle's fp32 scipy cg with
    correctly rounded dots, counts equal, x within the fp32 tolerance 1e-5."""
    from learningsparsepreconditioner4gpu_amd.dist_pcg import DistributedPCG

    A, L, b = _system("poisson")
    d = DistributedPCG(A, L, EPS, dtype=np.float32)
    it, conv, x = d.solve(b, rtol=1e-5)
    it_h, conv_h, x_h = d.solve_host(b, rtol=1e-5)
    assert (it_h, conv_h) == (it, conv) and torch.equal(x_h, x)
    ps = O.spai_operator(L.astype(np.float32), EPS)
    it_o, x_o, _ = O.pcg(A.astype(np.float32), b.astype(np.float32), ps, rtol=1e-5, dot="exact", dtype=np.float32)
    assert conv and it == it_o, (it, it_o)
    x = d.gather_solution(x)
    assert np.linalg.norm(x - x_o) <= 1e-5 * np.linalg.norm(x_o)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, kind, q, blocks=False, overlap=True):  # noqa: C901
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LSPCG_DIST_OVERLAP="1" if overlap else "0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from learningsparsepreconditioner4gpu_amd.dist_pcg import DistributedPCG, partition_rows

    A, L, b = _system(kind)
    if blocks:  # every rank hands over only its own rows of A, L and Lᵀ
        bounds = partition_rows(sp.csr_matrix(A).indptr, world)
        r0, r1 = bounds[rank], bounds[rank + 1]
        LT = sp.csr_matrix(L).T.tocsr()
        d = DistributedPCG.from_row_blocks(sp.csr_matrix(A)[r0:r1], sp.csr_matrix(L)[r0:r1], LT[r0:r1], n=A.shape[0],
                                           bounds=bounds, epsilon=EPS)
    else:
        d = DistributedPCG(A, L, EPS)
    it, conv, x, hist = d.solve(b, rtol=1e-8, return_history=True)
    it_h, conv_h, x_h, hist_h = d.solve_host(b, rtol=1e-8, return_history=True)
    same = (it_h, conv_h) == (it, conv) and np.array_equal(hist_h, hist) and torch.equal(x_h, x)
    xg = d.gather_solution(x)
    q.put((rank, it, bool(conv), xg, hist, d.plan.n_own, len(d.plan.halo), same, d.split, d.plan.n_int))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,blocks,overlap", [(2, False, True), (3, False, True), (3, True, True), (2, False, False)])
def test_multi_rank_matches_oracle(gpu_ctx, world, blocks, overlap):
    """blocks: DistributedPCG.from_row_blocks -- no rank holds the global system.  overlap: own rows
    numbered interior first, the interior rows' SpMVs enqueued while the halo exchange runs
    (LSPCG_DIST_OVERLAP=0: one row range)."""
    kind = "kuhn"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, kind, q, blocks, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=100) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A, L, b = _system(kind)
    it_o, x_o, h_o = _oracle(A, L, b, 1e-8)
    assert sum(o[5] for o in outs) == A.shape[0] and all(o[6] > 0 for o in outs)
    for rank, it, conv, xg, hist, _, _, same, split, _ in outs:
        assert split == overlap, rank
        assert same, rank  # device-side scalars = the host recurrence, bit for bit
        assert conv and it == it_o, (rank, it, it_o)
        np.testing.assert_allclose(hist, h_o[: it + 1], rtol=1e-12, atol=0)
        assert np.linalg.norm(xg - x_o) <= 1e-12 * np.linalg.norm(x_o)
    assert all(np.array_equal(outs[0][3], o[3]) for o in outs)  # every rank holds the same solution


def test_multi_rank_split_decision_is_collective(gpu_ctx):
    """a rank with no interior rows (the middle of a 6-row chain over 3 ranks) cannot
    overlap; the split is decided by all ranks together, so every rank runs one row range and the
    reductions keep one size on all ranks (the solve then matches the oracle)."""
    world, kind = 3, "chain"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, kind, q, False, True)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=100) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A, L, b = _system(kind)
    it_o, x_o, h_o = _oracle(A, L, b, 1e-8)
    assert [o[9] for o in outs][1] == 0  # the middle rank: no interior rows
    for rank, it, conv, xg, hist, _, _, same, split, _ in outs:
        assert not split and same, rank
        assert it == it_o, (rank, it, it_o)  # (6 rows: the oracle too runs its max_iter = n = 6 iterations)
        np.testing.assert_allclose(hist, h_o[: it + 1], rtol=1e-12, atol=0)
        assert np.linalg.norm(xg - x_o) <= 1e-12 * np.linalg.norm(x_o)


def _rank_rccl(port, q):
    """World 1 over nccl (RCCL): the collectives the multi-GPU paths issue, on device tensors."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import bench
    from learningsparsepreconditioner4gpu_amd import distributed as D
    from learningsparsepreconditioner4gpu_amd.dist_pcg import DistributedPCG

    A, L, b = _system("kuhn")
    d = DistributedPCG(A, L, EPS)
    it, conv, x = d.solve(b, rtol=1e-8)
    xg = d.gather_solution(x)
    recs = [D.SolveRecord(index=i, iters=10 + i, rel_res=0.5, t_prec=2e-3, t_solve=1e-3, n=100, nnz=500)
            for i in (2, 0)]
    got = D.gather_records(recs, 3)
    mx, sm = bench.reduce_timing(1.25, 7.0, torch.device("cuda", 0))
    dist.barrier()
    q.put((dist.get_backend(), it, bool(conv), xg, [(int(r.index), int(r.iters)) for r in got], mx, sm))
    dist.destroy_process_group()


def test_rccl_world1_collectives(gpu_ctx):
    """The nccl backend (RCCL) initialises on the box's GPU and carries the collectives of
    bench.py's max-over-ranks timing, distributed.gather_records and dist_pcg at world 1 (more
    ranks need more GPUs: the driver's scaling run; the multi-rank logic is covered over gloo above)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_rccl, args=(_free_port(), q))
    p.start()
    be, it, conv, xg, recs, mx, sm = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0 and be == "nccl"
    A, L, b = _system("kuhn")
    it_o, x_o, _ = _oracle(A, L, b, 1e-8)
    assert conv and it == it_o
    assert np.linalg.norm(xg - x_o) <= 1e-12 * np.linalg.norm(x_o)
    assert recs == [(0, 10), (2, 12)] and (mx, sm) == (1.25, 7.0)
