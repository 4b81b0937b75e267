"""One system row-partitioned over ranks.

Not in the reference: its systems each fit one process (``infer.py:278`` loops over samples; the
multi-GPU path of this package, ``distributed.py``, shards whole systems).  This is for a system
too large for one GPU's 288 GB.  Every rank owns a contiguous, nnz-balanced block of rows of A, L
and Lᵀ; one PCG iteration is scipy's ``cg`` (iterative.py:359-418, restated by the reference at
``validate.py:163-201``) with ``M⁻¹ r = L(Lᵀ r) + εr`` (``validate.py:173-182``):

    halo(r) -> t = Lᵀ r ; halo(t) -> z = L t + εr, ρ_k = r·z, ‖r_k‖²  [all-gather]
    top-of-loop test on ‖r_k‖ ; p = z + βp ; halo(p) -> q = A p, π = p·q  [all-gather]
    α = ρ/π ; x += αp ; r -= αq

The device phases are the native ``lspcg_part_*`` calls (csrc/lspcg_part.hip: the library's SpMV
kernels with own-row epilogues).  With more than one rank each rank's own rows are numbered
INTERIOR first (every column of the row, in A, L and Lᵀ, owned by the rank) then boundary; every
SpMV phase runs the interior rows while its halo all-to-all is in flight (RCCL: asynchronous on its
own stream) and the boundary rows after it (one part per row range, ``lspcg_part_set_rows``),
each row still summed in global column order (the same row bits); the dot partials of the two
ranges are gathered as two 64-group halves per rank.  ``LSPCG_DIST_OVERLAP=0`` keeps one range.  Exchanges go through ``torch.distributed``: the halo of a
vector is ONE ``all_to_all_single`` whose receive buffer is the tail of the rank's extended
vector (halo entries ordered by owner rank, so nothing is unpacked), and a dot product is an
all-gather of every rank's 64 per-group compensated (sum, correction) pairs into a device
buffer, summed by one single-thread kernel in rank-major order with double-double addition
(``lspcg_part_scalars``), then rounded -- every rank takes the same scalar, hence the same
convergence decision.  The scalars, scipy's top-of-loop test and the iteration count live in
the part's device state, so the host enqueues whole chunks of iterations and reads the state
once per chunk (no device-to-host round trip per reduction; ``solve_host`` keeps the round-3
host recurrence, bit-identical, for comparison).  With backend ``nccl`` (RCCL over xGMI) device
buffers are exchanged directly; with ``gloo`` (tests: several ranks on one GPU) they are staged
through host memory.  With one rank there is no exchange at all.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as dist

from . import _lib
from .sparse import Context, DeviceMatrix, _ptr

GROUPS = 64  # per-group DD slots of one reduction buffer (lspcg_part.hip kPartGroups)


# ---------------------------------------------------------------------------------------------
# host-side plan (pure numpy: tested on the CPU)
# ---------------------------------------------------------------------------------------------
def partition_rows(indptr: np.ndarray, world: int) -> List[int]:
    """Contiguous row blocks balanced by nnz + rows: bounds[r]..bounds[r+1] belong to rank r."""
    n = len(indptr) - 1
    work = np.asarray(indptr, dtype=np.int64) + np.arange(n + 1, dtype=np.int64)
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(work, work[-1] * r / world)))
    cuts.append(n)
    for r in range(1, world + 1):  # monotone (a rank may own nothing on tiny systems)
        cuts[r] = max(cuts[r], cuts[r - 1])
    return cuts


@dataclass
class HaloPlan:
    rank: int
    bounds: List[int]
    halo: np.ndarray          # global indices of the halo entries, ascending = grouped by owner
    recv_counts: List[int]    # halo entries per owner rank
    send_idx: np.ndarray      # own-row (local) indices sent, grouped by destination rank
    send_counts: List[int]
    # local numbering of the own rows: own_order[k] = global row of local row k (None: identity);
    # with the interior / boundary split, rows [0, n_int) are interior, [n_int, n_own) boundary
    own_order: Optional[np.ndarray] = None
    n_int: int = -1

    @property
    def n_own(self) -> int:
        return self.bounds[self.rank + 1] - self.bounds[self.rank]

    @property
    def n_ext(self) -> int:
        return self.n_own + len(self.halo)

    @property
    def order(self) -> np.ndarray:
        """Global row of every local own row."""
        r0 = self.bounds[self.rank]
        return self.own_order if self.own_order is not None else np.arange(r0, r0 + self.n_own)

    @property
    def local_of(self) -> np.ndarray:
        """Local index of every own row, indexed by global row - bounds[rank]."""
        inv = np.empty(self.n_own, dtype=np.int64)
        inv[self.order - self.bounds[self.rank]] = np.arange(self.n_own)
        return inv


def interior_rows(rows: Sequence[sp.csr_matrix], r0: int, r1: int) -> np.ndarray:
    """Own rows (in global order) whose every column, in every matrix of ``rows`` (the rank's row
    blocks, global column numbers), is owned by the rank: their SpMV rows need no halo entry."""
    n = r1 - r0
    ok = np.ones(n, dtype=bool)
    for M in rows:
        M = sp.csr_matrix(M)
        out = (M.indices < r0) | (M.indices >= r1)
        bad = np.add.reduceat(out.astype(np.int64), M.indptr[:-1]) if M.nnz else np.zeros(n, np.int64)
        bad = np.where(np.diff(M.indptr) > 0, bad, 0)  # reduceat on an empty row reads the next one
        ok &= bad == 0
    return ok


def split_order(rows: Sequence[sp.csr_matrix], r0: int, r1: int) -> Tuple[np.ndarray, int]:
    """Local numbering with the interior rows first: (global rows in local order, interior count)."""
    ok = interior_rows(rows, r0, r1)
    g = np.arange(r0, r1)
    return np.concatenate([g[ok], g[~ok]]), int(ok.sum())


def _needed_columns(mats: Sequence[sp.csr_matrix], r0: int, r1: int) -> np.ndarray:
    cols = [M.indices[M.indptr[r0]:M.indptr[r1]] for M in mats]
    return np.unique(np.concatenate(cols)) if cols else np.zeros(0, np.int64)


def build_plan(mats: Sequence[sp.csr_matrix], bounds: List[int], rank: int, split: bool = False) -> HaloPlan:
    """Halo of `rank` (columns of its rows in any of `mats` owned elsewhere) and what it sends
    (its own rows that the other ranks' rows reference, in their halo order); ``split``: own rows
    numbered interior first (split_order)."""
    world = len(bounds) - 1
    r0, r1 = bounds[rank], bounds[rank + 1]
    order, n_int = split_order([M[r0:r1] for M in mats], r0, r1) if split else (None, -1)
    owner = lambda g: np.searchsorted(bounds, g, side="right") - 1  # noqa: E731
    need = _needed_columns(mats, r0, r1)
    halo = need[(need < r0) | (need >= r1)]
    ho = owner(halo)
    recv_counts = [int(np.count_nonzero(ho == s)) for s in range(world)]
    send, send_counts = [], []
    for d in range(world):
        if d == rank:
            send_counts.append(0)
            continue
        nd = _needed_columns(mats, bounds[d], bounds[d + 1])
        mine = nd[(nd >= r0) & (nd < r1)]
        send.append(mine - r0)
        send_counts.append(int(mine.size))
    send_idx = np.concatenate(send).astype(np.int32) if send else np.zeros(0, np.int32)
    plan = HaloPlan(rank, list(bounds), halo.astype(np.int64), recv_counts, send_idx, send_counts, order, n_int)
    plan.send_idx = plan.local_of[send_idx.astype(np.int64)].astype(np.int32)
    return plan


def plan_device(group=None) -> torch.device:
    """Where the planning all-to-alls' tensors live: nccl (RCCL) moves device buffers only, so
    this rank's GPU there; the host otherwise (gloo)."""
    if _backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_ranks_agree(flag: bool, group=None) -> bool:
    """True when ``flag`` holds on EVERY rank of the group (one all-reduce MIN; the local flag without
    a process group): decisions that change the collectives' sizes must be taken together."""
    if _backend(group) is None:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=plan_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def build_plan_exchanged(rows: Sequence[sp.csr_matrix], bounds: List[int], rank: int, group=None,
                         split: bool = False) -> HaloPlan:
    """build_plan from this rank's OWN rows only (``rows``: the rank's row blocks, global column
    numbers): the halo comes from its own columns, and what it must send is what the other ranks
    ask for -- one all-to-all of request counts and one of the requested global indices
    (torch.distributed; O(own nnz) per rank instead of every rank rescanning every other rank's
    rows).  Equal to build_plan on the same matrices."""
    world = len(bounds) - 1
    r0, r1 = bounds[rank], bounds[rank + 1]
    cols = [M.indices for M in rows]
    need = np.unique(np.concatenate(cols)) if cols else np.zeros(0, np.int64)
    halo = need[(need < r0) | (need >= r1)].astype(np.int64)
    ho = np.searchsorted(bounds, halo, side="right") - 1
    recv_counts = [int(np.count_nonzero(ho == s)) for s in range(world)]
    order, n_int = split_order(rows, r0, r1) if split else (None, -1)
    be = _backend(group)
    if world == 1 or be is None:
        send_counts = [0] * world
        return HaloPlan(rank, list(bounds), halo, recv_counts, np.zeros(0, np.int32), send_counts, order, n_int)
    dev = plan_device(group)
    # my requests to owner s = my halo block owned by s (ascending); their counts first
    req_counts = torch.tensor(recv_counts, dtype=torch.int64, device=dev)
    got_counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(got_counts, req_counts, group=group)
    send_counts = [int(c) for c in got_counts.cpu()]
    got = torch.empty(int(sum(send_counts)), dtype=torch.int64, device=dev)
    dist.all_to_all_single(got, torch.from_numpy(halo).to(dev), send_counts, recv_counts, group=group)
    plan = HaloPlan(rank, list(bounds), halo, recv_counts, np.zeros(0, np.int32), send_counts, order, n_int)
    plan.send_idx = plan.local_of[got.cpu().numpy() - r0].astype(np.int32)
    return plan


def local_matrix(M: sp.csr_matrix, plan: HaloPlan) -> sp.csr_matrix:
    """The rank's rows of M over its extended numbering [own | halo], as a square n_ext matrix
    whose halo rows are empty.  Entries stay in GLOBAL column order inside each row (the local
    column numbers are then not ascending where a row has halo entries left of its own block):
    the SpMV kernels sum a row in stored order, so every row sum is scipy's csr_matvec order,
    the single-GPU solver's bits."""
    r0, r1 = plan.bounds[plan.rank], plan.bounds[plan.rank + 1]
    rows = (M if M.shape[0] == r1 - r0 else M[r0:r1]).tocsr()  # the global matrix or its row block
    rows.sort_indices()
    if plan.own_order is not None:  # local row order (interior first)
        rows = rows[plan.own_order - r0]
    g = rows.indices.astype(np.int64)
    own = (g >= r0) & (g < r1)
    loc = np.where(own, plan.local_of[np.clip(g - r0, 0, plan.n_own - 1)], plan.n_own + np.searchsorted(plan.halo, g))
    indptr = np.concatenate([rows.indptr, np.full(plan.n_ext - plan.n_own, rows.indptr[-1])])
    # stored (global) order kept: upload with DeviceMatrix.from_scipy(..., keep_order=True)
    return sp.csr_matrix((rows.data, loc.astype(np.int32), indptr), shape=(plan.n_ext, plan.n_ext))


def row_range(M: sp.csr_matrix, a: int, b: int) -> sp.csr_matrix:
    """M with only rows [a, b) kept (the others empty), same shape and entry order."""
    ip = M.indptr
    lo, hi = ip[a], ip[b]
    indptr = np.concatenate([np.zeros(a + 1, ip.dtype), ip[a + 1:b + 1] - lo, np.full(len(ip) - b - 1, hi - lo, ip.dtype)])
    return sp.csr_matrix((M.data[lo:hi], M.indices[lo:hi], indptr), shape=M.shape)


def dd_add(a: Tuple[float, float], b: Tuple[float, float]) -> Tuple[float, float]:
    """lspcg_internal.hpp dd_add (TwoSum of the heads, corrections added): IEEE doubles."""
    s = a[0] + b[0]
    bb = s - a[0]
    e = (a[0] - (s - bb)) + (b[0] - bb)
    return s, (a[1] + b[1]) + e


def sum_groups(gathered: np.ndarray, nd: int) -> List[float]:
    """gathered: [world, h * 64 * nd * 2] per-group (s, c) pairs (slot (g*nd + j)*2 of each of the
    rank's h halves of 64 groups: h = 2 with the interior / boundary split) -> nd totals, summed
    rank-major, half by half (lspcg_part_scalars' order with world * h)."""
    out = []
    for j in range(nd):
        acc = (0.0, 0.0)
        for row in gathered:
            v = row.reshape(-1, nd, 2)[:, j, :]
            for s, c in v[(v[:, 0] != 0) | (v[:, 1] != 0)]:  # adding an exact (0, 0) changes nothing
                acc = dd_add(acc, (float(s), float(c)))
        out.append(acc[0] + acc[1])
    return out


# ---------------------------------------------------------------------------------------------
# exchanges
# ---------------------------------------------------------------------------------------------
def _backend(group) -> Optional[str]:
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return dist.get_backend(group)


def exchange(recv: torch.Tensor, send: torch.Tensor, recv_counts: List[int], send_counts: List[int], group=None):
    """One all-to-all of halo entries (recv = the tail of an extended vector)."""
    be = _backend(group)
    if be is None or dist.get_world_size(group) == 1:
        return
    if be == "nccl" or not recv.is_cuda:
        dist.all_to_all_single(recv, send, recv_counts, send_counts, group=group)
        return
    rc = torch.empty(recv.shape, dtype=recv.dtype)  # gloo: host staging
    dist.all_to_all_single(rc, send.cpu(), recv_counts, send_counts, group=group)
    recv.copy_(rc)


def exchange_start(recv: torch.Tensor, send: torch.Tensor, recv_counts: List[int], send_counts: List[int], group=None):
    """``exchange`` begun asynchronously where the backend allows it: RCCL runs the all-to-all on its
    own stream (after the work already enqueued, e.g. the pack) and returns a handle; kernels
    enqueued before ``exchange_finish`` overlap it.  gloo (host-staged) completes here."""
    be = _backend(group)
    if be is None or dist.get_world_size(group) == 1:
        return None
    if be == "nccl":
        return dist.all_to_all_single(recv, send, recv_counts, send_counts, group=group, async_op=True)
    exchange(recv, send, recv_counts, send_counts, group)
    return None


def exchange_finish(work):
    """The compute stream waits for an exchange_start (no host wait under RCCL)."""
    if work is not None:
        work.wait()


def gather_device(t: torch.Tensor, group=None) -> torch.Tensor:
    """All ranks' copies of a small fixed-size device buffer, concatenated rank-major, on t's
    device (nccl: one all-gather, no host copy; gloo: staged through the host)."""
    be = _backend(group)
    if be is None or dist.get_world_size(group) == 1:
        return t.reshape(-1)
    w = dist.get_world_size(group)
    if be == "nccl" or not t.is_cuda:
        out = torch.empty(w * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.reshape(-1), group=group)
        return out
    tc = t.reshape(-1).cpu()
    parts = [torch.empty_like(tc) for _ in range(w)]
    dist.all_gather(parts, tc, group=group)
    return torch.cat(parts).to(t.device)


def gather_rows(t: torch.Tensor, group=None) -> np.ndarray:
    """All ranks' copies of a small fixed-size buffer -> [world, t.numel()] on the host."""
    be = _backend(group)
    if be is None or dist.get_world_size(group) == 1:
        return t.reshape(1, -1).cpu().numpy()
    w = dist.get_world_size(group)
    if be == "nccl" or not t.is_cuda:
        out = torch.empty(w * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.reshape(-1), group=group)
        return out.reshape(w, -1).cpu().numpy()
    tc = t.reshape(-1).cpu()
    parts = [torch.empty_like(tc) for _ in range(w)]
    dist.all_gather(parts, tc, group=group)
    return torch.stack(parts).numpy()


def next_chunk(chunk: int, max_chunk: int, k: int, rr: float, atol: float, max_iter: int, last):
    """Iterations to enqueue before the next state read, and the new ``last`` = (k, ‖r_k‖²): doubling
    while no decay has been observed, then the predicted remaining count (log(atol² / rr) over the
    observed log-decay per iteration, as lspcg_solver_solve's poll loop), capped by ``max_chunk``
    and ``max_iter - k``, at least 1."""
    nxt = min(2 * chunk, max_chunk)
    if last is not None and k > last[0] and 0.0 < rr < last[1]:
        rate = math.log(rr / last[1]) / (k - last[0])  # < 0
        need = math.log(atol * atol / rr) / rate if atol > 0 else float("inf")
        rem = max(1, int(math.ceil(need))) if need > 0 else 1
        nxt = max(1, min(rem, max_chunk, max(1, max_iter - k)))
    if last is None or k > last[0]:
        last = (k, rr)
    return nxt, last


# ---------------------------------------------------------------------------------------------
# the solver
# ---------------------------------------------------------------------------------------------
class DistributedPCG:
    """ext_spai PCG (``preconditioner="ext_spai"``, M⁻¹ = L Lᵀ + εI) or plain CG (L = None) of ONE
    system over the ranks of `group`.  A and L are the global scipy matrices (every rank reads
    the same host data and keeps only its rows on the device).  Iteration counts and iterates
    follow scipy's cg with compensated dot products; the dots are summed in a different order
    than the single-GPU solver's, so iterates agree to rounding (tests: 1e-12), not bit for bit."""

    def __init__(self, A, L=None, epsilon: float = 0.0, dtype=np.float64, group=None,
                 device: Optional[torch.device] = None):
        """A, L: the global matrices (every rank passes the same ones; only this rank's rows of
        A, L and Lᵀ are kept -- Lᵀ's row block is built from L's column block, never the whole
        transpose).  For systems whose global matrices do not fit one host, use from_row_blocks."""
        rank, world = self._rank_world(group)
        A = sp.csr_matrix(A, dtype=np.float64)
        bounds = partition_rows(A.indptr, world)
        r0, r1 = bounds[rank], bounds[rank + 1]
        blocks = [A[r0:r1]]
        if L is not None:
            L = sp.csr_matrix(L, dtype=np.float64)
            blocks += [L[r0:r1], sp.csc_matrix(L[:, r0:r1]).T.tocsr()]
        self._setup(blocks, A.shape[0], bounds, L is not None, epsilon, dtype, group, device)

    @classmethod
    def from_row_blocks(cls, A_rows, L_rows=None, LT_rows=None, *, n: int, bounds: Sequence[int],
                        epsilon: float = 0.0, dtype=np.float64, group=None, device: Optional[torch.device] = None):
        """Each rank passes only ITS row blocks (global column numbers) of A, L and Lᵀ for the row
        partition ``bounds`` (partition_rows of the global row pointer): no rank ever holds the
        global system; the halo plan is exchanged (build_plan_exchanged).  ``n`` and ``bounds``
        are required; L_rows and LT_rows come together; every block must be (own rows) x n."""
        if (L_rows is None) != (LT_rows is None):
            raise ValueError("from_row_blocks: pass both L_rows and LT_rows, or neither")
        rank, world = cls._rank_world(group)
        bounds = [int(b) for b in bounds]
        if len(bounds) != world + 1 or bounds[0] != 0 or bounds[-1] != int(n):
            raise ValueError(f"from_row_blocks: bounds must have {world + 1} entries from 0 to n = {n}")
        shape = (bounds[rank + 1] - bounds[rank], int(n))
        for name, M in (("A_rows", A_rows), ("L_rows", L_rows), ("LT_rows", LT_rows)):
            if M is not None and tuple(M.shape) != shape:
                raise ValueError(f"from_row_blocks: {name} has shape {tuple(M.shape)}, rank {rank} needs {shape}")
        self = cls.__new__(cls)
        self._setup([A_rows] + ([L_rows, LT_rows] if L_rows is not None else []), int(n), list(bounds),
                    L_rows is not None, epsilon, dtype, group, device)
        return self

    @staticmethod
    def _rank_world(group):
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(group), dist.get_world_size(group)
        return 0, 1

    def _setup(self, blocks, n, bounds, has_L, epsilon, dtype, group, device):
        import os

        self.group = group
        self.rank, self.world = self._rank_world(group)
        # interior rows overlap the halo exchange (more than one rank; LSPCG_DIST_OVERLAP=0: one range)
        self.split = self.world > 1 and os.environ.get("LSPCG_DIST_OVERLAP", "1") != "0"
        blocks = [sp.csr_matrix(M, dtype=np.float64) for M in blocks]
        for M in blocks:
            M.sort_indices()
        self.n = int(n)
        self.eps = float(epsilon)
        self.np_dtype = np.dtype(dtype)
        self.tdtype = torch.float64 if self.np_dtype == np.float64 else torch.float32
        self.ctx = Context.get(device)
        self.bounds = list(bounds)
        if len(self.bounds) != self.world + 1 or any(b1 <= b0 for b0, b1 in zip(self.bounds, self.bounds[1:])):
            raise ValueError(f"{self.world} ranks for {self.n} rows: every rank must own at least one row")
        self.plan = build_plan_exchanged(blocks, self.bounds, self.rank, group, split=self.split)
        mats = blocks
        L = blocks[1] if has_L else None
        p = self.plan
        if self.split:
            # nothing to overlap on a rank with no interior or no boundary rows; the halves of the
            # reductions are gathered from every rank, so the choice is collective (any rank without
            # both kinds of rows turns the split off everywhere)
            self.split = all_ranks_agree(0 < p.n_int < p.n_own, group)
        sidx = np.ascontiguousarray(p.send_idx, dtype=np.int32)

        def make_part(local, n_own, r0):
            dm = [DeviceMatrix.from_scipy(M, dtype=dtype, ctx=self.ctx, keep_order=True) for M in local]
            for M in dm:
                M.prepare_spmv()
            h = C.c_void_p()
            _lib.call("lspcg_part_create", self.ctx.handle, dm[0].handle, dm[1].handle if L is not None else None,
                      dm[2].handle if L is not None else None, n_own, sidx.ctypes.data_as(C.c_void_p),
                      int(sidx.size), C.byref(h))
            if r0:
                _lib.call("lspcg_part_set_rows", h, int(r0))
            return h, dm

        local = [local_matrix(M, p) for M in mats]
        if self.split:
            # the main part runs the boundary rows' SpMVs and every elementwise phase, the state and
            # the exchanges; the interior part only the interior rows' SpMVs
            self.handle, self._mats = make_part([row_range(M, p.n_int, p.n_own) for M in local], p.n_own, p.n_int)
            self.h_int, self._mats_int = make_part([row_range(M, 0, p.n_int) for M in local], p.n_int, 0)
        else:
            self.handle, self._mats = make_part(local, p.n_own, 0)
            self.h_int, self._mats_int = None, []
        self.halves = 2 if self.split else 1
        dev = self.ctx.torch_device
        ne, no = p.n_ext, p.n_own
        self.r = torch.zeros(ne, dtype=self.tdtype, device=dev)
        self.t = torch.zeros(ne, dtype=self.tdtype, device=dev)
        self.p = torch.zeros(ne, dtype=self.tdtype, device=dev)
        self.z = torch.zeros(max(no, 1), dtype=self.tdtype, device=dev)
        self.q = torch.zeros(max(no, 1), dtype=self.tdtype, device=dev)
        self.x = torch.zeros(max(no, 1), dtype=self.tdtype, device=dev)
        self.send = torch.zeros(max(int(sidx.size), 1), dtype=self.tdtype, device=dev)
        self.red = torch.zeros(2 * GROUPS * 2 * 2, dtype=torch.float64, device=dev)  # [half][64][nd][2]
        self.has_L = L is not None
        self.hist_dev = None

    def __del__(self):
        for name in ("handle", "h_int"):
            h = getattr(self, name, None)
            if h is not None and h.value and _lib._lib is not None:
                _lib._lib.lspcg_part_destroy(h)
                setattr(self, name, None)

    # ---- pieces
    def _T(self, v: float) -> float:
        return float(self.np_dtype.type(v))

    def _sqrt(self, v: float) -> float:
        return float(np.sqrt(self.np_dtype.type(v)))

    def _spmv(self, v: torch.Tensor, call):
        """One SpMV phase on v's halo: pack, the all-to-all started, the interior rows' SpMV (which
        reads own entries only) enqueued while it is in flight, then the boundary rows'.  ``call(h,
        red)`` enqueues the phase on part h with its reduction half."""
        p = self.plan
        work = None
        if self.world > 1:
            _lib.call("lspcg_part_pack", self.handle, _ptr(v), _ptr(self.send))
            work = exchange_start(v[p.n_own:], self.send[:p.send_idx.size], p.recv_counts, p.send_counts, self.group)
        if self.split:
            call(self.h_int, 0)
        exchange_finish(work)
        call(self.handle, 1 if self.split else 0)

    def _red(self, nd: int, half: int) -> torch.Tensor:
        """Half `half` of the reduction buffer for nd dots: [64][nd][2] doubles, halves adjacent."""
        return self.red[half * GROUPS * nd * 2:(half + 1) * GROUPS * nd * 2]

    def _halo(self, v: torch.Tensor):
        p = self.plan
        if self.world == 1:
            return
        _lib.call("lspcg_part_pack", self.handle, _ptr(v), _ptr(self.send))
        exchange(v[p.n_own:], self.send[:p.send_idx.size], p.recv_counts, p.send_counts, self.group)

    def _reduce(self, nd: int, halves: int = 1) -> List[float]:
        return sum_groups(gather_rows(self.red[:halves * GROUPS * nd * 2], self.group), nd)

    def own_slice(self) -> slice:
        return slice(self.bounds[self.rank], self.bounds[self.rank + 1])

    def _own_rows(self, v_global: np.ndarray) -> np.ndarray:
        """This rank's entries of a global vector, in the local (interior-first) order."""
        return np.asarray(v_global)[self.plan.order]

    def _to_global_order(self, x_local: torch.Tensor) -> torch.Tensor:
        """This rank's rows of a local-order vector, back in global row order."""
        if self.plan.own_order is None:
            return x_local.clone()
        idx = torch.as_tensor(self.plan.local_of, device=x_local.device)
        return x_local[idx]

    # ---- the SpMV phases on both row ranges
    def _lt(self):
        self._spmv(self.r, lambda h, half: _lib.call("lspcg_part_lt", h, _ptr(self.r), _ptr(self.t)))

    def _l(self):
        self._spmv(self.t, lambda h, half: _lib.call("lspcg_part_l", h, _ptr(self.t), _ptr(self.r), self.eps,
                                                      _ptr(self.z), _ptr(self._red(2, half))))

    def _a(self):
        self._spmv(self.p, lambda h, half: _lib.call("lspcg_part_a", h, _ptr(self.p), _ptr(self.q),
                                                      _ptr(self._red(1, half))))

    # ---- solve (device-side scalar recurrence)
    def _scalars(self, nd: int, phase: int, halves: int = 1):
        g = gather_device(self.red[:halves * GROUPS * nd * 2], self.group) if nd else None
        _lib.call("lspcg_part_scalars", self.handle, _ptr(g) if g is not None else None, self.world * halves, phase)
        self._keep = g  # the gathered buffer stays alive until the kernel that reads it has run

    def _iteration(self):
        """One scipy cg iteration, enqueued without a host round trip; every scalar is read from and
        written to the device state, and every update is skipped once the state says done."""
        if self.has_L:
            self._lt()
            self._l()
            self._scalars(2, 1, self.halves)  # ρ, ‖r_k‖², the top-of-loop test, β
            z = self.z
        else:
            self._scalars(0, 2)
            z = self.r
        _lib.call("lspcg_part_update_p_dev", self.handle, _ptr(z), _ptr(self.p))
        self._a()
        self._scalars(1, 3, self.halves)  # π, α
        _lib.call("lspcg_part_update_xr_dev", self.handle, _ptr(self.p), _ptr(self.q), _ptr(self.x), _ptr(self.r))
        if not self.has_L:
            _lib.call("lspcg_part_norms", self.handle, _ptr(self.r), _ptr(self.r), _ptr(self.red))
            self._scalars(2, 4)

    def _status(self):
        it, done = C.c_int64(), C.c_int()
        _lib.call("lspcg_part_status", self.handle, C.byref(it), C.byref(done))
        return it.value, done.value

    def _progress(self):
        it, done, rr, atol = C.c_int64(), C.c_int(), C.c_double(), C.c_double()
        _lib.call("lspcg_part_progress", self.handle, C.byref(it), C.byref(done), C.byref(rr), C.byref(atol))
        return it.value, done.value, rr.value, atol.value

    def solve(self, b_global: np.ndarray, rtol: float = 1e-6, max_iter: int = 0, return_history: bool = False,
              max_chunk: int = 16):
        """scipy cg from x0 = 0 on the global rhs (every rank passes the same vector).  Returns
        ``(iters, converged, x_own[, history])``; x_own: this rank's rows of the solution.
        Iterations are enqueued in chunks with the device state read once per chunk: 1, 2, 4, ...
        ``max_chunk`` until the residual has decayed twice, then sized by the predicted remaining
        iterations (next_chunk; the single-GPU solver's rule), so few iterations run past
        convergence -- each would still pay its halo exchanges and all-gathers.  Iterations
        enqueued past convergence skip every update (predicated on the state), so count, history
        and x are those of the converged iteration."""
        p = self.plan
        no = p.n_own
        mi = int(max_iter) if max_iter and max_iter > 0 else self.n
        b = torch.as_tensor(self._own_rows(b_global), dtype=self.tdtype).to(self.ctx.torch_device)
        if self.hist_dev is None or self.hist_dev.numel() < mi + 2:
            self.hist_dev = torch.empty(mi + 2, dtype=torch.float64, device=self.ctx.torch_device)
        self.hist_dev.fill_(float("nan"))
        self.x.zero_()
        self.r.zero_()
        self.r[:no] = b
        self.p.zero_()
        _lib.call("lspcg_part_state_init", self.handle, float(rtol), mi, _ptr(self.hist_dev))
        _lib.call("lspcg_part_norms", self.handle, _ptr(self.r), _ptr(self.r), _ptr(self.red))
        self._scalars(2, 0)
        k, done = self._status()
        if done == 4:  # ‖b‖ = 0: scipy returns b
            self.x[:no] = b
            out = (0, True, self._to_global_order(self.x[:no]))
            return out + ((self.hist_dev[:1].cpu().numpy(),) if return_history else ())
        chunk = 1
        last = None  # (iteration, ‖r‖²) of the previous state read
        while not done:
            for _ in range(chunk):
                self._iteration()
            k, done, rr, atol = self._progress()
            chunk, last = next_chunk(chunk, int(max_chunk), k, rr, atol, mi, last)
        iters = mi if done == 3 else k
        out = (iters, done == 1, self._to_global_order(self.x[:no]))
        if return_history:
            # a non-finite stop reports max_iter (pymathprim's count): NaN after the last written
            # entry, iters + 1 entries, as lspcg_solver_solve does
            h = np.full(iters + 1, np.nan)
            got = self.hist_dev[: min(k, iters) + 1].cpu().numpy()
            h[:got.size] = got
            out = out + (h,)
        return out

    # ---- solve (host scalar recurrence: round 3's path, kept for comparison)
    def solve_host(self, b_global: np.ndarray, rtol: float = 1e-6, max_iter: int = 0,
                   return_history: bool = False):
        """``solve`` with the scalars summed and tested on the host after every reduction (two
        device-to-host round trips per iteration); the same bits as ``solve``."""
        p = self.plan
        no = p.n_own
        mi = int(max_iter) if max_iter and max_iter > 0 else self.n
        b = torch.as_tensor(self._own_rows(b_global), dtype=self.tdtype).to(self.ctx.torch_device)
        self.x.zero_()
        self.r.zero_()
        self.r[:no] = b
        self.p.zero_()
        _lib.call("lspcg_part_norms", self.handle, _ptr(self.r), _ptr(self.r), _ptr(self.red))
        rr0, bb = (self._T(v) for v in self._reduce(2))
        bn = self._sqrt(bb)
        atol = max(0.0, rtol * bn)
        hist = [self._sqrt(rr0)]
        if bn == 0.0:  # scipy returns b
            self.x[:no] = b
            return (0, True, self._to_global_order(self.x[:no])) + ((np.array(hist),) if return_history else ())
        rr, rho_prev, k, code = rr0, 0.0, 0, 0
        while True:
            if self.has_L:
                self._lt()
                self._l()
                rho, rr_k = (self._T(v) for v in self._reduce(2, self.halves))
                z = self.z
            else:  # CG: z = r, ρ = ‖r‖² (from the previous update, or the init)
                rr_k = rr if k > 0 else rr0
                rho = rr_k
                z = self.r
            if k > 0:
                rr = rr_k
                hist.append(self._sqrt(rr))
            # scipy's top-of-loop test (k_update_p_g)
            if k >= mi:
                code = 2
            else:
                rn = self._sqrt(rr)
                if rn < atol:
                    code = 1
                elif not math.isfinite(rn):
                    code = 3
            if code:
                break
            beta = 0.0 if k == 0 else self._T(self.np_dtype.type(rho) / self.np_dtype.type(rho_prev))
            _lib.call("lspcg_part_update_p", self.handle, _ptr(z), _ptr(self.p), beta, int(k == 0))
            self._a()
            (pq,) = (self._T(v) for v in self._reduce(1, self.halves))
            alpha = self._T(self.np_dtype.type(rho) / self.np_dtype.type(pq))
            _lib.call("lspcg_part_update_xr", self.handle, alpha, _ptr(self.p), _ptr(self.q), _ptr(self.x),
                      _ptr(self.r))
            if not self.has_L:  # ‖r_{k+1}‖² for the next test
                _lib.call("lspcg_part_norms", self.handle, _ptr(self.r), _ptr(self.r), _ptr(self.red))
                rr = self._T(self._reduce(2)[0])
            rho_prev = rho
            k += 1
        iters = mi if code == 3 else k
        out = (iters, code == 1, self._to_global_order(self.x[:no]))
        if return_history:
            # a non-finite stop reports max_iter (pymathprim's count): NaN-padded to iters + 1
            # entries, as lspcg_solver_solve does
            h = np.full(iters + 1, np.nan)
            h[:len(hist)] = hist[:iters + 1]
            out = out + (h,)
        return out

    def gather_solution(self, x_own: torch.Tensor) -> np.ndarray:
        """The full solution on every rank (host), from each rank's own rows."""
        w = self.world
        if w == 1:
            return x_own.cpu().numpy().astype(np.float64)
        m = max(self.bounds[r + 1] - self.bounds[r] for r in range(w))
        buf = torch.zeros(m, dtype=torch.float64, device=self.ctx.torch_device)
        buf[:x_own.numel()] = x_own[: self.plan.n_own].to(torch.float64)
        rows = gather_rows(buf, self.group)
        return np.concatenate([rows[r][: self.bounds[r + 1] - self.bounds[r]] for r in range(w)])
