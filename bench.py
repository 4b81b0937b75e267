#!/usr/bin/env python
"""Headline benchmark: GNN-SPAI preconditioned CG on MI355X (BASELINE.json metric).

A "step" is one full PCG solve (ext_spai, M⁻¹ = L Lᵀ + εI, rtol 1e-8, x0 = 0,
b = A·mask as infer.py:297-299) of one system held in HBM.  Setup (outside the timed
region, like the reference's "precond time"): host generation of the system, the GNN
forward that emits L (HIP), and device assembly of A and L with Dirichlet masking.

value = CG iterations completed by ALL ranks / max-over-ranks wall time of the K timed
solves.  Multi-GPU: one process per GPU (torchrun), each rank solves its own independent
system (no data-path collective); one RCCL all-reduce of the per-rank timings at the end.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload kuhn101]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

METRIC = "CG iters/sec + time-to-rel-residual-1e-8; SpMV achieved HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md "Chip-level parameters")
FLUSH_BYTES = 512 << 20  # > 256 MiB Infinity Cache


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def spmv_bytes(n: int, nnz: int, dtype_bytes: int = 8) -> int:
    """Algorithmic bytes of one scalar CSR SpMV: vals + col idx per nnz,
    row pointer, x read once, y written once."""
    return (dtype_bytes + 4) * nnz + 4 * (n + 1) + 2 * dtype_bytes * n


def bsr3_bytes(nb: int, nnzb: int) -> int:
    """Algorithmic bytes of one BSR 3x3 SpMV: 9 fp64 values + 1 column per block,
    block row pointer, x read once (24 B per block row), y written once."""
    return (72 + 4) * nnzb + 4 * (nb + 1) + 24 * nb + 24 * nb


def gnn_flops(n_nodes: int, n_edges: int, f_in: int, e_in: int, e_out: int, layers: int = 4, h: int = 16) -> float:
    """Multiply-add flops (x2) of one NodeEdgeProcessing forward (gnns.py:77-97, F = 16, 2-layer
    MLPs): node / edge encoders, per MP layer the message and edge MLPs (48->16->16->16) on every
    edge and the node MLP (16->16->16->16) on every node, the edge decoder (48->16->16->b²)."""
    mlp = lambda i, o: 2 * (i * h + h * h + h * o)
    per_edge = mlp(e_in, h) + layers * 2 * mlp(3 * h, h) + mlp(3 * h, e_out)
    per_node = mlp(f_in, h) + layers * mlp(h, h)
    return float(per_edge) * n_edges + float(per_node) * n_nodes


def host_cpu() -> dict:
    """CPU model and logical CPUs of the host running the bench (lscpu, else /proc/cpuinfo)."""
    import subprocess

    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:  # pragma: no cover - lscpu absent
        pass
    if model is None:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:  # pragma: no cover
            pass
    return {"model": model, "nproc": os.cpu_count()}


def pcg_bytes_per_iter(n: int, nnz_a: int, nnz_l: int) -> int:
    """Algorithmic bytes of one ext_spai PCG iteration: 3 SpMVs (x read and
    y written once each) + 10 further fp64 vector passes (r in Lt+εr; z, p read + p written in
    the p-update; x, p, r, q read + x, r written in the x/r update)."""
    return spmv_bytes(n, nnz_a) + 2 * spmv_bytes(n, nnz_l) + 8 * n * 10


def reduce_timing(elapsed: float, iters: float, device) -> tuple:
    """Whole-job numbers of a multi-rank run: wall time = MAX over ranks, iterations = SUM
    (one all-reduce each; RCCL on the GPU, gloo in the CPU test)."""
    import torch
    import torch.distributed as dist

    mx = torch.tensor([elapsed], dtype=torch.float64, device=device)
    sm = torch.tensor([iters], dtype=torch.float64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx[0]), float(sm[0])


KERNEL_NAME = {1: "k_spmv_sdia", 16: "k_spmv_sell<int16 columns>", 17: "k_spmv_sellj", 18: "k_spmv_sellj<XS>",
               32: "k_spmv_sell<int32 columns>"}
KIND_TEXT = {1: "SELL-DIA: one slot per distinct row-relative offset of the 64-row slice, 2-B row masks, no columns",
             8: "SELL-64C: one-byte codes into per-slice dictionaries of <= 64 row-relative offsets",
             16: "16-bit column offsets",
             17: "SELL-64J: lanes sorted by row length inside each 64-row slice, groups stored for their active "
                 "lanes only, 16-bit column offsets",
             18: "SELL-64X: SELL-64J whose 16-bit column words index an LDS copy of the 256-row tile's x blocks "
                 "(16 entries each, loaded once per tile)",
             32: "int32 columns"}
JAG_PAD = 1.15  # csrc/lspcg_sell.hpp kSellJagPad
XS_MAX = 256    # csrc/lspcg_sell.hpp kSellXMax: x blocks per 256-row tile
XS_MIN_N = 262144  # csrc/lspcg_sell.hpp kSellXMinN


def sell_slots(indptr: np.ndarray) -> int:
    """Stored slots of the SELL-64 layout (csrc/lspcg_sell.hpp): per 64-row slice, 64 x the
    slice's longest row rounded up to a multiple of 4."""
    lens = np.diff(indptr)
    ns = (lens.size + 63) // 64
    pad = np.zeros(ns * 64, dtype=np.int64)
    pad[: lens.size] = lens
    return int(256 * ((pad.reshape(ns, 64).max(axis=1) + 3) // 4).sum())


def jag_elems(indptr: np.ndarray) -> int:
    """Stored entries of the SELL-64J layout (csrc/lspcg_sell.hpp kSellJag): every row's entries
    rounded up to whole 4-entry groups (a group stores only the lanes whose rows reach it)."""
    return int(4 * ((np.diff(indptr) + 3) // 4).sum())


def xs_blocks(indptr: np.ndarray, indices: np.ndarray) -> np.ndarray:
    """Distinct 16-entry x blocks (col // 16) each 256-row tile reads (the SELL-64X staged lists)."""
    n = indptr.size - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    key = np.unique((rows // 256) * (1 << 32) + indices.astype(np.int64) // 16)
    return np.bincount(key >> 32, minlength=(n + 255) // 256)


def dia_counts(indptr: np.ndarray, indices: np.ndarray) -> np.ndarray:
    """Distinct row-relative offsets col - row per 64-row slice (SELL-DIA slots per row)."""
    n = indptr.size - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    key = np.unique((rows // 64) * (1 << 33) + (indices.astype(np.int64) - rows + (1 << 32)))
    return np.bincount(key >> 33, minlength=(n + 63) // 64)


def sell_kind(indptr: np.ndarray, indices: np.ndarray) -> int:
    """Column storage the SELL-64 build picks (csrc/lspcg_sell.hip, sorted rows): 1 = SELL-DIA
    (<= 16 distinct offsets col - row per 64-row slice, no more slots than 4-entry groups), 17 =
    SELL-64J (16-bit offsets, SELL-64 would pad more than JAG_PAD x nnz, no row beyond 64 entries),
    16 = 16-bit offsets from the slice's first row, 32 = int32 columns."""
    n = indptr.size - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    if rows.size == 0:
        return 32
    d = dia_counts(indptr, indices)
    if d.max() <= 16 and 64 * d.sum() <= sell_slots(indptr):
        return 1
    if not np.all(np.abs(indices.astype(np.int64) - (rows // 64) * 64) <= 32767):
        return 32
    if sell_slots(indptr) > JAG_PAD * rows.size and np.diff(indptr).max() <= 64:
        return 18 if n >= XS_MIN_N and xs_blocks(indptr, indices).max() <= XS_MAX else 17
    return 16


def sell_format_bytes(indptr: np.ndarray, indices: np.ndarray, kind: int, value_bytes: int) -> int:
    """Matrix bytes one SELL-64 SpMV streams.  SELL-DIA: 64 x D_s value slots per slice + the 2-B row
    masks (128 B per slice) + the slice's 16-entry int32 offset dictionary (64 B); otherwise every
    stored slot's value and column (2 B offset or 4 B index)."""
    ns = (indptr.size + 62) // 64
    if kind == 1:
        return int(64 * dia_counts(indptr, indices).sum() * value_bytes) + ns * (128 + 64)
    if kind == 17:  # + the lane -> row bytes (64) and group counts (16) per slice
        return int(jag_elems(indptr) * (value_bytes + 2)) + ns * (64 + 16)
    if kind == 18:  # + the tiles' block lists (4 B per block, 4 B per tile)
        return (int(jag_elems(indptr) * (value_bytes + 2)) + ns * (64 + 16)
                + 4 * int(xs_blocks(indptr, indices).sum()) + 4 * ((indptr.size + 254) // 256))
    return int(sell_slots(indptr) * (value_bytes + {16: 2, 32: 4}[kind]))


def pcg_loop_spmv(A, p, q, reps: int, kind: int) -> dict:
    """The SpMV the PCG loop runs (fp32-stored values -- exact for the reference's fp32-born
    matrices -- and the loop's column storage `kind`) timed cold / warm on the same matrix,
    against the bytes of its own format: stored slots + x read + y written."""
    import ctypes as C

    from learningsparsepreconditioner4gpu_amd import _lib

    out = {}
    for label, flush in (("cold", FLUSH_BYTES), ("warm", 0)):
        ms = C.c_double()
        _lib.call("lspcg_spmv_sell_timed", A.ctx.handle, A.handle, 3 | (8 if kind == 1 else 0) | (16 if kind in (17, 18) else 0) | (32 if kind == 18 else 0),
                  C.c_void_p(p.data_ptr()),
                  C.c_void_p(q.data_ptr()), reps if flush else 3 * reps, flush, C.byref(ms))
        out[label] = ms.value
    As = A.to_scipy()
    fmt = sell_format_bytes(As.indptr, As.indices, kind, 4) + 16 * A.n
    return {"kernel": f"{KERNEL_NAME[kind]}<double,float> as in the PCG loop (values stored as fp32 -- lossless "
                      f"for the reference's fp32-born A and L -- {KIND_TEXT[kind]})",
            "format_bytes": fmt, "avg_launch_ms_cold": out["cold"], "avg_launch_ms_warm": out["warm"],
            "achieved_format_GBs_cold": fmt / (out["cold"] * 1e-3) / 1e9,
            "frac_format_cold": fmt / (out["cold"] * 1e-3) / 1e9 / HBM_PEAK_GBS}


def loop_dominant(kernels: dict, A, n: int, nnz_l: int) -> dict:
    """The longest launch of the PCG iteration against three byte counts, each labelled:
    * format bytes: SELL slots x 6 B (fp32 values, 16-bit columns -- the loop's lossless compact
      views of A, L and Lᵀ, which share one pattern) + the fp64 vectors it reads / writes;
    * counter bytes: HBM traffic of the same kernel from the committed PMC passes
      (profiles/pcg_loop_traffic.json, FETCH_SIZE x 2 + WRITE_SIZE) when they match this system;
    * SURVEY 8(d) bytes: fp64 / int32 CSR of the matrix + the vectors -- NOT what the loop moves
      (compact format, part of the working set served by the Infinity Cache), so this fraction
      can exceed 1 and is reported for reference only."""
    vec = {"KA t=L^T r": 2, "KB z=L t+eps r, rho": 3, "UP p, x": 5, "KC q=A p, pi": 2, "UR r": 3}
    name = max(kernels, key=kernels.get)
    t = kernels[name]
    out = {"kernel": name, "us": t * 1e6, "all_us": {k: v * 1e6 for k, v in kernels.items()}}
    if A.block_size == 1:
        As = A.to_scipy()
        kind = sell_kind(As.indptr, As.indices)
        out["format"] = f"SELL-64, fp32 values, {KIND_TEXT[kind]}"
        fmt = (sell_format_bytes(As.indptr, As.indices, kind, 4) if name.startswith("K") else 0) + 8 * n * vec[name]
        out.update({"format_bytes": fmt, "achieved_GBs_format": fmt / t / 1e9,
                    "frac_format": fmt / t / 1e9 / HBM_PEAK_GBS})
        survey = ((spmv_bytes(n, nnz_l) - 16 * n) if name.startswith("K") else 0) + 8 * n * vec[name]
        out.update({"survey_bytes": survey, "frac_survey_bytes": survey / t / 1e9 / HBM_PEAK_GBS,
                    "survey_bytes_note": "fp64/int32 CSR bytes of SURVEY 8(d); the loop reads a compact format and "
                                         "Infinity-Cache-resident lines, so this fraction may exceed 1"})
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pcg_loop_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        kind_ok = A.block_size != 1 or tj.get("column_kind", 16) == sell_kind(A.to_scipy().indptr, A.to_scipy().indices)
        if tj.get("n") == n and kind_ok and name in tj.get("kernels", {}):
            tb = tj["kernels"][name]["traffic_bytes"]
            out.update({"counter_bytes": tb, "frac_counter_bytes": tb / t / 1e9 / HBM_PEAK_GBS,
                        "counter_bytes_source": "profiles/pcg_loop_traffic.json"})
    return out


def cpu_solve(A, b, M, rtol: float, max_iter: int, threads: int):
    """The reference's CPU restatement (validate.py:163-201 / 316-333: scipy cg, explicit-Lᵀ SPAI
    LinearOperator), timed like validate.py:196-198 (time around cg only); BLAS threads limited
    to `threads` (scipy's CSR matvec is single-threaded either way).  Returns (iterations, s)."""
    from scipy.sparse.linalg import cg
    from threadpoolctl import threadpool_limits

    count = 0

    def cb(_x):
        nonlocal count
        count += 1

    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        cg(A, b, M=M, callback=cb, rtol=rtol, maxiter=max_iter)
        dt = time.perf_counter() - t0
    return count, dt


def cpu_rate(A, b, M, rtol: float, max_iter: int, threads: int, reps: int = 5) -> dict:
    """1 warm-up + the median of `reps` bounded solves: iterations/s."""
    cpu_solve(A, b, M, rtol, max_iter, threads)
    runs = [cpu_solve(A, b, M, rtol, max_iter, threads) for _ in range(reps)]
    its = [r[0] for r in runs]
    dts = sorted(r[1] for r in runs)
    med = dts[len(dts) // 2]
    return {"iters_per_solve": int(np.median(its)), "median_s": med, "it_per_s": float(np.median(its)) / med,
            "threads": threads}


def cpu_baseline(A, L, eps, gt, max_iter: int, rtol: float, all_threads: bool = False) -> dict:
    """ext_spai on the bench system, bounded to max_iter iterations per solve, at 1 BLAS thread
    (and at nproc threads with --cpu-all-threads: measured slower on the 256-thread box host, 7.3
    vs 43.4 iterations/s, profiles/r3_bench_v2.json -- scipy's CSR matvec is single-threaded and
    256 BLAS threads only add overhead to the dots)."""
    from oracle import linalg as O

    Aop = A.astype(np.float64)
    M = O._Op(O.spai_operator(L.astype(np.float64), eps), A.shape, np.float64)
    b = Aop @ gt
    out = {"1": cpu_rate(Aop, b, M, rtol, max_iter, 1)}
    if all_threads:
        out["nproc"] = cpu_rate(Aop, b, M, rtol, max_iter, os.cpu_count() or 1)
    return out


def reference_iters(workload: str, boo) -> dict:
    """The REFERENCE's own count on this very system (tests/golden/traj_<workload>.npz, written by
    tests/golden/make_golden.py: get_pcg_iter_time_scipy on the bench's A and GNN-L at 1 / 2 / 4 / 8
    OpenBLAS threads), if the fixture exists and its GNN-output sha256 equals this run's."""
    import hashlib

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", f"traj_{workload}.npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)
    sha = hashlib.sha256(np.ascontiguousarray(boo.detach().cpu().numpy()).tobytes()).hexdigest()
    out = {"counts_by_openblas_threads": dict(zip([str(int(t)) for t in z["ref_threads"]],
                                                  [int(c) for c in z["ref_counts"]])),
           "oracle_correctly_rounded_count": int(z["oracle_exact_count"]), "same_L": sha == str(z["boo_sha256"]),
           "source": f"tests/golden/traj_{workload}.npz (validate.py:163-201 run on this A and GNN-L)"}
    rpath = path[:-4] + "_refgnn.npz"
    if os.path.exists(rpath):  # the reference end to end: its own GNN forward -> its L -> its PCG
        r = np.load(rpath)
        stride = int(r["stride"])
        got = boo.detach().reshape(-1, *r["ref_sample"].shape[1:])[::stride].cpu().numpy().astype(np.float64)
        err = float(np.abs(got - r["ref_sample"].astype(np.float64)).max())
        out["reference_gnn"] = {
            "counts_by_openblas_threads": dict(zip([str(int(t)) for t in r["ref_threads"]],
                                                   [int(c) for c in r["refL_counts"]])),
            "oracle_correctly_rounded_count": int(r["oracle_exact_count"]),
            "gnn_max_abs_err_vs_reference_sampled": err, "gnn_max_abs_reference": float(r["max_abs_ref"]),
            "source": f"tests/golden/traj_{workload}_refgnn.npz (the reference's NodeEdgeProcessing forward, "
                      "to_csr_cpu and get_pcg_iter_time_scipy on this system)"}
    return out


def parity_rows(A, L, eps: float, b, rtol: float, threads=(1, 8)) -> dict:
    """The headline solve in the parity dot order (dot_order="openblas": numpy's ddot at T OpenBLAS
    threads, the reference's recorded trajectory bit for bit): iterations and time, 1 warm-up +
    median of 3."""
    import torch

    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    out = {}
    for th in threads:
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64,
                                            dot_order="openblas", dot_threads=th)
        s.set_spai(L, eps, block_size=L.block_size)
        x = torch.zeros_like(b)
        ts = []
        for _ in range(4):
            x.zero_()
            it, conv, t = s.solve(b, x, rtol=rtol)
            ts.append(t)
        med = float(np.median(ts[1:]))
        out[f"openblas_{th}_threads"] = {"iters": it, "converged": bool(conv), "time_to_rtol_ms": med * 1e3,
                                         "it_per_s": it / med}
        del s
    return out


def irregular_row(workload: str, eps: float, rtol: float, reps: int) -> dict:
    """An irregular ordering of the headline's 1M-row system (problems.renumber: a seeded random
    symmetric permutation then reverse Cuthill-McKee -- banded like an RCM-ordered tet mesh, ~32
    distinct row-relative offsets per 64-row slice, so the 16-bit SELL-64 views instead of
    SELL-DIA): GNN-L on it, the PCG loop (1 warm-up + median of 3 solves) and the fp64 SpMV
    against the SURVEY 8(d) CSR bytes, cold."""
    import torch

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    A_raw, mask, feats, bs, e2n = P.workload(workload)
    smp = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=smp.x.shape[1], edge_features=smp.edge_attr.shape[1], block_size=bs,
                                  epsilon=eps, seed=0)
    d = smp.to("cuda")
    L, _ = ws.inference_step(d)
    A = ws.system_matrix(d)
    b = A.matvec(d.mask.reshape(-1).to(torch.float64))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
    s.set_spai(L, eps, block_size=bs)
    setup_ms = (time.perf_counter() - t0) * 1e3
    x = torch.zeros_like(b)
    ts = []
    for _ in range(4):
        x.zero_()
        it, conv, t = s.solve(b, x, rtol=rtol)
        ts.append(t)
    med = float(np.median(ts[1:]))
    try:
        loop = s.time_kernels(b, 40)
    except RuntimeError:
        loop = {}
    Ah = A.to_scipy()
    kind_loop = sell_kind(Ah.indptr, Ah.indices)
    p = torch.randn(A.n, dtype=torch.float64, device="cuda")
    q = torch.empty_like(p)
    kind = A.prepare_spmv()
    spmv_ro = A.spmv_reorder_info  # (reordered: the timing covers x's gather, the SpMV and y's scatter)
    cold = A.spmv_timed(p, q, reps, flush_bytes=FLUSH_BYTES)
    warm = A.spmv_timed(p, q, 3 * reps)
    alg = spmv_bytes(A.n, A.nnz)
    dc = dia_counts(Ah.indptr, Ah.indices)
    how = ("random symmetric permutation + RCM" if workload.endswith("rcm") else
           "random symmetric permutation" if workload.endswith("rand") else "the generator's spatial bucket order")
    what = ("the unstructured Delaunay heat system (problems.delaunay_heat: qhull tets of a seeded uniform point "
            "cloud, P1 Laplacian + lumped mass, heat_tetmesh.py)" if workload.startswith("delaunay")
            else "the headline system renumbered")
    lens = np.diff(Ah.indptr)
    pad = sell_slots(Ah.indptr) / max(A.nnz, 1)
    # why these views (a mesh whose loop misses the structured headline's per-entry time
    # names the format it runs on and the reason)
    view_text = {"sdia": "SELL-DIA", "sell16": "SELL-64 with 16-bit column offsets", "sell32": "SELL-64 with int32 columns",
                 "sellc": "SELL-64C (one-byte offset codes)", "sell16j": "SELL-64J (jagged: no padded slots)",
                 "sell16x": "SELL-64X (jagged, x blocks staged in LDS per 256-row tile)", "csr": "the staged CSR kernel"}
    ro = s.reorder_info
    reason = (f"input numbering: {dc.mean():.0f} distinct row-relative offsets per 64-row slice on average (max "
              f"{int(dc.max())}; SELL-DIA needs <= 16 in every slice, SELL-64C <= 64 in most), rows of "
              f"{int(lens.min())}-{int(lens.max())} entries (SELL-64 would store {pad:.2f} slots per entry); "
              + ("the solver runs on its device-RCM placement (mean |col - row| %.0f -> %.0f) with "
                 % (ro["mean_offset_before"], ro["mean_offset_after"]) if ro["applied"] else "the solver runs ")
              + view_text.get(s.views["A"]["columns"], s.views["A"]["columns"]) + " views")
    return {"workload": f"{workload}: {what} ({how}), n={A.n}, nnz={A.nnz}, ext_spai, rtol {rtol:g}",
            "views_reason": reason,
            "row_entries": {"mean": float(lens.mean()), "min": int(lens.min()), "max": int(lens.max())},
            "sell_slots_per_nnz": pad,
            "solver_reorder": s.reorder_info, "solver_setup_ms": setup_ms,
            "distinct_offsets_per_slice": {"mean": float(dc.mean()), "max": int(dc.max())},
            "bandwidth": int(np.abs(Ah.indices - np.repeat(np.arange(A.n), np.diff(Ah.indptr))).max()),
            "spmv_column_storage": KIND_TEXT[kind_loop], "solver_views": s.views, "iters": it, "converged": bool(conv),
            "time_to_rtol_ms": med * 1e3, "pcg_iter_us": med / it * 1e6,
            "pcg_iter_ps_per_nnz": med / it * 1e12 / max(A.nnz, 1),
            "loop_kernels_us": {k: v * 1e6 for k, v in loop.items()},
            "spmv": {"kernel": f"{KERNEL_NAME.get(kind, 'k_spmv')}<double,double>"
                               + (" on P A P^T (device RCM): x gathered, y scattered, all three launches timed"
                                  if spmv_ro["applied"] else ""), "reorder": spmv_ro, "avg_launch_ms_cold": cold,
                     "avg_launch_ms_warm": warm, "alg_bytes": alg, "achieved_GBs_cold": alg / (cold * 1e-3) / 1e9,
                     "frac_cold": alg / (cold * 1e-3) / 1e9 / HBM_PEAK_GBS}}


def c1_rows(rtol: float, all_threads: bool = False) -> dict:
    """BASELINE config 1 (datagen/synthetic.py N = 10240, CG, b = A·1): the reference's CPU path
    (scipy cg, full solve, 1 warm-up + median of 5, 1 BLAS thread; nproc threads with
    --cpu-all-threads) beside the HIP solver on the same system, in the default dot order and in
    the parity order (the reference's own count at 1 OpenBLAS thread, 3236)."""
    import scipy.sparse as sp
    import torch

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.synthetic_c1())
    n = A.shape[0]
    b = A @ np.ones(n)
    cpu = {"1": cpu_rate(A, b, None, rtol, n, 1)}
    if all_threads:
        cpu["nproc"] = cpu_rate(A, b, None, rtol, n, os.cpu_count() or 1)
    bt = torch.from_numpy(b).cuda()
    x = torch.zeros_like(bt)
    gpu = {}
    for label, order, threads in (("compensated", "compensated", 1), ("openblas", "openblas", 1),
                                  ("openblas_8_threads", "openblas", 8)):
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="none", dot_order=order,
                                            dot_threads=threads)
        ts = []
        for _ in range(6):
            x.zero_()
            it, conv, t = s.solve(bt, x, rtol=rtol)
            ts.append(t)
        med = float(np.median(ts[1:]))
        gpu[label] = {"iters": it, "time_to_rtol_ms": med * 1e3, "it_per_s": it / med}
    return {"workload": "synthetic C1 n=10240 nnz=%d, CG (none), b = A·1, rtol %g" % (A.nnz, rtol),
            "gpu": gpu, "reference_iters": {"1_openblas_thread": 3236, "8_openblas_threads": 3229}, "cpu": cpu}


def c5_rows(rtol: float, concurrency: int = 4, dataset: str = "heat_batch8") -> dict:
    """C5 (the heat-tet batch, 8 systems of 400-32 k vertices -- the reference's real
    dataset sizes; ``delaunay_batch8``: the same sizes on unstructured Delaunay tet meshes): the
    batch's ext_spai solves one after another (the reference's loop), with `concurrency` in flight
    (linalg.solve_many) and as ONE lockstep batch (linalg.BatchedConjugateGradient), best of 3
    each; every system keeps its own count."""
    import torch

    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient, solve_many
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = synthetic_dataset(dataset)
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=1, seed=0)
    jobs = []
    for smp in samples:
        d = smp.to("cuda")
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d)
        b = A.matvec(d.mask.reshape(-1).to(torch.float64))
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
        s.set_spai(L, ws.epsilon)
        jobs.append((s, b, torch.zeros_like(b)))
    solve_many(jobs, rtol, concurrency=1)  # graphs built
    out = {"workload": "C5 %s: 8 heat-tet systems (n = %d..%d), ext_spai, rtol %g"
                       % (dataset, min(j[0].n for j in jobs), max(j[0].n for j in jobs), rtol),
           "views": sorted({j[0].views["A"]["columns"] for j in jobs})}
    for k in (1, concurrency):
        best = None
        for _ in range(3):
            for j in jobs:
                j[2].zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = solve_many(jobs, rtol, concurrency=k)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None or dt < best else best
        its = [r[0] for r in res]
        out[f"concurrency_{k}"] = {"wall_ms": best * 1e3, "systems_per_s": len(jobs) / best,
                                   "iters_total": int(sum(its)), "us_per_iter_per_system": best * 1e6 / sum(its)}
    out["iters"] = its
    from learningsparsepreconditioner4gpu_amd.linalg import BatchedConjugateGradient

    B = BatchedConjugateGradient([j[0].A for j in jobs], [j[0]._L for j in jobs], ws.epsilon)
    bs = [j[1] for j in jobs]
    xs = [torch.zeros_like(b) for b in bs]
    B.solve(bs, xs, rtol)  # graphs built
    best = None
    for _ in range(3):
        for x in xs:
            x.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res, _ = B.solve(bs, xs, rtol)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    bits = [r[0] for r in res]
    out["batched"] = {"wall_ms": best * 1e3, "systems_per_s": len(jobs) / best, "iters_total": int(sum(bits)),
                      "us_per_iter_per_system": best * 1e6 / sum(bits), "us_per_lockstep_iter": best * 1e6 / max(bits),
                      "iters_equal_sequential": bits == its}
    return out


def config_rows() -> dict:
    """BASELINE.md §2's other configurations beside the headline: C2 Poisson-2D 256² (rtol 1e-8),
    C3 heat on the voxelised bunny (rtol 1e-6), C4 elasticity BSR 3×3 (rtol 1e-8) and C5 the 8
    heat systems (rtol 1e-8, sum and max over the batch), each with the GNN-inferred L (seeded
    random init) and ext_spai: the HIP solver (1 warm-up + median of 5 solves) and the reference's
    scipy restatement on the same A, L, b (1 thread; 1 warm-up + median of 3; full solves, C4
    bounded to 60 iterations per solve: its 2.5 k iterations take minutes on one core)."""
    import scipy.sparse as sp
    import torch

    from oracle import linalg as O
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    def one(sample, rtol, cpu_max_iter):
        ws = SimpleInferenceWorkspace(node_features=sample.x.shape[1], edge_features=sample.edge_attr.shape[1],
                                      block_size=sample.block_size, seed=0)
        d = sample.to("cuda")
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d)
        gt = d.mask.reshape(-1).to(torch.float64)
        b = A.matvec(gt)
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
        s.set_spai(L, ws.epsilon, block_size=L.block_size)
        x = torch.zeros_like(b)
        ts = []
        for _ in range(6):
            x.zero_()
            it, conv, t = s.solve(b, x, rtol=rtol)
            ts.append(t)
        t_gpu = float(np.median(ts[1:]))
        A_h, L_h = sp.csr_matrix(A.to_scipy()), sp.csr_matrix(L.to_scipy())
        b_h = A_h @ gt.cpu().numpy()
        M = O._Op(O.spai_operator(L_h, ws.epsilon), A_h.shape, np.float64)
        mi = cpu_max_iter or A_h.shape[0]
        cpu = cpu_rate(A_h, b_h, M, rtol, mi, 1, reps=3)
        return {"n": A.n, "nnz": A.nnz, "views": s.views["A"]["columns"], "iters": it, "converged": bool(conv),
                "gpu_ms": t_gpu * 1e3, "gpu_us_per_iter": t_gpu * 1e6 / max(it, 1),
                "gpu_it_per_s": it / t_gpu, "cpu_iters": cpu["iters_per_solve"], "cpu_s": cpu["median_s"],
                "cpu_it_per_s": cpu["it_per_s"], "cpu_bounded": bool(cpu_max_iter)}

    def wl(name):
        A, mask, feats, bs, e2n = P.workload(name)
        return make_sample(A, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)

    out = {"C2_poisson256": one(wl("poisson256"), 1e-8, 0), "C3_heat_bunny": one(wl("bunny"), 1e-6, 0),
           "C4_elasticity": one(wl("elast"), 1e-8, 60)}
    for ds in ("heat_batch8", "delaunay_batch8"):  # C5 and its variant on unstructured Delaunay meshes
        rows = [one(smp, 1e-8, 0) for smp in synthetic_dataset(ds)]
        out[f"C5_{ds}"] = {
            "systems": rows, "gpu_ms_sum": sum(r["gpu_ms"] for r in rows), "gpu_ms_max": max(r["gpu_ms"] for r in rows),
            "cpu_s_sum": sum(r["cpu_s"] for r in rows), "cpu_s_max": max(r["cpu_s"] for r in rows)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="kuhn101")
    ap.add_argument("--epsilon", type=float, default=3e-3)
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--cpu-iters", type=int, default=60,
                    help="iterations per bounded CPU baseline solve (1 warm-up + median of 5, at nproc and 1 BLAS threads)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-all-threads", action="store_true",
                    help="also time the CPU legs at nproc BLAS threads (slower than 1 thread on the box host)")
    ap.add_argument("--no-variants", action="store_true", help="skip the none / diagonal / random-rhs time-to-rtol rows")
    ap.add_argument("--spmv-reps", type=int, default=30)
    ap.add_argument("--configs", action="store_true",
                    help="instead of the headline line: C2-C5 GPU rows beside the reference's scipy CPU path")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per local rank; more ranks than GPUs (a gloo rehearsal on one GPU) share them
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if args.configs:  # side table (BASELINE.md §2 configurations), rank 0 of a 1-GPU run only
        print(json.dumps({"configs": config_rows(), "cpu": host_cpu(), "cpu_threads": 1}), flush=True)
        return
    if world > 1:
        # RCCL over xGMI; LSPCG_DIST_BACKEND=gloo rehearses several ranks on ONE GPU (RCCL refuses that)
        backend = os.environ.get("LSPCG_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": torch.device("cuda", local)} if backend == "nccl" else {}))

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    # ---- setup (untimed): host system, GNN -> L on device, A on device
    t0 = time.time()
    A_raw, mask, feats, bs, e2n = P.workload(args.workload)
    sample = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    log(f"rank {rank}: system {args.workload} n={A_raw.shape[0]} nnz={A_raw.nnz} host setup {time.time() - t0:.1f}s")
    ws = SimpleInferenceWorkspace(node_features=sample.x.shape[1], edge_features=sample.edge_attr.shape[1],
                                  block_size=bs, epsilon=args.epsilon, seed=0)
    dev_sample = sample.to("cuda")
    for _ in range(2):
        L, gnn_dt = ws.inference_step(dev_sample)  # warm the GNN (infer.py:270-275)
    gnn_times = []
    for _ in range(5):
        L, gnn_dt = ws.inference_step(dev_sample)
        gnn_times.append(gnn_dt)
    log(f"rank {rank}: GNN forward ms {[round(t * 1e3, 3) for t in gnn_times]}")
    gnn_fl = gnn_flops(sample.x.shape[0], sample.edge_index.shape[1], sample.x.shape[1], sample.edge_attr.shape[1],
                       bs * bs)
    ref_iters = reference_iters(args.workload, ws.forward(dev_sample.x, dev_sample.edge_index, dev_sample.edge_attr))
    A = ws.system_matrix(dev_sample)
    n, nnz_a, nnz_l = A.n, A.nnz, L.nnz
    gt = dev_sample.mask.reshape(-1).to(torch.float64)
    b = A.matvec(gt)
    solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
    prec_s = solver.set_spai(L, args.epsilon, block_size=L.block_size)
    x = torch.zeros_like(b)

    def step():
        x.zero_()
        it, conv, solve_s = solver.solve(b, x, rtol=args.rtol)
        return it, conv, solve_s

    for _ in range(args.warmup):
        it, conv, _ = step()
    log(f"rank {rank}: warmup done, iterations/solve={it} converged={conv}")

    # ---- timed region
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    iters = []
    solve_times = []
    for _ in range(args.steps):
        it, conv, solve_s = step()
        iters.append(it)
        solve_times.append(solve_s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    total_iters = float(sum(iters))
    if world > 1:
        elapsed, total_iters = reduce_timing(elapsed, total_iters, torch.device("cuda", local))

    # ---- the loop's own launches, each bracketed by HIP events (one untimed 40-iteration pass on
    # the solver stream after the timed region): the dominant kernel against its format bytes
    try:
        loop_kernels = solver.time_kernels(b, 40)
    except RuntimeError as e:  # other schedules (LSPCG_NO_SELL, fused): not instrumented
        log(f"rank {rank}: no per-launch loop timing: {e}")
        loop_kernels = {}
    loop_dom = loop_dominant(loop_kernels, A, n, nnz_l) if loop_kernels else None

    views = solver.views

    # ---- time-to-rtol beside the neural preconditioner (infer.py:310-321 rows): CG and Jacobi on the
    # same system and rhs, and every method with infer.py's rhs="random" (:300-302, b = A (randn ⊙ mask))
    variants = None
    if not args.no_variants:
        variants = {}
        rng = np.random.default_rng(0)
        b_rand = A.matvec(torch.from_numpy(rng.standard_normal(n) * gt.cpu().numpy()).cuda())
        for meth in ("ext_spai", "none", "diagonal"):
            sv = solver if meth == "ext_spai" else PreconditionedConjugateGradient(A, device="cuda", preconditioner=meth,
                                                                                 dtype=np.float64)
            row = {}
            for rhs_name, bb in (("mask", b), ("random", b_rand)):
                xx = torch.zeros_like(bb)
                ts = []
                for _ in range(3):
                    xx.zero_()
                    it_v, conv_v, t_v = sv.solve(bb, xx, rtol=args.rtol)
                    ts.append(t_v)
                row[rhs_name] = {"iters": it_v, "converged": bool(conv_v), "time_to_rtol_ms": float(np.median(ts)) * 1e3}
            variants[meth] = row
            if sv is not solver:
                del sv
        log(f"rank {rank}: variants {variants}")

    # ---- the SpMV of A (fp64, the reference's scalar CSR / BSR 3x3) against the HBM roofline: first
    # the staged kernel, then after the analysis step (SELL-64 / BSELL-64 copy, fp64 values, 16-bit
    # column offsets) -- the product's lspcg_spmv path, which the roofline line reports
    p = torch.randn(n, dtype=torch.float64, device="cuda")
    q = torch.empty_like(p)
    csr_cold = A.spmv_timed(p, q, args.spmv_reps, flush_bytes=FLUSH_BYTES)
    csr_warm = A.spmv_timed(p, q, args.spmv_reps * 3)
    kind = A.prepare_spmv()
    ms_cold = A.spmv_timed(p, q, args.spmv_reps, flush_bytes=FLUSH_BYTES)
    ms_warm = A.spmv_timed(p, q, args.spmv_reps * 3)
    if A.block_size == 3:
        if kind == 1:
            kernel = ("k_spmv_bsdia3<double,double> BSELL-DIA block copy of the fp64 BSR 3x3 A (one slot per "
                      "distinct block offset of the 64-block-row slice, no columns, 16-B value loads), bit-exact "
                      "scipy bsr_matvec order")
        elif kind:
            kernel = (f"k_spmv_bsell3<double,double,int{kind}> BSELL-64 block copy of the fp64 BSR 3x3 A (one "
                      f"{kind}-bit column per block, 16-B value loads), bit-exact scipy bsr_matvec order")
        else:
            kernel = "k_spmv<double,3> staged BSR 3x3 SpMV of A, bit-exact scipy bsr_matvec order"
        alg = bsr3_bytes(n // 3, A.nnzb)
        alg_formula = "(72+4)·nnzb + 4·(N_b+1) + 24·N_b + 24·N_b (SURVEY.md 8(d), BSR b=3)"
    else:
        kernel = (f"{KERNEL_NAME[kind]}<double,double> SELL-64 copy of the fp64 CSR A ({KIND_TEXT[kind]}, "
                  "fp64 values), bit-exact scipy order" if kind else
                  "k_spmv<double,1> staged scalar CSR SpMV of A, bit-exact scipy order")
        alg = spmv_bytes(n, nnz_a)
        alg_formula = "12·nnz + 20·n + 4 (SURVEY.md 8(d), scalar CSR fp64)"
    # BSR: scalar SELL views only; the loop's views share A's pattern and column storage
    pcg_spmv = pcg_loop_spmv(A, p, q, args.spmv_reps, kind) if A.block_size == 1 and kind else None
    gbs_cold = alg / (ms_cold * 1e-3) / 1e9
    gbs_warm = alg / (ms_warm * 1e-3) / 1e9
    it_per_solve = iters[-1]
    t_iter = float(np.median(solve_times)) / max(it_per_solve, 1)
    pcg_gbs = pcg_bytes_per_iter(n, nnz_a, nnz_l) / t_iter / 1e9

    # HBM bytes per launch of the same kernel on the same matrix from the committed PMC passes
    # (tools/spmv_traffic.sh: FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction), if they match
    traffic = None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "spmv_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("n") == n and tj.get("nnz") == nnz_a and tj.get("kernel_kind") == kind:
            traffic = tj["traffic_bytes"]

    cpu = None
    c1 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        hc = host_cpu()
        try:
            A_h = A.to_scipy()
            L_h = L.to_scipy()
            if L.block_size > 1:
                L_h = L_h.tocsr()
                A_h = A_h.tocsr()
            gt_h = gt.cpu().numpy()
            log(f"cpu baseline: scipy cg, <= {args.cpu_iters} iterations per solve, 1 warm-up + median of 5, "
                f"1 BLAS thread" + (f" and {hc['nproc']}" if args.cpu_all_threads else ""))
            cb = cpu_baseline(A_h, L_h, args.epsilon, gt_h, args.cpu_iters, args.rtol, args.cpu_all_threads)
            best = max(cb.values(), key=lambda r: r["it_per_s"])
            cpu = {"value": best["it_per_s"], "unit": "CG iters/s", "cores": best["threads"], "kind": "port",
                   "cpu_model": hc["model"], "nproc": hc["nproc"], "by_threads": cb,
                   "sample": f"ext_spai PCG on the same system (scipy {__import__('scipy').__version__} cg + explicit-Lᵀ "
                             f"SPAI LinearOperator, validate.py:163-201), solves bounded to {args.cpu_iters} "
                             f"iterations, 1 warm-up + median of 5, 1 BLAS thread (scipy's CSR matvec is "
                             f"single-threaded; nproc = {hc['nproc']} BLAS threads measured slower, "
                             "--cpu-all-threads)"}
        except Exception as e:  # pragma: no cover - reported, not fatal
            cpu = {"value": None, "unit": "CG iters/s", "cores": 1, "kind": "port", "sample": f"failed: {e}",
                   "cpu_model": hc["model"], "nproc": hc["nproc"]}
        try:
            c1 = c1_rows(1e-8, args.cpu_all_threads)
        except Exception as e:  # pragma: no cover
            c1 = {"failed": str(e)}
    c5 = None
    parity = None
    irregular = None
    if rank == 0 and world == 1 and not args.no_variants:
        try:
            c5 = c5_rows(args.rtol)
            c5["delaunay_batch8"] = c5_rows(args.rtol, dataset="delaunay_batch8")
        except Exception as e:  # pragma: no cover
            c5 = {"failed": str(e)}
        try:
            parity = parity_rows(A, L, args.epsilon, b, args.rtol)
        except Exception as e:  # pragma: no cover
            parity = {"failed": str(e)}
        if args.workload == "kuhn101":
            try:
                irregular = {w: irregular_row(w, args.epsilon, args.rtol, args.spmv_reps)
                             for w in ("kuhn101rcm", "kuhn101rand", "delaunay1m")}
                for row in irregular.values():  # per-entry loop time against this run's structured headline
                    row["pcg_iter_per_nnz_vs_headline"] = row["pcg_iter_ps_per_nnz"] / (t_iter * 1e12 / max(A.nnz, 1))
            except Exception as e:  # pragma: no cover
                irregular = {"failed": str(e)}

    if rank == 0:
        value = total_iters / elapsed
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "CG iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: Kuhn-tet grid Laplacian (Dirichlet face), seeded random-init GNN weights",
            "config": {
                "workload": f"{args.workload}: ext_spai PCG to rel-residual {args.rtol:g}, n={n}, nnz(A)={nnz_a}, "
                            f"nnz(L)={nnz_l}, GNN-inferred L (F=16, 4 MP layers)",
                "n": n, "nnz_A": nnz_a, "nnz_L": nnz_l, "precond": "ext_spai", "epsilon": args.epsilon,
                "rtol": args.rtol, "iters_per_solve": it_per_solve, "systems_per_gpu": 1,
                "parallelism": f"independent systems, 1 per GPU x {world}",
            },
            "reference_iters": ref_iters,
            "time_to_rtol_ms": float(np.median(solve_times)) * 1e3,
            "time_to_rtol_variants": variants,
            "gnn_tflops": gnn_fl / float(np.median(gnn_times)) / 1e12,
            "gnn_tflops_frac_of_157": gnn_fl / float(np.median(gnn_times)) / 157.3e12,
            "gnn_flops_per_forward": gnn_fl,
            # the reference's "Total Time" row (infer.py:372-384): precond (GNN) + solve; plus the
            # device Lᵀ / SELL view setup, which the reference does on the host outside its timers
            "total_ms": (float(np.median(solve_times)) + float(np.median(gnn_times)) + prec_s) * 1e3,
            "gnn_precond_ms": float(np.median(gnn_times)) * 1e3,
            "lt_setup_ms": prec_s * 1e3,
            "pcg_iter_us": t_iter * 1e6,
            # SURVEY 8(d) fp64/int32 CSR bytes per iteration / iteration time: the loop READS a
            # lossless compact format (fp32 values, 16-bit columns) and part of its ~200 MB working
            # set stays in the 256 MiB Infinity Cache, so this can exceed HBM-achievable rates --
            # it is a cache-assisted, compact-format figure, not an HBM roofline fraction
            "pcg_alg_GBs": pcg_gbs,
            "pcg_alg_GBs_note": "cache-assisted, compact-format figure (SURVEY 8(d) CSR bytes / iteration time)",
            "roofline": {
                "kernel": kernel,
                "bound": "hbm", "achieved": gbs_cold, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs_cold / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_unit": "bytes per launch (profiles/spmv_traffic.json)",
                "alg_bytes_per_launch": alg, "alg_bytes_formula": alg_formula,
                "avg_launch_ms_cold": ms_cold, "avg_launch_ms_warm": ms_warm,
                "achieved_warm": gbs_warm,
                "csr_staged_ms_cold": csr_cold, "csr_staged_ms_warm": csr_warm,
                "csr_staged_achieved": alg / (csr_cold * 1e-3) / 1e9,
                "method": "cold = a 512 MiB read before every launch; launch time = the SpMV kernel's own start/end stamps (hipExtLaunchKernelGGL events on the ctx stream, the duration rocprofv3's kernel trace reports), averaged over the launches",
            },
            "pcg_loop_spmv": pcg_spmv,
            "solver_views": views,
            "pcg_loop_kernels": loop_dom,
            "cpu_baseline": cpu,
            "c1_synthetic": c1,
            "c5_heat_batch": c5,
            "parity_mode": parity,
            "irregular_1m": irregular,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
