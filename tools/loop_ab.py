#!/usr/bin/env python
"""Interleaved A/B of PCG loop variants on a bench system (measurement only, GPU box).

    python tools/loop_ab.py '{"base": {}, "var": {"LSPCG_X": "1"}}' [workload] [rounds] [out.jsonl]

Builds the workload once (the bench's seeded GNN-L), creates one solver per variant (environment
switches are read at solver creation), then runs `rounds` rounds of one solve per variant in
turn (A B A B ...: box drift hits every variant alike) and reports, per variant, the median
microseconds per iteration, the iteration count and whether x and the residual history are
bit-identical to the first variant's.  With LOOP_AB_KERNELS=1 it also reports the per-launch
times of the loop (lspcg_solver_time_kernels, direct launches); LOOP_AB_MAXIT caps the iterations
of every solve (timing-only variants whose arithmetic is not the solver's); LOOP_AB_REPLICAS = k
times every variant on k solvers (buffer placements) and reports the median over all of them.
"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.data import make_sample
from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace


def main():
    variants = json.loads(sys.argv[1])
    wl = sys.argv[2] if len(sys.argv) > 2 else "kuhn101"
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 9
    out = sys.argv[4] if len(sys.argv) > 4 else None
    A_raw, mask, feats, bs, e2n = P.workload(wl)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs,
                                  seed=0)
    ds = s.to("cuda")
    L, _ = ws.inference_step(ds)
    A = ws.system_matrix(ds)
    b = A.matvec(ds.mask.reshape(-1).to(torch.float64))
    # LOOP_AB_REPLICAS solvers per variant, created interleaved (a1 b1 a2 b2 ...): where a solver's
    # buffers land moves its loop by ~1 us on its own (an A/A pair of one box: 69.0 vs 68.1), so
    # every variant is timed over several placements
    reps = int(os.environ.get("LOOP_AB_REPLICAS", "1"))
    solvers = {k: [] for k in variants}
    base_env = dict(os.environ)
    for _ in range(reps):
        for name, env in variants.items():
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(env)
            sv = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
            sv.set_spai(L, 3e-3, block_size=bs)
            solvers[name].append(sv)
    os.environ.clear()
    os.environ.update(base_env)
    times = {k: [] for k in variants}
    per_rep = {k: [[] for _ in range(reps)] for k in variants}
    res = {}
    for r in range(rounds + 1):
        for i in range(reps):
            for name in variants:
                sv = solvers[name][i]
                x = torch.zeros_like(b)
                it, conv, sec, hist = sv.solve(b, x, rtol=1e-8, max_iter=int(os.environ.get("LOOP_AB_MAXIT", "0")),
                                               return_history=True)
                if r > 0:
                    times[name].append(sec / it * 1e6)
                    per_rep[name][i].append(sec / it * 1e6)
                res[name] = (it, x, hist)
    first = next(iter(variants))
    rows = []
    for name in variants:
        it, x, hist = res[name]
        row = {"workload": wl, "variant": name, "env": variants[name], "iters": it,
               "us_per_iter_median": float(np.median(times[name])), "us_per_iter_min": float(np.min(times[name])),
               "per_solver_median": [float(np.median(v)) for v in per_rep[name]],
               "same_bits_as_" + first: bool(torch.equal(x, res[first][1]) and np.array_equal(hist, res[first][2]))}
        if os.environ.get("LOOP_AB_KERNELS") == "1":
            try:
                row["kernels_us"] = {k: v * 1e6 for k, v in solvers[name][0].time_kernels(b, 40).items()}
            except RuntimeError as e:
                row["kernels_us"] = str(e)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if out:
        with open(out, "a") as f:
            for row in rows:
                f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
