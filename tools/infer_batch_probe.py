"""infer.run on the C5 heat batch: one system at a time (the reference's loop), 4 solves in flight,
and windows of 8 (one GNN forward + one batched solve per window): host wall of the whole run and
the per-record mean GNN / solve times."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from learningsparsepreconditioner4gpu_amd.infer import run, synthetic_dataset  # noqa: E402
from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace  # noqa: E402


def main():
    samples = synthetic_dataset("heat_batch8")
    ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=1, seed=0)
    run(samples, ws, rtol=1e-8, warmup=2)  # warm everything
    for label, kw in (("sequential", {}), ("concurrency4", {"concurrency": 4}), ("batch8", {"batch": 8})):
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            recs = run(samples, ws, rtol=1e-8, warmup=1, **kw)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if best is None or dt < best[0]:
                best = (dt, recs)
        dt, recs = best
        print(json.dumps({"mode": label, "wall_ms": dt * 1e3, "gnn_ms_mean": 1e3 * sum(r.t_prec for r in recs) / len(recs),
                          "solve_ms_mean": 1e3 * sum(r.t_solve for r in recs) / len(recs),
                          "iters": [int(r.iters) for r in recs]}), flush=True)


if __name__ == "__main__":
    main()
