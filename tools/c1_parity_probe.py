"""BASELINE config 1 (synthetic n = 10,240, CG) in both dot orders: iterations, time to rtol and
per-iteration cost, for rocprofv3 kernel stats of the parity mode's k_dot_openblas launches.

    python tools/c1_parity_probe.py [--reps 3] [--threads 1]
"""
import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=1)
    args = ap.parse_args()
    import torch

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient

    A = sp.csr_matrix(P.synthetic_c1())
    b = torch.from_numpy(A @ np.ones(A.shape[0])).cuda()
    x = torch.zeros_like(b)
    for order in ("compensated", "openblas"):
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="none", dot_order=order,
                                            dot_threads=args.threads)
        ts = []
        for _ in range(args.reps + 1):
            x.zero_()
            it, conv, t = s.solve(b, x, rtol=1e-8)
            ts.append(t)
        med = float(np.median(ts[1:]))
        print(json.dumps({"order": order, "threads": args.threads, "iters": it, "converged": bool(conv),
                          "time_to_rtol_ms": med * 1e3, "us_per_iter": med / it * 1e6}), flush=True)


if __name__ == "__main__":
    main()
