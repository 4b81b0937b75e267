#!/usr/bin/env python
"""Measurement aid: the process's library layout under the same launcher as a crashed run.

Imports what bench.py imports, runs a few concurrent solves (linalg.solve_many, the bench's
c5 leg) and writes /proc/self/maps plus the load address of liblspcg_hip.so to
``--out``.  tools/symbolize.py maps the frames of a crash log onto these libraries (anchored on
libc's ``__restore_rt`` frame for the libraries loaded at start-up and on liblspcg_hip.so for the
ones loaded with torch), then resolves them with the symbol tables of this image's libraries.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import numpy as np
    import torch

    torch.cuda.set_device(0)
    from learningsparsepreconditioner4gpu_amd import _lib
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient, solve_many

    A, _mask, _f = P.poisson2d_grid(64, 64)
    jobs = []
    for _ in range(4):
        s = PreconditionedConjugateGradient(A, device="cuda", preconditioner="diagonal", dtype=np.float64)
        b = torch.ones(A.shape[0], dtype=torch.float64, device="cuda")
        jobs.append((s, b, torch.zeros_like(b)))
    solve_many(jobs, 1e-8, concurrency=4)
    torch.cuda.synchronize()
    lib = _lib.load()
    addr = ctypes.cast(lib.lspcg_solver_solve, ctypes.c_void_p).value
    with open(args.out, "w") as f:
        f.write(f"# lspcg_solver_solve {addr:#x}\n")
        f.write(open("/proc/self/maps").read())
    print("maps written", args.out, flush=True)


if __name__ == "__main__":
    main()
