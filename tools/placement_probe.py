"""Measurement only (GPU box): how much a locality-improving placement could gain on the unstructured
Delaunay system.  The named workload is renumbered by a Morton (z-order) curve over its vertex
coordinates -- an upper bound for what a coordinate-free placement could reach -- and bench.irregular_row
runs on it (GNN-L, the loop, the standalone SpMV), one JSON line each.

    python tools/placement_probe.py delaunay1m [delaunay64k ...]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from learningsparsepreconditioner4gpu_amd import problems as P  # noqa: E402


def morton_perm(nodes: np.ndarray, bits: int = 10) -> np.ndarray:
    lo, hi = nodes.min(0), nodes.max(0)
    q = np.minimum(((nodes - lo) / (hi - lo + 1e-12) * (1 << bits)).astype(np.int64), (1 << bits) - 1)
    key = np.zeros(len(nodes), np.int64)
    for b in range(bits):
        for d in range(3):
            key |= ((q[:, d] >> b) & 1) << (3 * b + d)
    return np.argsort(key, kind="stable")


def main():
    base = P.workload
    for wl in sys.argv[1:] or ["delaunay1m"]:
        A, mask, nodes, bs, e2n = base(wl)
        perm = morton_perm(np.asarray(nodes)[:, :3])
        B = sp.csr_matrix(sp.csr_matrix(A)[perm][:, perm])
        B.sort_indices()
        name = wl + "_morton"
        P.workload = lambda n, _r=(B, mask[perm], nodes[perm], bs, e2n), _name=name: _r if n == _name else base(n)
        t0 = time.time()
        row = bench.irregular_row(name, 3e-3, 1e-8, 30)
        row["probe_wall_s"] = time.time() - t0
        print(json.dumps({name: row}), flush=True)
        P.workload = base


if __name__ == "__main__":
    main()
