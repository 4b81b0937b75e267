"""bench.irregular_row on named workloads (measurement only, GPU box): the GNN-L ext_spai loop,
its views / reorder decision, per-launch loop times and the standalone SpMV, one JSON line each.

    python tools/irregular_probe.py delaunay1m [delaunay64k kuhn101rcm ...]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    for wl in sys.argv[1:] or ["delaunay1m"]:
        t0 = time.time()
        bench.log(f"{wl}: start")
        row = bench.irregular_row(wl, 3e-3, 1e-8, 30)
        row["probe_wall_s"] = time.time() - t0
        print(json.dumps({wl: row}), flush=True)


if __name__ == "__main__":
    main()
