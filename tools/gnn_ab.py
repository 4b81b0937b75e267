"""Interleaved A/B of GNN builds (measurement only, GPU box): each variant is a library path
(LSPCG_LIB) or "" for the in-tree build; `rounds` rounds run tools/gnn_run.py once per variant
in turn, each in its own process, and the median forward_ms / wall_ms per variant is printed,
with the max |difference| of its GNN output vs the first variant's.

    python tools/gnn_ab.py '{"base": "", "gs": "exp/liblspcg_gs.so"}' [rounds] [out.jsonl]
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def main():
    variants = json.loads(sys.argv[1])
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    out = sys.argv[3] if len(sys.argv) > 3 else None
    runs = {k: [] for k in variants}
    for r in range(rounds):
        for name, lib in variants.items():
            env = dict(os.environ)
            if lib:
                env["LSPCG_LIB"] = str(ROOT / lib)
            dump = f"/tmp/gnn_ab_{name}.npy" if r == 0 else ""
            cmd = [sys.executable, "-u", str(ROOT / "tools" / "gnn_run.py"), "--reps", "5"]
            if dump:
                cmd += ["--dump", dump]
            res = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
            if res.returncode:
                sys.stderr.write(res.stderr[-2000:])
                sys.exit(res.returncode)
            runs[name].append(json.loads(res.stdout.strip().splitlines()[-1]))
            print(name, runs[name][-1], flush=True)
    first = next(iter(variants))
    ref = np.load(f"/tmp/gnn_ab_{first}.npy")
    rows = []
    for name in variants:
        o = np.load(f"/tmp/gnn_ab_{name}.npy")
        rows.append({"variant": name, "lib": variants[name],
                     "forward_ms_median": float(np.median([x["forward_ms"] for x in runs[name]])),
                     "wall_ms_median": float(np.median([x["wall_ms"] for x in runs[name]])),
                     "max_abs_diff_vs_" + first: float(np.max(np.abs(o - ref))),
                     "max_abs_out": float(np.max(np.abs(ref)))})
        print(json.dumps(rows[-1]), flush=True)
    if out:
        with open(out, "a") as f:
            for row in rows:
                f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
