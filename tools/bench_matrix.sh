#!/bin/bash
# bench.py over every workload on one box (no CPU leg), one JSON line each, into
# gpurun_out/matrix/; summarise with tools/bench_matrix.sh --summary (CPU side).
set -o pipefail
if [ "$1" == "--summary" ]; then
  # --summary [BASELINE.json]: print the matrix; with a baseline matrix (an earlier summary, e.g.
  # profiles/r1_bench_matrix_v12.json) flag every field that moved more than 10 % the wrong way
  BASE="$2" python3 - <<'PY'
import glob, json, os, sys
out = []
for f in sorted(glob.glob("gpurun_out/matrix/*.json")):
    d = json.load(open(f))
    c = d["config"]
    out.append({"workload": os.path.basename(f)[:-5], "n": c["n"], "nnz_A": c["nnz_A"], "precond": c["precond"],
                "iters": c["iters_per_solve"], "it_per_s": d["value"], "us_per_iter": d["pcg_iter_us"],
                "time_to_rtol_ms": d["time_to_rtol_ms"], "gnn_ms": d["gnn_precond_ms"], "lt_setup_ms": d["lt_setup_ms"],
                "roofline_frac": d["roofline"]["frac"]})
print(json.dumps(out, indent=1))
base = os.environ.get("BASE")
if base:
    higher_better = {"it_per_s", "roofline_frac"}
    lower_better = {"us_per_iter", "time_to_rtol_ms", "gnn_ms", "lt_setup_ms", "iters"}
    ref = {r["workload"]: r for r in json.load(open(base))}
    bad = []
    for r in out:
        b = ref.get(r["workload"])
        if not b:
            continue
        for k in higher_better | lower_better:
            if k not in b or not b[k] or r.get(k) is None:
                continue
            ratio = r[k] / b[k]
            if (k in higher_better and ratio < 0.9) or (k in lower_better and ratio > 1.1):
                bad.append(f"{r['workload']}.{k}: {b[k]:.4g} -> {r[k]:.4g} ({ratio:.2f}x)")
    print("REGRESSIONS (> 10 %) vs " + base + ":" if bad else "no field regressed by more than 10 % vs " + base)
    for line in bad:
        print("  " + line)
    sys.exit(1 if bad else 0)
PY
  exit $?
fi
mkdir -p gpurun_out/matrix
# WORKLOADS (env, optional): another list, e.g. WORKLOADS="kuhn61 kuhn81" EXTRA="--no-variants"
for W in ${WORKLOADS:-kuhn101 kuhn101rcm kuhn101rand kuhn151 kuhn201 elast poisson256 kuhn41 synthetic}; do
  timeout -k 10 240 python bench.py --workload $W --no-cpu --steps 3 --warmup 1 $EXTRA > gpurun_out/matrix/$W.json 2> gpurun_out/matrix/$W.err || exit 1
  echo "$W done"
done
