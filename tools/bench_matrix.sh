#!/bin/bash
# bench.py over every workload on one box (no CPU leg), one JSON line each, into
# gpurun_out/matrix/; summarise with tools/bench_matrix.sh --summary (CPU side).
set -o pipefail
if [ "$1" == "--summary" ]; then
  python3 - <<'PY'
import glob, json, os
out = []
for f in sorted(glob.glob("gpurun_out/matrix/*.json")):
    d = json.load(open(f))
    c = d["config"]
    out.append({"workload": os.path.basename(f)[:-5], "n": c["n"], "nnz_A": c["nnz_A"], "precond": c["precond"],
                "iters": c["iters_per_solve"], "it_per_s": d["value"], "us_per_iter": d["pcg_iter_us"],
                "time_to_rtol_ms": d["time_to_rtol_ms"], "gnn_ms": d["gnn_precond_ms"], "lt_setup_ms": d["lt_setup_ms"],
                "roofline_frac": d["roofline"]["frac"]})
print(json.dumps(out, indent=1))
PY
  exit 0
fi
mkdir -p gpurun_out/matrix
for W in kuhn101 kuhn151 kuhn201 elast poisson256 kuhn41 synthetic; do
  timeout -k 10 240 python bench.py --workload $W --no-cpu --steps 3 --warmup 1 > gpurun_out/matrix/$W.json 2> gpurun_out/matrix/$W.err || exit 1
  echo "$W done"
done
