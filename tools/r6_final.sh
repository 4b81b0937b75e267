#!/bin/bash
# Round-6 evidence run (GPU box): default bench, its rocprofv3 kernel stats + trace split, the
# delaunay1m loop's PMC bytes, the configs side table.  bash tools/r6_final.sh TAG [steps...]
# steps: bench prof dtraffic configs (default: all).  Every GPU step has its own time limit.
set -o pipefail
tag=$1; shift
steps=${*:-bench prof dtraffic configs}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
for s in $steps; do
  case $s in
    bench)
      timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$out/bench.json')); print('bench', d['value'], d['pcg_iter_us'], d['roofline']['frac'])" ;;
    prof)
      bash tools/prof_bench.sh "$tag" || exit $?
      f=$(find "gpurun_out/prof_$tag" -name "*kernel_stats.csv" | head -1); cp "$f" "$out/kernel_stats.csv"
      python3 tools/trace_split.py "$(find "gpurun_out/prof_$tag" -name "*kernel_trace.csv" | head -1)" > "$out/trace_split.json" 2>&1 || true
      find "gpurun_out/prof_$tag" -name "*kernel_trace.csv" -delete
      python3 -c "import json; d = json.load(open('$out/trace_split.json')); print('trace', json.dumps(d.get('pcg_loop_kernels_us')))" || true ;;
    dtraffic)
      bash tools/pmc_run.sh "d$tag" tools/loop_pmc_run.py delaunay1m 40 -- FETCH_SIZE WRITE_SIZE || exit $?
      python3 tools/loop_traffic.py "d$tag" 18 > "$out/delaunay_loop_traffic.json" && cat "$out/delaunay_loop_traffic.json"
      find "gpurun_out/pmc_d$tag" -name "*.csv" -size +2M -delete ;;
    configs)
      timeout -k 10 900 python -u bench.py --configs > "$out/configs.json" 2> "$out/configs.err" || { tail -5 "$out/configs.err"; exit 1; }
      echo configs ok ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
