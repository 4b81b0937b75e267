#!/bin/bash
# GPU evidence run: full GPU suite, smoke, default bench (optionally rocprofv3 kernel stats and
# the roofline SpMV's PMC traffic).  Usage (on the box, via gpurun):
#   bash tools/gpu_suite.sh TAG [tests] [bench] [prof] [traffic] [looptraffic] [gnn] [t=FILES] [ab=JSON]
# Every GPU step runs under its own time limit; the script stops at the first failing step.
set -o pipefail
tag=$1; shift
steps=${*:-tests bench}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
for s in $steps; do
  case $s in
    tests)
      LSPCG_PARITY_LOG=$out/parity_traj.jsonl timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/gpu_tests.txt" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 "$out/gpu_tests.txt"; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit $?
      grep smoke "$out/smoke.txt" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
      python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['value'], d['pcg_iter_us'], d['gnn_precond_ms'], d['roofline']['frac'], d['roofline']['kernel'][:40], d['pcg_loop_kernels']['all_us'])" ;;
    prof)
      bash tools/prof_bench.sh "$tag" || exit $?
      f=$(find "gpurun_out/prof_$tag" -name "*kernel_stats.csv" | head -1); cp "$f" "$out/kernel_stats.csv"
      # the per-dispatch trace is tens of MB: keep the roofline SpMV's launches and the loop's
      python3 tools/trace_split.py "$(find "gpurun_out/prof_$tag" -name "*kernel_trace.csv" | head -1)" > "$out/trace_split.json" 2>&1 || true
      find "gpurun_out/prof_$tag" -name "*kernel_trace.csv" -delete
      python3 -c "import json; d = json.load(open('$out/trace_split.json')); print(json.dumps(d.get('pcg_loop_kernels_us')))" || true ;;
    traffic)
      bash tools/spmv_traffic.sh "$tag" || exit $?
      cat "gpurun_out/traffic_$tag/summary.json" ;;
    looptraffic)  # the PCG loop's five launches: FETCH_SIZE / WRITE_SIZE passes over a short bench
      bash tools/pmc_run.sh "$tag" bench.py --steps 1 --warmup 1 --no-cpu --no-variants -- FETCH_SIZE WRITE_SIZE || exit $?
      python3 tools/loop_traffic.py "$tag" 1 > "$out/pcg_loop_traffic.json" && cat "$out/pcg_loop_traffic.json"
      find "gpurun_out/pmc_$tag" -name "*.csv" -size +2M -delete ;;
    ab=*)  # interleaved loop A/B: ab='{"base": {}, "x": {"ENV": "1"}}'
      LOOP_AB_REPLICAS=${LOOP_AB_REPLICAS:-1} timeout -k 10 600 python -u tools/loop_ab.py "${s#ab=}" kuhn101 ${LOOP_AB_ROUNDS:-11} "$out/loop_ab.jsonl" > "$out/loop_ab.txt" 2>&1 || exit $?
      cat "$out/loop_ab.txt" ;;
    gnn)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_gnn.py -x -q --timeout 200 --timeout-method thread > "$out/gnn_tests.txt" 2>&1
      rc=$?; tail -2 "$out/gnn_tests.txt"; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 120 python -u tools/gnn_run.py --reps 5 > "$out/gnn_run.json" 2> "$out/gnn_run.err" || exit $?
      cat "$out/gnn_run.json"
      (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/gnn_prof" -o gnn -- python3 tools/gnn_run.py --reps 5 > "$out/gnn_prof.log" 2>&1) || exit $?
      f=$(find "$out/gnn_prof" -name "*kernel_stats.csv" | head -1); python3 tools/stats.py "$f" 2>/dev/null | head -20 || head -20 "$f"
      find "$out/gnn_prof" -name "*kernel_trace.csv" -delete ;;
    t=*)  # a subset of the GPU tests: t=tests/test_gpu_sell.py[,tests/...]
      files=$(echo "${s#t=}" | tr ',' ' ')
      timeout -k 10 600 python -u -m pytest $files -m gpu -x -q --timeout 200 --timeout-method thread > "$out/subset_tests.txt" 2>&1
      rc=$?; echo "subset tests rc=$rc"; tail -3 "$out/subset_tests.txt"; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
