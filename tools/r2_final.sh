#!/bin/bash
# round-2 final evidence: full GPU suite, smoke, default bench, rocprofv3 kernel stats of the
# default bench, PMC HBM traffic of the roofline SpMV
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/final/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.txt 2>&1 || exit $?
grep smoke gpurun_out/final/smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/final/bench.json')); print(d['value'], d['pcg_iter_us'], d['roofline']['frac'], d['c5_heat_batch']['batched'])"
bash tools/prof_bench.sh final || exit $?
f=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/final/kernel_stats.csv
bash tools/spmv_traffic.sh final || exit $?
cat gpurun_out/traffic_final/summary.json
