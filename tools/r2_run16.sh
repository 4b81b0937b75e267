#!/bin/bash
# full GPU suite + smoke + default bench + rocprofv3 kernel stats of the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/gpu_tests_v16.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/gpu_tests_v16.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke_v16.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r2/bench_v16.json 2> gpurun_out/r2/bench_v16.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r2/bench_v16.json')); print(round(d['value']), round(d['pcg_iter_us'],2), d['roofline']['frac'], d['gnn_precond_ms'], d['total_ms'])
"
