#!/bin/bash
# Round-2 session 2 baseline: full GPU suite, smoke, default bench, rocprofv3 stats of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gpu_tests_v9.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/gpu_tests_v9.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke_v9.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r2/bench_v9.json 2> gpurun_out/r2/bench_v9.err || exit 1
cat gpurun_out/r2/bench_v9.json
