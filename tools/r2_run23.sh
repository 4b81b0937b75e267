#!/bin/bash
# session-3 baseline: full GPU suite, smoke, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t23.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2/t23.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke23.txt 2>&1 || exit $?
cat gpurun_out/r2/smoke23.txt
timeout -k 10 200 python -u bench.py > gpurun_out/r2/bench23.json 2> gpurun_out/r2/bench23.err || exit $?
cat gpurun_out/r2/bench23.json
