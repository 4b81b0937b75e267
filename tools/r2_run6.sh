#!/bin/bash
# full GPU suite, then the default bench (CPU legs included), elasticity and kuhn151 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
export LSPCG_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r2/parity6.jsonl
rm -f $LSPCG_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests6.txt 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python bench.py > gpurun_out/r2/bench6.json 2> gpurun_out/r2/bench6.err || exit 1
timeout -k 10 300 python bench.py --workload elast --no-cpu --steps 3 --warmup 1 > gpurun_out/r2/elast6.json 2> gpurun_out/r2/elast6.err || exit 1
timeout -k 10 300 python bench.py --workload kuhn151 --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/kuhn151_6.json 2> gpurun_out/r2/kuhn151_6.err || exit 1
exit $rc
