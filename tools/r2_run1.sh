#!/bin/bash
# round-2 GPU run: full GPU suite with the parity log, then the bench on kuhn151 with setup profiling
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
export LSPCG_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r2/parity.jsonl
rm -f $LSPCG_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
LSPCG_SETUP_PROFILE=1 timeout -k 10 300 python bench.py --workload kuhn151 --no-cpu --steps 3 --warmup 1 > gpurun_out/r2/kuhn151.json 2> gpurun_out/r2/kuhn151.err || exit 1
LSPCG_SETUP_PROFILE=1 timeout -k 10 300 python bench.py --workload kuhn101 --no-cpu --steps 3 --warmup 1 > gpurun_out/r2/kuhn101.json 2> gpurun_out/r2/kuhn101.err || exit 1
grep "lspcg setup" gpurun_out/r2/*.err
exit $rc
