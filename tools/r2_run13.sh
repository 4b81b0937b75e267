#!/bin/bash
# single-system multi-rank PCG (dist_pcg) on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_pcg.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/t13.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/r2/t13.txt; exit $rc
