#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_pcg.py tests/test_gpu_linalg.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t22.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2/t22.txt; exit $rc
