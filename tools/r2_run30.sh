#!/bin/bash
# sync-free triangular solves: precond parity + IC timings (sync-free vs per-level launches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_precond.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/t30.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/t30.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/baseline_probe.py > gpurun_out/r2/baseline30_syncfree.jsonl 2>&1 || exit $?
grep '"ic"' gpurun_out/r2/baseline30_syncfree.jsonl
LSPCG_TRSV_LEVELS=1 timeout -k 10 300 python -u tools/baseline_probe.py > gpurun_out/r2/baseline30_levels.jsonl 2>&1 || exit $?
grep '"ic"' gpurun_out/r2/baseline30_levels.jsonl
