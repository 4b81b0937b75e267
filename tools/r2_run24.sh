#!/bin/bash
# batched lockstep PCG: parity tests + throughput probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r2/t24.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r2/t24.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/batch_probe.py > gpurun_out/r2/batch_probe24.jsonl 2> gpurun_out/r2/batch_probe24.err || exit $?
cat gpurun_out/r2/batch_probe24.jsonl
