#!/bin/bash
# batch wired into infer / bench: tests + default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t28.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2/t28.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r2/bench28.json 2> gpurun_out/r2/bench28.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r2/bench28.json')); print(d['value'], d['roofline']['frac']); print(json.dumps(d['c5_heat_batch']))"
