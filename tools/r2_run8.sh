#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/t9.txt 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bsell_probe.py > gpurun_out/r2/bsell_probe9.jsonl 2> gpurun_out/r2/bsell_probe9.err || exit 1
timeout -k 10 200 python tools/bsell_probe.py >> gpurun_out/r2/bsell_probe9.jsonl 2>> gpurun_out/r2/bsell_probe9.err || exit 1
timeout -k 10 300 python bench.py --workload elast --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/elast9.json 2> gpurun_out/r2/elast9.err || exit 1
