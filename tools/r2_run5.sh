#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -k "pcg_sell_equals or persist" > gpurun_out/r2/t5_sell.txt 2>&1
rc=$?; echo "sell rc=$rc"; [ $rc -ne 0 ] && exit $rc
LSPCG_PERSIST_STAMPS=1 timeout -k 10 300 python -u tools/persist_probe.py --workloads heat_batch8,poisson256 --reps 1 > gpurun_out/r2/persist_probe5s.jsonl 2> gpurun_out/r2/persist_probe5s.err || exit 1
timeout -k 10 300 python -u tools/persist_probe.py --workloads heat_batch8,poisson256,kuhn41 > gpurun_out/r2/persist_probe5.jsonl 2> gpurun_out/r2/persist_probe5.err
echo "probe rc=$?"
