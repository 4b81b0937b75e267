#!/bin/bash
# round-2 GPU run 2: persistent solve + GraphSpmv/AATPE parity, then the persistent-vs-split probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
export LSPCG_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r2/parity2.jsonl
rm -f $LSPCG_PARITY_LOG
timeout -k 10 300 python -u -m pytest tests/test_gpu_sell.py -x -v --timeout 120 --timeout-method thread -k "pcg_sell_equals" > gpurun_out/r2/t_sell.txt 2>&1
rc=$?; echo "sell rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_traj.py tests/test_gpu_fuzz.py tests/test_gpu_graph.py tests/test_gpu_golden.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/t_more.txt 2>&1
rc=$?; echo "more rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/persist_probe.py > gpurun_out/r2/persist_probe.jsonl 2> gpurun_out/r2/persist_probe.err
echo "probe rc=$?"
