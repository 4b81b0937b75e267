#!/bin/bash
# one-workgroup solve at 1024 threads for 1024 < n <= 2560: parity + range sweep (5-kernel / 512x5 / 1024x2-3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2/small37
timeout -k 10 400 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_fuzz.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t37.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2/t37.txt; [ $rc -eq 0 ] || exit $rc
for W in kuhn10 kuhn11 kuhn12 kuhn13; do
  for cfg in "0 1" "4096 0" "4096 1"; do
    set -- $cfg
    LSPCG_SMALL_N=$1 LSPCG_SMALL_BIG=$2 timeout -k 10 120 python bench.py --workload $W --no-cpu --no-variants --steps 5 --warmup 2 --spmv-reps 5 > gpurun_out/r2/small37/${W}_$1_$2.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r2/small37/${W}_$1_$2.json'));print('$W', 'small_n=$1 big=$2', d['config']['n'], d['config']['iters_per_solve'], round(d['pcg_iter_us'],2))"
  done
done
