#!/bin/bash
# one-wave consumer sums up to 512 partials: parity subset + elast / kuhn41 / poisson256 groups vs auto
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_traj.py tests/test_gpu_configs.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t38.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2/t38.txt; [ $rc -eq 0 ] || exit $rc
for w in elast kuhn41 poisson256; do
  for mode in 1 auto; do
    if [ $mode = auto ]; then unset LSPCG_SPLIT_REDUCE; else export LSPCG_SPLIT_REDUCE=$mode; fi
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/b38_${w}_$mode.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r2/b38_${w}_$mode.json')); print('$w', 'mode $mode', round(d['pcg_iter_us'],2), d['config']['iters_per_solve'])"
  done
done
