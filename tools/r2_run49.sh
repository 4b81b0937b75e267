#!/bin/bash
# elementwise launches with one vector per thread for mid-size n: parity subset + A/B timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_traj.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t49.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2/t49.txt; [ $rc -eq 0 ] || exit $rc
for w in poisson256 kuhn41 elast; do
  for mode in 0 1; do
    LSPCG_ELEM_ONE=$mode timeout -k 10 300 python -u bench.py --workload $w --no-cpu --no-variants --steps 5 --warmup 1 > gpurun_out/r2/b49_${w}_$mode.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r2/b49_${w}_$mode.json')); print('$w', 'one=$mode', round(d['pcg_iter_us'],2))"
  done
done
