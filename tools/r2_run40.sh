#!/bin/bash
# auto no-group reductions for mid-size grids: parity subset + mid-size and headline timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_traj.py tests/test_gpu_fuzz.py tests/test_gpu_golden.py tests/test_gpu_linalg.py tests/test_gpu_configs.py tests/test_gpu_dist_pcg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t40.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/t40.txt; [ $rc -eq 0 ] || exit $rc
for w in poisson256 kuhn41 kuhn101; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu --no-variants --steps 5 > gpurun_out/r2/b40_$w.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r2/b40_$w.json')); print('$w', round(d['pcg_iter_us'],2), d['config']['iters_per_solve'])"
done
timeout -k 10 300 python -u tools/batch_probe.py > gpurun_out/r2/batch_probe40.jsonl 2>/dev/null || exit $?
grep '"threads": 1,' gpurun_out/r2/batch_probe40.jsonl
