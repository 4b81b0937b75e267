#!/bin/bash
# state reads overlapped with the first loads: parity subset + loop timings + batch probe + C2/C4 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_traj.py tests/test_gpu_batch.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t29.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/t29.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-variants --steps 5 > gpurun_out/r2/bench29_$i.json 2>/dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r2/bench29_$i.json')); print('kuhn101', round(d['value']), round(d['pcg_iter_us'],1), d['pcg_loop_kernels']['all_us'], d['c5_heat_batch']['batched']['us_per_lockstep_iter'], d['c5_heat_batch']['concurrency_1']['us_per_iter_per_system'])"
done
timeout -k 10 300 python -u bench.py --workload elast --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/elast29.json 2>/dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r2/elast29.json')); print('elast', round(d['value']), round(d['pcg_iter_us'],1), d['pcg_loop_kernels']['all_us'])"
timeout -k 10 300 python -u bench.py --workload poisson256 --no-cpu --no-variants --steps 5 > gpurun_out/r2/poisson29.json 2>/dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r2/poisson29.json')); print('poisson256', round(d['value']), round(d['pcg_iter_us'],1), d['pcg_loop_kernels']['all_us'])"
