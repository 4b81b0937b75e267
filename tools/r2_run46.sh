#!/bin/bash
# BSELL-64 software pipeline: BSR parity + elasticity roofline / loop
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_sell.py tests/test_gpu_batch.py tests/test_gpu_linalg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t46.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2/t46.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload elast --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/elast46_$i.json 2>/dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r2/elast46_$i.json')); r=d['roofline']; print('elast', round(d['pcg_iter_us'],2), round(r['frac'],3), round(r['avg_launch_ms_cold']*1e3,2), {k: round(v,1) for k,v in d['pcg_loop_kernels']['all_us'].items()})"
done
