#!/bin/bash
# column loads issued before value loads in the SELL / BSELL kernels: parity + timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_configs.py tests/test_gpu_traj.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/t21.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2/t21.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bsell_probe.py > gpurun_out/r2/bsell_probe21.jsonl 2>/dev/null || exit 1
timeout -k 10 200 python tools/bsell_probe.py >> gpurun_out/r2/bsell_probe21.jsonl 2>/dev/null || exit 1
cat gpurun_out/r2/bsell_probe21.jsonl
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --no-variants --steps 5 > gpurun_out/r2/bench21_$i.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r2/bench21_$i.json')); print(round(d['value']), round(d['pcg_iter_us'],2), round(d['roofline']['avg_launch_ms_cold']*1e3,2), round(d['roofline']['frac'],3), {k:round(v,1) for k,v in d['pcg_loop_kernels']['all_us'].items()})"
done
timeout -k 10 300 python bench.py --workload elast --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/elast21.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r2/elast21.json')); print('elast', round(d['value']), round(d['pcg_iter_us'],2), round(d['roofline']['avg_launch_ms_cold']*1e3,2), round(d['roofline']['frac'],3))"
