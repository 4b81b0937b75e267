#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python tools/xcd_probe.py > gpurun_out/r2/xcd_probe.json 2> gpurun_out/r2/xcd_probe.err || exit 1
cat gpurun_out/r2/xcd_probe.json
for v in 0 1 0 1; do
LSPCG_SELL_XCD=$v timeout -k 10 300 python bench.py --no-cpu --no-variants --steps 5 > gpurun_out/r2/bench_xcd$v.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r2/bench_xcd$v.json')); print('xcd=$v', round(d['value']), round(d['pcg_iter_us'],2), round(d['roofline']['avg_launch_ms_cold']*1e3,2), round(d['roofline']['frac'],3), d['pcg_loop_kernels']['all_us'])"
done
