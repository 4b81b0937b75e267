#!/bin/bash
# fused 3-launch schedule: full GPU suite, default bench, bench with LSPCG_FUSED3=0, batch probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gpu_tests_v11.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/gpu_tests_v11.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r2/bench_v11.json 2> gpurun_out/r2/bench_v11.err || exit 1
LSPCG_FUSED3=0 timeout -k 10 300 python bench.py --no-cpu --no-variants > gpurun_out/r2/bench_v11_split5.json 2> gpurun_out/r2/bench_v11_split5.err || exit 1
timeout -k 10 300 python tools/batch_probe.py > gpurun_out/r2/batch_probe11.jsonl 2> gpurun_out/r2/batch_probe11.err || exit 1
python3 -c "
import json
for f in ['bench_v11','bench_v11_split5']:
    d=json.load(open('gpurun_out/r2/'+f+'.json')); print(f, round(d['value']), round(d['pcg_iter_us'],2), d['time_to_rtol_ms'], d.get('pcg_loop_kernels',{}).get('all_us'))
"
cat gpurun_out/r2/batch_probe11.jsonl
