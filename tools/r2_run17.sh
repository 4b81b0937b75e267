#!/bin/bash
# BASELINE configurations C2-C5: GPU rows beside the scipy CPU path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 900 python bench.py --configs > gpurun_out/r2/configs_v17.json 2> gpurun_out/r2/configs_v17.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r2/configs_v17.json'))['configs']
for k,v in d.items():
    if k.startswith('C5'): print(k, round(v['gpu_ms_sum'],2), round(v['gpu_ms_max'],2), round(v['cpu_s_sum'],3), round(v['cpu_s_max'],3), [r['iters'] for r in v['systems']], [r['cpu_iters'] for r in v['systems']])
    else: print(k, v['n'], v['iters'], v['cpu_iters'], round(v['gpu_ms'],2), round(v['cpu_s'],3), round(v['gpu_it_per_s']), round(v['cpu_it_per_s']))
"
