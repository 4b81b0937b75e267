#!/bin/bash
# UP / UR at 1 M rows: 1006 workgroups x 2 vectors per thread vs 2012 x 1 (LSPCG_ELEM_WIDE=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
for rep in 1 2; do
for wide in 0 1; do
  LSPCG_ELEM_WIDE=$wide timeout -k 10 300 python -u bench.py --no-cpu --no-variants --steps 5 --warmup 2 > gpurun_out/r2/b52_${wide}_$rep.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r2/b52_${wide}_$rep.json')); print('wide $wide', round(d['pcg_iter_us'],2), {k: round(v,1) for k,v in d['pcg_loop_kernels']['all_us'].items()})"
done
done
