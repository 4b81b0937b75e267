#!/bin/bash
# KA (non-reducing SELL launches) grid cap sweep at kuhn101 (LSPCG_SELL_NCAP)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
for cap in none 1536 2048 3072; do
  if [ $cap = none ]; then unset LSPCG_SELL_NCAP; else export LSPCG_SELL_NCAP=$cap; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-variants --steps 5 --warmup 2 > gpurun_out/r2/b51_$cap.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r2/b51_$cap.json')); print('ncap $cap', round(d['pcg_iter_us'],2), {k: round(v,1) for k,v in d['pcg_loop_kernels']['all_us'].items()})"
done
