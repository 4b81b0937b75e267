#!/bin/bash
# mid-size single solves: split groups (default) vs consumers summing every workgroup partial
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
for mode in 1 2; do
  for w in poisson256 kuhn41; do
    LSPCG_SPLIT_REDUCE=$mode timeout -k 10 300 python -u bench.py --workload $w --no-cpu --no-variants --steps 5 > gpurun_out/r2/sr34_${mode}_$w.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r2/sr34_${mode}_$w.json')); print('mode $mode', '$w', round(d['pcg_iter_us'],2), d['config']['iters_per_solve'])"
  done
done
