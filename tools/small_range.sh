#!/bin/bash
# One-workgroup solve vs the 5-kernel schedule across its n range (R = 1, 2, 5 rows per thread):
# default bench on small Kuhn grids with LSPCG_SMALL_N=0 and default.
set -o pipefail
mkdir -p gpurun_out/small_range
for W in kuhn8 kuhn10 kuhn12 kuhn13; do
  for N in 0 4096; do
    LSPCG_SMALL_N=$N timeout -k 10 120 python bench.py --workload $W --no-cpu --steps 5 --warmup 2 --spmv-reps 5 > gpurun_out/small_range/${W}_$N.json 2> gpurun_out/small_range/${W}_$N.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/small_range/${W}_$N.json'));print('$W', $N, d['config']['n'], d['config']['iters_per_solve'], round(d['pcg_iter_us'],2))"
  done
done
