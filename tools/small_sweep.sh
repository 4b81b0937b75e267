#!/bin/bash
# k_pcg_small A/B on the GPU box: solve times of the heat_batch8 systems + kuhn41 with the
# one-workgroup solve off (LSPCG_SMALL_N=0) and on up to n = 2560 (LSPCG_SMALL_N=4096).
set -o pipefail
mkdir -p gpurun_out/small
for N in 0 4096; do
  LSPCG_SMALL_N=$N timeout -k 10 200 python tools/solve_overhead.py > gpurun_out/small/overhead_$N.jsonl 2> gpurun_out/small/overhead_$N.err || exit 1
done
