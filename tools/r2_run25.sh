#!/bin/bash
# kernel trace of the batched lockstep solve, one rocprofv3 pass per batch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for set in heat_batch8 poisson256x8; do
  mkdir -p gpurun_out/r2/prof25_$set
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof25_$set -o batch -- python3 tools/batch_kernels.py $set > gpurun_out/r2/batch_kernels25_$set.txt 2>&1 || exit $?
  grep set gpurun_out/r2/batch_kernels25_$set.txt
  f=$(find gpurun_out/r2/prof25_$set -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:12]: print(r['Name'][:120], r['Calls'], r['AverageNs'])
"
done
