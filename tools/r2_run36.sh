#!/bin/bash
# batched solve v2 (per-system last-arriver reductions): parity tests, probe, kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r2/t36.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -9 gpurun_out/r2/t36.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/batch_probe.py > gpurun_out/r2/batch_probe36.jsonl 2> gpurun_out/r2/batch_probe36.err || exit $?
grep batch gpurun_out/r2/batch_probe36.jsonl
for set in heat_batch8 poisson256x8; do
  mkdir -p gpurun_out/r2/prof36_$set
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof36_$set -o batch -- python3 tools/batch_kernels.py $set > gpurun_out/r2/batch_kernels36_$set.txt 2>&1 || exit $?
  grep set gpurun_out/r2/batch_kernels36_$set.txt
  f=$(find gpurun_out/r2/prof36_$set -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:6]: print(r['Name'][:100], r['Calls'], r['AverageNs'])
"
done
