#!/bin/bash
# round-2 profiles of the default bench: rocprofv3 kernel stats + PMC HBM traffic of the roofline SpMV
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/prof_bench.sh r2 || exit 1
f=$(find gpurun_out/prof_r2 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/prof_r2/kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_r2/kernel_stats.csv')))[:14]: print(r['Name'][:80], r['Calls'], r['AverageNs'])
"
bash tools/spmv_traffic.sh r2 || exit 1
cat gpurun_out/traffic_r2/summary.json
