#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2/prof41
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof41 -o ainv -- python3 tools/ainv_probe.py kuhn41 > gpurun_out/r2/ainv41.txt 2>&1 || exit $?
grep ainv_setup gpurun_out/r2/ainv41.txt
f=$(find gpurun_out/r2/prof41 -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:10]: print(r['Name'][:80], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
"
