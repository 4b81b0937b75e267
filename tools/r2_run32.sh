#!/bin/bash
# sync-free trsv: workgroups per CU sweep (kernel trace at kuhn41) + IC timings at kuhn41 / kuhn101
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for wpc in 1; do
  mkdir -p gpurun_out/r2/prof32_$wpc
  LSPCG_TRSV_WG_PER_CU=$wpc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof32_$wpc -o ic -- python3 tools/ic_probe.py kuhn41 > gpurun_out/r2/ic32_$wpc.txt 2>&1 || exit $?
  f=$(find gpurun_out/r2/prof32_$wpc -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:2]: print('wpc $wpc', r['Name'][:50], r['Calls'], r['AverageNs'])
"
done
timeout -k 10 300 python -u tools/ic_probe.py kuhn101 || exit $?
