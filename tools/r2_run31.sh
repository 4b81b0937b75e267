#!/bin/bash
# kernel traces of PCG-IC at kuhn41: sync-free vs per-level triangular solves
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for mode in syncfree levels; do
  mkdir -p gpurun_out/r2/prof31_$mode
  if [ $mode = levels ]; then export LSPCG_TRSV_LEVELS=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof31_$mode -o ic -- python3 tools/ic_probe.py kuhn41 > gpurun_out/r2/ic31_$mode.txt 2>&1 || exit $?
  grep '"w"' gpurun_out/r2/ic31_$mode.txt
  f=$(find gpurun_out/r2/prof31_$mode -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]: print(r['Name'][:90], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
"
done
