#!/bin/bash
# GNN: encoder fused into layer 1 -- parity tests, A/B timing, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/t15.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/t15.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/gnn_run.py --reps 10 > gpurun_out/r2/gnn_fused.json 2>/dev/null || exit 1
LSPCG_GNN_NO_FUSE=1 timeout -k 10 120 python tools/gnn_run.py --reps 10 > gpurun_out/r2/gnn_nofuse.json 2>/dev/null || exit 1
cat gpurun_out/r2/gnn_fused.json gpurun_out/r2/gnn_nofuse.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_gnn15 -o run -- python3 tools/gnn_run.py --reps 5 > /dev/null 2>&1 || exit 1
find gpurun_out/r2/prof_gnn15 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r2/gnn15_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/r2/gnn15_kernel_stats.csv')))[:10]: print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
