#!/bin/bash
# Device RCM evidence: the reorder tests (exact order vs the sequential restatement) and the
# irregular rows of the bench (solver setup with the analysis).  Usage: bash tools/r5_rcm.sh TAG
set -o pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_reorder.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/reorder_tests.txt" 2>&1
rc=$?; tail -3 "$out/reorder_tests.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > "$out/bench.json" 2> "$out/bench.err" || exit $?
python3 -c "
import json; d=json.load(open('$out/bench.json'))
for k, r in d['irregular_1m'].items(): print(k, r['solver_reorder'], r['solver_setup_ms'], r['pcg_iter_us'], r['iters'])"
