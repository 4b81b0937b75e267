#!/bin/bash
# concurrent independent solves probe + bench matrix (lt_setup regression check vs r1 v12)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python tools/batch_probe.py > gpurun_out/r2/batch_probe10.jsonl 2> gpurun_out/r2/batch_probe10.err || exit 1
cat gpurun_out/r2/batch_probe10.jsonl
timeout -k 10 900 tools/bench_matrix.sh || exit 1
