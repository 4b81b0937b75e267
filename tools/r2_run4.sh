#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
LSPCG_PERSIST_STAMPS=1 timeout -k 10 300 python -u tools/persist_probe.py --workloads heat_batch8,poisson256 --reps 1 > gpurun_out/r2/persist_probe4.jsonl 2> gpurun_out/r2/persist_probe4.err
echo "probe rc=$?"
