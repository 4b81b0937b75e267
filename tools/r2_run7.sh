#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
rm -f gpurun_out/r2/bsell_probe.jsonl
for q in 1 2 4; do
  LSPCG_BSELL_QB=$q timeout -k 10 200 python tools/bsell_probe.py >> gpurun_out/r2/bsell_probe.jsonl 2>> gpurun_out/r2/bsell_probe.err || exit 1
done
for q in 2 4; do
  LSPCG_BSELL_QB=$q timeout -k 10 300 python bench.py --workload elast --no-cpu --no-variants --steps 3 --warmup 1 > gpurun_out/r2/elast7_q$q.json 2> gpurun_out/r2/elast7_q$q.err || exit 1
done
