#!/bin/bash
# Process-to-process spread of the kuhn101 loop with and without A's one-byte value codes
# (LSPCG_VALUE_CODES=1: A's loop bytes 61 -> 15 MB, the working set ~236 -> ~191 MB against the
# 256 MiB Infinity Cache).  Alternating processes.  Usage: bash tools/r5_codes_var.sh TAG [ROUNDS]
set -o pipefail
tag=$1
rounds=${2:-4}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
for r in $(seq 1 $rounds); do
  for v in 0 1; do
    LSPCG_VALUE_CODES=$v timeout -k 10 200 python -u bench.py --workload kuhn101 --no-cpu --steps 10 --warmup 2 --no-variants > "$out/codes${v}_$r.json" 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('$out/codes${v}_$r.json')); k=d['pcg_loop_kernels']['all_us']
print(json.dumps({'codes': $v, 'round': $r, 'us_iter': round(d['pcg_iter_us'], 2), 'kernels': {a: round(b, 2) for a, b in k.items()}}))" | tee -a "$out/codes_var.jsonl"
  done
done
