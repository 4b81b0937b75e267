#!/bin/bash
# BSELL-DIA (BSR 3x3 SELL-DIA) evidence: BSR parity tests, C4 loop A/B against BSELL-64, the C4
# standalone SpMV roofline line.  Usage (on the box, via gpurun): bash tools/r5_bsdia.sh TAG
set -o pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_configs.py tests/test_gpu_linalg.py \
  tests/test_gpu_reorder.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/bsr_tests.txt" 2>&1
rc=$?; tail -3 "$out/bsr_tests.txt"; [ $rc -eq 0 ] || exit $rc
LOOP_AB_KERNELS=1 LOOP_AB_REPLICAS=2 timeout -k 10 400 python -u tools/loop_ab.py '{"bsdia": {}, "bsell": {"LSPCG_BSDIA": "0"}}' elast 7 "$out/c4_loop_ab.jsonl" > "$out/c4_loop_ab.txt" 2>&1
rc=$?; cat "$out/c4_loop_ab.txt" | tail -20; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  LSPCG_BSDIA=$v timeout -k 10 300 python -u bench.py --workload elast --steps 3 --warmup 1 --no-cpu --no-variants > "$out/bench_elast_bsdia$v.json" 2> "$out/bench_elast_bsdia$v.err" || exit $?
  python3 -c "
import json; d=json.load(open('$out/bench_elast_bsdia$v.json')); r=d['roofline']; print('bsdia=$v', d['value'], d['pcg_iter_us'], r['frac'], r['avg_launch_ms_cold'], r['kernel'][:30])"
done
