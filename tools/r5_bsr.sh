#!/bin/bash
# BSR 3x3 (C4 elasticity) A/B: standalone BSELL sweep (1 vs 3 waves per slice), then the C4 bench
# with each kernel, then the BSR-touching GPU tests.  Usage (on the box): bash tools/r5_bsr.sh TAG
set -o pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 300 python -u tools/sell_sweep.py --bsr > "$out/bsr_sweep.jsonl" 2> "$out/bsr_sweep.err" || exit $?
cat "$out/bsr_sweep.jsonl"
for wv in 1 3 1 3; do
  LSPCG_BSELL_WAVES=$wv timeout -k 10 300 python -u bench.py --workload elast --steps 3 --warmup 1 --no-cpu --no-variants \
    > "$out/bench_elast_w$wv.json" 2>> "$out/bench.err" || exit $?
  python3 -c "
import json; d=json.load(open('$out/bench_elast_w$wv.json')); print('waves $wv', d['value'], d['pcg_iter_us'], d['roofline']['frac'], d['roofline'].get('kernel'), d['pcg_loop_kernels'].get('all_us'))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_sell.py tests/test_gpu_batch.py tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.txt" 2>&1
rc=$?; tail -3 "$out/tests.txt"; exit $rc
