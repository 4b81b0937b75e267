#!/bin/bash
# elementwise launches with 4 vectors per thread (kElemUnroll = 4): parity subset + timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_traj.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t53.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r2/t53.txt; [ $rc -eq 0 ] || exit $rc
for w in kuhn101 poisson256 elast; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu --no-variants --steps 5 --warmup 1 > gpurun_out/r2/b53_$w.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r2/b53_$w.json')); print('$w', round(d['pcg_iter_us'],2), {k: round(v,1) for k,v in d['pcg_loop_kernels']['all_us'].items()})"
done
