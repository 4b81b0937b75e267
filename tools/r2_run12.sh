#!/bin/bash
# concurrent solves in the product (infer.run concurrency, linalg.solve_many) + bench C5 row
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_linalg.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/t12.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/t12.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r2/bench_v12.json 2> gpurun_out/r2/bench_v12.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r2/bench_v12.json')); print(round(d['value']), round(d['pcg_iter_us'],2), json.dumps(d['c5_heat_batch']))
"
