#!/bin/bash
# multi-rank rehearsal on ONE GPU: bench.py and infer under torchrun, 2 ranks, gloo backend
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
export LSPCG_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-variants > gpurun_out/r2/bench_torchrun2_gloo.json 2> gpurun_out/r2/bench_torchrun2_gloo.err || exit 1
cat gpurun_out/r2/bench_torchrun2_gloo.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','n_gpus','ms_per_step','scaling')}, d['config']['parallelism'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29732 -m learningsparsepreconditioner4gpu_amd.infer --dataset heat_batch8 --rtol 1e-8 --baselines none --warmup 2 --out-dir gpurun_out/r2/infer2 --concurrency 2 > gpurun_out/r2/infer_torchrun2_gloo.txt 2>&1 || exit 1
tail -12 gpurun_out/r2/infer_torchrun2_gloo.txt
ls gpurun_out/r2/infer2
