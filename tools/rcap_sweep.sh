set -o pipefail
mkdir -p gpurun_out/rcap
for X in 1536 1342 1024 2013 4025 1536; do
  LSPCG_SELL_RCAP=$X timeout -k 10 150 python bench.py --no-cpu --steps 5 --warmup 2 --spmv-reps 5 > gpurun_out/rcap/b_$X.json 2> gpurun_out/rcap/b_$X.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/rcap/b_$X.json'));print($X, round(d['pcg_iter_us'],2), {k:round(v,1) for k,v in d['pcg_loop_kernels']['all_us'].items()})"
done
