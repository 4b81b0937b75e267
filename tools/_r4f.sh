set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4f; mkdir -p $out
bash tools/prof_bench.sh r4f || exit $?
f=$(find gpurun_out/prof_r4f -name "*kernel_stats.csv" | head -1); cp "$f" $out/kernel_stats.csv
python3 tools/trace_split.py "$(find gpurun_out/prof_r4f -name "*kernel_trace.csv" | head -1)" > $out/trace_split.json 2>&1 || true
find gpurun_out/prof_r4f -name "*kernel_trace.csv" -delete
python3 -c "
import json; d=json.load(open('$out/trace_split.json')); print(json.dumps(d['pcg_loop_kernels_us'])); print(d['sell'])"
bash tools/spmv_traffic.sh r4f || exit $?
cat gpurun_out/traffic_r4f/summary.json
bash tools/pmc_run.sh r4f bench.py --steps 1 --warmup 1 --no-cpu --no-variants -- FETCH_SIZE WRITE_SIZE || exit $?
python3 tools/loop_traffic.py r4f 1 > $out/pcg_loop_traffic.json && cat $out/pcg_loop_traffic.json
find gpurun_out/pmc_r4f gpurun_out/traffic_r4f -name "*.csv" -size +2M -delete
