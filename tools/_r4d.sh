set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4d; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?; tail -3 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/loop_ab.py '{"base": {}, "ntx": {"LSPCG_EXP": "1"}}' kuhn101 9 $out/loop_ab.jsonl > $out/loop_ab.txt 2>&1 || exit $?
cat $out/loop_ab.txt
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['value'], d['pcg_iter_us'], d['gnn_precond_ms'], d['roofline']['frac'], d['reference_iters'], d['parity_mode'], d['irregular_1m'])"
bash tools/prof_bench.sh r4d || exit $?
f=$(find gpurun_out/prof_r4d -name "*kernel_stats.csv" | head -1); cp "$f" $out/kernel_stats.csv
python3 tools/trace_split.py "$(find gpurun_out/prof_r4d -name "*kernel_trace.csv" | head -1)" > $out/trace_split.json 2>&1 || true
find gpurun_out/prof_r4d -name "*kernel_trace.csv" -delete
tail -3 gpurun_out/prof_r4d/bench.err
