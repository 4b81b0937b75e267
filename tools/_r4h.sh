set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4h; mkdir -p $out
timeout -k 10 400 python -u tools/loop_ab.py '{"base": {}, "pf": {"LSPCG_EXP": "4"}, "fork": {"LSPCG_EXP": "8"}, "pf+fork": {"LSPCG_EXP": "12"}}' kuhn101 11 $out/loop_ab.jsonl > $out/loop_ab.txt 2>&1 || exit $?
cat $out/loop_ab.txt
LSPCG_EXP=12 timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_traj.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.txt 2>&1; rc=$?; tail -2 $out/tests.txt; exit $rc
