#!/bin/bash
# Round-6 GPU step runner: bash tools/r6_gpu.sh TAG [t=tests,..] [probe=wl,wl] [bench] ...
set -o pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
for s in "$@"; do
  case $s in
    t=*)
      files=$(echo "${s#t=}" | tr ',' ' ')
      timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > "$out/tests.txt" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 "$out/tests.txt"; [ $rc -eq 0 ] || exit $rc ;;
    probe=*)
      wls=$(echo "${s#probe=}" | tr ',' ' ')
      timeout -k 10 900 python -u tools/irregular_probe.py $wls > "$out/probe.jsonl" 2> "$out/probe.err"
      rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/probe.err"; exit $rc; } ;;
    jag=*)
      for wl in $(echo "${s#jag=}" | tr ',' ' '); do
        timeout -k 10 300 python -u tools/jag_probe.py $wl >> "$out/jag.jsonl" 2>> "$out/jag.err" || { tail -5 "$out/jag.err"; exit 1; }
      done; cat "$out/jag.jsonl" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
      python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['value'], d['pcg_iter_us'], d['gnn_precond_ms'], d['roofline']['frac'])" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
