#!/bin/bash
# HBM traffic of the roofline SpMV: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
# they do not fit one TCC pass), counters only, no tracing domains (MI355X_MICROARCH.md "HBM").
# Summary -> gpurun_out/traffic_<tag>/summary.json (tools/spmv_traffic_summary.py).
set -o pipefail
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/traffic_$tag
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $out/$c -o pmc -- python3 tools/spmv_roofline_run.py > $out/$c.json 2> $out/$c.err || exit $?
done
python3 tools/spmv_traffic_summary.py $out > $out/summary.json
