#!/bin/bash
# rocprofv3 kernel-trace stats of tools/pcg_probe.py (PCG schedule A/B) into gpurun_out/probe_<tag>/
set -o pipefail
tag=${1:-p}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe_$tag -o probe -- python3 tools/pcg_probe.py $PROBE_ARGS > gpurun_out/probe_$tag/probe.log 2>&1
