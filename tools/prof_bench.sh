#!/bin/bash
# Profile the default bench command on the GPU box: kernel-trace stats into gpurun_out/prof_<tag>/
set -o pipefail
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$tag
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o bench -- python3 bench.py > gpurun_out/prof_$tag/bench.json 2> gpurun_out/prof_$tag/bench.err
