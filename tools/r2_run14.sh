#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 200 python tools/dist_debug.py 2>&1 | grep -v "hostname\|amdgpu.ids" > gpurun_out/r2/dist_debug.txt; rc=$?
cat gpurun_out/r2/dist_debug.txt; exit $rc
