#!/bin/bash
# GNN kernel A/B under rocprofv3 --kernel-trace --stats: the in-tree build against a variant library
# (tools/build_variant.py), alternating, each tools/gnn_run.py --reps 20 (GPU box, measurement only).
#   bash tools/r6_gnn_prof.sh <variant.so>
set -o pipefail
var=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6gp
for v in base vf base2 vf2; do
  unset LSPCG_LIB
  case $v in vf*) export LSPCG_LIB=$var ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6gp/$v -o run -- python3 tools/gnn_run.py --reps 20 > gpurun_out/r6gp/$v.out 2> gpurun_out/r6gp/$v.err || exit $?
  find gpurun_out/r6gp/$v -name "*kernel_trace.csv" -delete
done
