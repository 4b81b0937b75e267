#!/bin/bash
# Generic PMC collection: one rocprofv3 --pmc pass per counter set (counters only, no tracing
# domains), program directly after `--`.
#   bash tools/pmc_run.sh <tag> <python script + args> -- "<set1>" "<set2>" ...
set -o pipefail
tag=$1; shift
prog=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do prog+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o pmc -- python3 "${prog[@]}" > $out/p$i.out 2> $out/p$i.err || exit $?
done
