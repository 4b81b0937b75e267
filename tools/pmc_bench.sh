#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only, no tracing domains) on the bench PCG loop.
set -o pipefail
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU" "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_WAIT_INST_LDS MemUnitStalled"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu --spmv-reps 3 > $out/p$i.json 2> $out/p$i.err || exit $?
done
