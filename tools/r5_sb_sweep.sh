#!/bin/bash
# BSELL-DIA block slots per batch: the C4 bench line per variant library (tools/_variants/, built by
# tools/build_variant.py with -DLSPCG_BSDIA_SB64=k -DLSPCG_BSDIA_SB32=k).  Usage: bash tools/r5_sb_sweep.sh TAG
set -o pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
for v in base sb1 sb4 sb8 base2; do
  lib=learningsparsepreconditioner4gpu_amd/liblspcg_hip.so
  case $v in sb*) lib=tools/_variants/liblspcg_$v.so ;; esac
  LSPCG_LIB=$lib timeout -k 10 300 python -u bench.py --workload elast --steps 5 --warmup 1 --no-cpu --no-variants > "$out/elast_$v.json" 2> "$out/elast_$v.err" || exit $?
  python3 -c "
import json; d=json.load(open('$out/elast_$v.json')); r=d['roofline']; k=d['pcg_loop_kernels']['all_us']
print(json.dumps({'v': '$v', 'it_s': d['value'], 'us_iter': d['pcg_iter_us'], 'frac': r['frac'], 'cold_us': r['avg_launch_ms_cold']*1e3, 'warm_us': r['avg_launch_ms_warm']*1e3, 'kernels': k}))" | tee -a "$out/sb_sweep.jsonl"
done
