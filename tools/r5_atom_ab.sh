#!/bin/bash
# Timing-only A/B: the loop with the split reduction's ticket + sweep (in-tree library) vs group
# totals accumulated by no-return atomics (tools/_variants/liblspcg_atom.so, wrong arithmetic,
# iterations forced to 212).  Alternating processes.  Usage: bash tools/r5_atom_ab.sh TAG
set -o pipefail
tag=$1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p "$out"
for v in base atom base atom; do
  lib=learningsparsepreconditioner4gpu_amd/liblspcg_hip.so
  [ $v = atom ] && lib=tools/_variants/liblspcg_atom.so
  LSPCG_LIB=$lib LOOP_AB_MAXIT=212 LOOP_AB_REPLICAS=2 LOOP_AB_KERNELS=1 timeout -k 10 300 python -u tools/loop_ab.py "{\"$v\": {}}" kuhn101 5 "$out/atom_ab.jsonl" > "$out/atom_ab_$v.txt" 2>&1 || exit $?
  grep '"variant"' "$out/atom_ab_$v.txt" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['iters'], round(d['us_per_iter_median'],2), d['per_solver_median'], {k: round(v,2) for k,v in d['kernels_us'].items()} if isinstance(d.get('kernels_us'), dict) else d.get('kernels_us'))"
done
