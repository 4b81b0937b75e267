"""Summarise rocprofv3 PMC csv passes per kernel (average per dispatch)."""
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_spmv|k_update|k_mp_layer"
import re
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if not re.search(pat, name):
            continue
        short = re.sub(r"lspcg::", "", name)
        short = re.sub(r"\(.*", "", short)[:100]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}  (n={len(v)})")
