"""Summarise rocprofv3 PMC csv passes (tools/pmc_run.sh) per kernel: counter values summed per
dispatch, then averaged over dispatches.

    python tools/pmc_summary.py <tag> [kernel-regex]
"""
import csv
import glob
import re
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_spmv|k_update|k_mp_layer"
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if not re.search(pat, name):
            continue
        short = re.sub(r"\(.*", "", re.sub(r"lspcg::", "", name))[:110]
        per[short][r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, d in per.items():
    print(k)
    for c, v in sorted(d.items()):
        vals = list(v.values())
        print(f"   {c:36s} {sum(vals) / len(vals):18.1f}  (dispatches={len(vals)})")
