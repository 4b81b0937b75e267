"""Print the key fields of tools/irregular_probe.py output (one line per workload)."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        (k, v), = json.loads(line).items()
        lk = v.get("loop_kernels_us") or {}
        print(k, "n", v["workload"].split("n=")[1].split(",")[0], "it", v["iters"], "us/it %.1f" % v["pcg_iter_us"],
              "views", v["solver_views"]["A"]["columns"], "reorder", v["solver_reorder"]["applied"],
              "setup %.1f ms" % v["solver_setup_ms"], "pad %.2f" % v.get("sell_slots_per_nnz", 0))
        print("   loop", {a.split()[0]: round(b, 1) for a, b in lk.items()},
              "spmv %.1f us frac %.3f" % (v["spmv"]["avg_launch_ms_cold"] * 1e3, v["spmv"]["frac_cold"]), v["spmv"]["kernel"])
