"""Per-launch HBM bytes of the PCG loop's five kernels from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) over `bench.py --steps 1 --warmup 1 --no-cpu --no-variants`
(tools/pmc_run.sh <tag> bench.py ... -- FETCH_SIZE WRITE_SIZE), written in the format bench.py
reads from profiles/pcg_loop_traffic.json.

    python tools/loop_traffic.py <tag> <column_kind> > profiles/pcg_loop_traffic.json

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE x 2; both counters in KiB.  Median per
dispatch over the ext_spai split schedule's launches (the only ones with these epilogues)."""
import csv
import glob
import json
import re
import sys

KERNELS = {"KA t=L^T r": r"k_spmv_s(?:ellj?|dia)<double, float.*EpiT<double, false>",
           "KB z=L t+eps r, rho": r"k_spmv_s(?:ellj?|dia)<double, float.*EpiZG<double, false>",
           "UP p, x": r"k_update_p_g<double",
           "KC q=A p, pi": r"k_spmv_s(?:ellj?|dia)<double, float.*EpiQG<double>",
           "UR r": r"k_update_r_g<double"}


def per_dispatch(tag, counter):
    vals = {k: {} for k in KERNELS}
    for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for k, pat in KERNELS.items():
                if re.search(pat, r.get("Kernel_Name", "")):
                    key = (f, r["Dispatch_Id"])
                    vals[k][key] = vals[k].get(key, 0.0) + float(r["Counter_Value"])
    return {k: sorted(v.values()) for k, v in vals.items()}


def main():
    tag, kind = sys.argv[1], int(sys.argv[2])
    fetch = per_dispatch(tag, "FETCH_SIZE")
    write = per_dispatch(tag, "WRITE_SIZE")
    run = None
    for line in open(f"gpurun_out/pmc_{tag}/p1.out"):
        if line.startswith("{"):
            run = json.loads(line)
    out = {"workload": run["config"]["workload"].split(":")[0], "n": run["config"]["n"], "nnz": run["config"]["nnz_A"],
           "column_kind": kind, "source": f"gpurun_out/pmc_{tag}",
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py --steps 1 --warmup 1 --no-cpu "
                     "--no-variants; bytes = FETCH_SIZE x 2 (gfx950) x 1024 + WRITE_SIZE x 1024, median per dispatch",
           "kernels": {}}
    for k in KERNELS:
        if not fetch[k] or not write[k]:
            continue
        f = fetch[k][len(fetch[k]) // 2] * 1024 * 2
        w = write[k][len(write[k]) // 2] * 1024
        out["kernels"][k] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w, "dispatches": len(fetch[k])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
