"""Per-launch HBM bytes of the roofline SpMV from the two PMC passes of tools/spmv_traffic.sh.

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE counts 128-B requests at 64 B, so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are in KiB.  Only the
SpMV dispatches (EpiStore fp64/fp64 kernel) enter the average; the flush kernel does not.
(The SELL kernel's 8-B column-offset loads are an uncalibrated width: the x2 is applied to all
fetched bytes, which can overstate them.)"""
import csv
import glob
import json
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(f"{d}/{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            roof = "k_spmv<double, double, 1" in name or "k_spmv_sell<double, double" in name or "k_spmv_sdia<double, double" in name
            if roof and "EpiStore" in name and r["Counter_Name"] == counter:
                vals.setdefault(r["Dispatch_Id"], 0.0)
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    d = sys.argv[1]
    fetch = per_dispatch(d, "FETCH_SIZE")
    write = per_dispatch(d, "WRITE_SIZE")
    run = json.loads(open(f"{d}/FETCH_SIZE.json").read().strip().splitlines()[-1])
    # every dispatch except the untimed first one follows a 512 MiB flush (cold)
    f = sorted(fetch)[len(fetch) // 2] * 1024 * 2  # median, KiB -> B, x2 gfx950 correction
    w = sorted(write)[len(write) // 2] * 1024
    out = {"workload": run["workload"], "n": run["n"], "nnz": run["nnz"], "alg_bytes": run["alg_bytes"],
           "kernel_kind": run.get("kernel_kind", 0),
           "fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w, "dispatches": len(fetch),
           "traffic_over_alg": (f + w) / run["alg_bytes"],
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median per dispatch, "
                     "FETCH_SIZE x2 (gfx950), KiB -> B"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
