"""Split the roofline SpMV's rocprofv3 kernel-trace durations into cold (dispatch right after the
L3-evicting k_flush_read) and warm (right after another SpMV) launches, so the profile's average
can be compared with bench.py's HIP-event cold / warm figures.

    python tools/trace_split.py gpurun_out/prof_<tag>/bench_kernel_trace.csv
"""
import csv
import json
import sys

KEY = "EpiStore<double>"  # standalone SpMV of A (bench.py roofline launches: staged CSR, then SELL)


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    prev = ""
    for r in rows:
        name = r["Kernel_Name"]
        if KEY in name and ("k_spmv<double, double, 1," in name or "k_spmv_sell<double, double," in name or "k_spmv_sdia<double, double," in name):
            kern = "sell" if "k_spmv_s" in name else "csr"
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            out.setdefault(kern, ([], []))[0 if "k_flush_read" in prev else 1].append(dur)
        prev = name
    med = lambda v: sorted(v)[len(v) // 2] if v else None
    avg = lambda v: sum(v) / len(v) if v else None
    res = {}
    for kern, (cold, warm) in out.items():
        res[kern] = {"cold_n": len(cold), "cold_avg_us": avg(cold), "cold_median_us": med(cold), "warm_n": len(warm),
                     "warm_avg_us": avg(warm), "warm_median_us": med(warm)}
    # the PCG loop's five launches (graph-replayed and direct), average duration per kind
    import re
    loop = {"KA t=L^T r": r"k_spmv_s(?:ell|dia)<double, float.*EpiT<double, false>",
            "KB z=L t+eps r, rho": r"k_spmv_s(?:ell|dia)<double, float.*EpiZG<double, false>",
            "UP p, x": r"k_update_p_g<double>", "KC q=A p, pi": r"k_spmv_s(?:ell|dia)<double, float.*EpiQG<double>",
            "UR r": r"k_update_r_g<double>"}
    lk = {}
    for r in rows:
        for k, pat in loop.items():
            if re.search(pat, r["Kernel_Name"]):
                lk.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    # the bench system's launches only: drop the predicated launches that exit at once (chunk tails
    # after convergence) and smaller systems' launches -- keep those >= half the 90th percentile
    def big(v):
        p90 = sorted(v)[int(0.9 * (len(v) - 1))]
        return [d for d in v if d >= 0.5 * p90]
    res["pcg_loop_kernels_us"] = {k: {"n": len(big(v)), "avg": avg(big(v)), "median": med(big(v))} for k, v in lk.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
