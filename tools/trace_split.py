"""Split the roofline SpMV's rocprofv3 kernel-trace durations into cold (dispatch right after the
L3-evicting k_flush_read) and warm (right after another SpMV) launches, so the profile's average
can be compared with bench.py's HIP-event cold / warm figures.  One bucket per KERNEL (staged CSR
``k_spmv``, SELL-DIA ``k_spmv_sdia``, SELL-64 with 16-bit / int32 columns ``k_spmv_sell``): the
bench's irregular-ordering leg launches the SELL-64 kernel on a system of the same size, so a
shared bucket would mix two kernels.  With ``--alg-bytes B`` (default: the headline kuhn101
system's §8(d) bytes, 12 nnz + 20 n + 4 = 201,442,412) each bucket also gets the cold average's
TB/s and its fraction of 8 TB/s -- what bench.py reports as ``roofline.frac``.

    python tools/trace_split.py gpurun_out/prof_<tag>/bench_kernel_trace.csv [--alg-bytes B]
"""
import csv
import json
import sys

KEY = "EpiStore<double>"  # standalone SpMV of A (bench.py roofline launches: staged CSR, then SELL)
PEAK_TBS = 8.0
ALG_BYTES = 12 * 15069699 + 20 * 1030301 + 4


def _kernel_bucket(name):
    if "k_spmv_sdia<double, double," in name:
        return "sdia"
    if "k_spmv_sell<double, double, short" in name:
        return "sell_int16"
    if "k_spmv_sell<double, double, int" in name:
        return "sell_int32"
    if "k_spmv<double, double, 1," in name:
        return "csr"
    return None


def main(path, alg_bytes=ALG_BYTES):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    prev = ""
    for r in rows:
        name = r["Kernel_Name"]
        kern = _kernel_bucket(name) if KEY in name else None
        if kern:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            out.setdefault(kern, ([], []))[0 if "k_flush_read" in prev else 1].append(dur)
        prev = name
    med = lambda v: sorted(v)[len(v) // 2] if v else None
    avg = lambda v: sum(v) / len(v) if v else None
    res = {}
    for kern, (cold, warm) in out.items():
        res[kern] = {"cold_n": len(cold), "cold_avg_us": avg(cold), "cold_median_us": med(cold), "warm_n": len(warm),
                     "warm_avg_us": avg(warm), "warm_median_us": med(warm)}
        if cold:
            tbs = alg_bytes / (avg(cold) * 1e-6) / 1e12
            res[kern].update(alg_bytes=alg_bytes, cold_TBps=tbs, cold_frac_of_8TBps=tbs / PEAK_TBS)
    # the PCG loop's five launches (graph-replayed and direct), average duration per kind
    import re
    # (KA / KB / KC: the headline's SELL-DIA kernels only -- the bench's irregular rows run systems of
    # the same size on SELL-64 / SELL-64C / SELL-64X kernels; UP / UR are the same kernels for all of
    # them and pooled)
    loop = {"KA t=L^T r": r"k_spmv_sdia<double, float.*EpiT<double, false>",
            "KB z=L t+eps r, rho": r"k_spmv_sdia<double, float.*EpiZG<double, false>",
            "UP p, x": r"k_update_p_g<double", "KC q=A p, pi": r"k_spmv_sdia<double, float.*EpiQG<double>",
            "UR r": r"k_update_r_g<double"}
    # the bench system's launches only: the largest grid of each kind (smaller systems -- C1, C5 --
    # launch smaller grids), without the predicated launches that exit at once after convergence
    # (chunk tails: < 1/3 of that grid's median)
    def grid(r):
        for key in ("Grid_Size", "Grid_Size_X"):
            if key in r and r[key]:
                return int(r[key])
        return 0
    lk = {}
    for r in rows:
        for k, pat in loop.items():
            if re.search(pat, r["Kernel_Name"]):
                lk.setdefault(k, []).append((grid(r), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3,
                                             r["Kernel_Name"]))
    out = {}
    for k, v in lk.items():
        g = max(x[0] for x in v)
        # the bench system's own kernel: the most frequent name at that grid (the irregular leg's
        # system has the same n but runs the SELL-64 kernels, and far fewer launches)
        names = {}
        for x in v:
            if x[0] == g:
                names[x[2]] = names.get(x[2], 0) + 1
        top = max(names, key=names.get)
        d = [x[1] for x in v if x[0] == g and x[2] == top]
        m = med(d)
        d = [x for x in d if x >= m / 3]
        out[k] = {"grid": g, "n": len(d), "avg": avg(d), "median": med(d)}
    res["pcg_loop_kernels_us"] = out
    # the bench system's GNN forwards (largest grid of each GNN kernel): per-kernel average and the
    # forward's kernel sum (num_mp_layers - 1 plain layers + the first layer + decoder + node encoder)
    gnn = {"k_encode<false>": r"k_encode<false>", "k_mp_layer<0>": r"k_mp_layer<(?:(?:false|true), )?0>",
           "k_mp_layer<S1E>": r"k_mp_layer<(?:(?:false|true), )?[123]>", "k_edge_dec": r"k_edge_dec<"}
    gk = {}
    for r in rows:
        for k, pat in gnn.items():
            if re.search(pat, r["Kernel_Name"]):
                gk.setdefault(k, []).append((grid(r), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
    g_out = {}
    for k, v in gk.items():
        g = max(x[0] for x in v)
        d = [x[1] for x in v if x[0] == g]
        g_out[k] = {"grid": g, "n": len(d), "avg": avg(d), "median": med(d), "min": min(d)}
    if "k_mp_layer<0>" in g_out and "k_mp_layer<S1E>" in g_out:
        per_fwd = g_out["k_mp_layer<0>"]["n"] // max(1, g_out["k_mp_layer<S1E>"]["n"])
        fwd = per_fwd * g_out["k_mp_layer<0>"]["avg"] + g_out["k_mp_layer<S1E>"]["avg"] + \
            g_out.get("k_edge_dec", {}).get("avg", 0.0) + g_out.get("k_encode<false>", {}).get("avg", 0.0)
        g_out["forward_kernel_sum_us"] = fwd
        g_out["plain_layers_per_forward"] = per_fwd
    res["gnn_forward_us"] = g_out
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    args = sys.argv[1:]
    ab = ALG_BYTES
    if "--alg-bytes" in args:
        i = args.index("--alg-bytes")
        ab = int(args[i + 1])
        del args[i:i + 2]
    main(args[0], ab)
