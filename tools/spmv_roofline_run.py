"""Run only the bench's roofline SpMV (fp64 A of the kuhn101 system after the SELL analysis step,
or the staged CSR kernel with --csr; cold launches).

Used under rocprofv3 --pmc by tools/spmv_traffic.sh so that the counter rows of the SpMV
dispatches are exactly the launches bench.py times (same matrix, same flush)."""
import argparse
import json
import sys

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="kuhn101")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm", action="store_true", help="back-to-back launches instead of cold ones")
    ap.add_argument("--csr", action="store_true", help="staged CSR kernel (skip the SELL analysis step)")
    args = ap.parse_args()
    sys.path.insert(0, ".")
    from bench import FLUSH_BYTES, spmv_bytes
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    A_raw, mask, feats, bs, e2n = P.workload(args.workload)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs,
                                  seed=0)
    A = ws.system_matrix(s.to("cuda"))
    x = torch.randn(A.n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    kind = 0 if args.csr else A.prepare_spmv()
    ms = A.spmv_timed(x, y, args.reps, flush_bytes=0 if args.warm else FLUSH_BYTES)
    print(json.dumps({"workload": args.workload, "n": A.n, "nnz": A.nnz, "alg_bytes": spmv_bytes(A.n, A.nnz),
                      "avg_ms": ms, "mode": "warm" if args.warm else "cold", "kernel_kind": kind}))


if __name__ == "__main__":
    main()
