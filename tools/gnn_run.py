"""Run the GNN forward (inference_step) on a bench workload a few times -- a target for
rocprofv3 (tools/pmc_run.sh) and a quick timing of the GNN alone."""
import argparse
import json
import sys
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="kuhn101")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before each wall-clock call")
    ap.add_argument("--dump", default="", help="save the forward's output here (.npy)")
    args = ap.parse_args()
    sys.path.insert(0, ".")
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    A_raw, mask, feats, bs, e2n = P.workload(args.workload)
    s = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], block_size=bs,
                                  seed=0)
    d = s.to("cuda")
    ws.forward(d.x, d.edge_index, d.edge_attr)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.reps):
        ws.forward(d.x, d.edge_index, d.edge_attr)
    ev1.record()
    torch.cuda.synchronize()
    fwd_ms = ev0.elapsed_time(ev1) / args.reps
    walls, pre = [], []
    for _ in range(args.reps):  # host clock around one call from an idle device (inference_step's dt)
        torch.cuda.synchronize()
        if args.idle_ms:
            time.sleep(args.idle_ms * 1e-3)
        t0 = time.perf_counter()
        ws.forward(d.x, d.edge_index, d.edge_attr)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        pre.append((t1 - t0) * 1e3)
    if args.dump:
        import numpy as np
        np.save(args.dump, ws.forward(d.x, d.edge_index, d.edge_attr).float().cpu().numpy())
    print(json.dumps({"workload": args.workload, "edges": int(d.edge_index.shape[1]), "forward_ms": fwd_ms,
                      "wall_ms": sorted(walls)[len(walls) // 2], "host_return_ms": sorted(pre)[len(pre) // 2]}))


if __name__ == "__main__":
    main()
