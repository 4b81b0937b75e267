"""Run the GNN forward (inference_step) on a bench workload a few times -- a target for
rocprofv3 (tools/pmc_run.sh) and a quick timing of the GNN alone."""
import argparse
import json
import sys

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="kuhn101")
    ap.add_argument("--reps", type=int, default=3)
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
    print(json.dumps({"workload": args.workload, "edges": int(d.edge_index.shape[1]),
                      "forward_ms": ev0.elapsed_time(ev1) / args.reps}))


if __name__ == "__main__":
    main()
