#!/usr/bin/env python
"""Fixture input: the HIP GNN's raw output ``boo`` ([E, b, b] fp32) on a bench workload.

bench.py's setup verbatim (problems.workload -> make_sample -> SimpleInferenceWorkspace(seed=0)
-> forward), run twice to check the forward is deterministic.  Writes ``<out>/<workload>.npy`` and
``<out>/<workload>.json`` (sha256 of the bytes, E, b).  tests/golden/make_golden.py ``headline``
feeds this L through the reference's own to_csr_cpu + get_pcg_iter_time_scipy (this container);
the GPU tests recompute ``boo`` on the box and check its sha256 before comparing trajectories.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="kuhn101")
    ap.add_argument("--dataset", default=None, help="an infer.synthetic_dataset name: one file per system, "
                                                      "<dataset>_<k>.npy (the workspace is built once, as bench.c5_rows)")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import numpy as np
    import torch

    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    if args.dataset:
        from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset

        samples = synthetic_dataset(args.dataset)
        ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=samples[0].edge_attr.shape[1],
                                      seed=0)
        for k, smp in enumerate(samples):
            dump(ws, smp.to("cuda"), f"{args.dataset}_{k}", 1, int(smp.num_nodes), args.out)
        return
    A_raw, mask, feats, bs, e2n = P.workload(args.workload)
    sample = make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n)
    ws = SimpleInferenceWorkspace(node_features=sample.x.shape[1], edge_features=sample.edge_attr.shape[1],
                                  block_size=bs, epsilon=3e-3, seed=0)
    dump(ws, sample.to("cuda"), args.workload, bs, int(A_raw.shape[0]), args.out)


def dump(ws, d, name, bs, n, out):
    import numpy as np
    import torch

    outs = []
    for _ in range(2):
        boo = ws.forward(d.x, d.edge_index, d.edge_attr)
        torch.cuda.synchronize()
        outs.append(boo.detach().cpu().numpy().astype(np.float32, copy=False))
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32)), "GNN forward not deterministic"
    a = np.ascontiguousarray(outs[0])
    os.makedirs(out, exist_ok=True)
    np.save(os.path.join(out, f"{name}.npy"), a)
    meta = {"workload": name, "shape": list(a.shape), "block_size": bs,
            "sha256": hashlib.sha256(a.tobytes()).hexdigest(), "n": n}
    json.dump(meta, open(os.path.join(out, f"{name}.json"), "w"))
    print(json.dumps(meta), flush=True)


if __name__ == "__main__":
    main()
