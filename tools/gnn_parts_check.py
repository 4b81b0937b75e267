"""Debug aid: the HIP GNN forward against the oracle for 0 / 1 / 4 message-passing layers on a small
Poisson graph (max |difference| per setting), to localise a wrong stage.  GPU box; measurement only."""
import sys

sys.path.insert(0, ".")
import numpy as np
import torch

from oracle import gnn as OG
from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.data import make_sample
from learningsparsepreconditioner4gpu_amd.nn import build_gnn

A, mask, _ = P.poisson2d_grid(23, 19)
s = make_sample(A, mask)
for layers in (0, 1, 4):
    ref = OG.build(s.x.shape[1], s.edge_attr.shape[1], 1, seed=0, num_mp_layers=layers)
    gpu = build_gnn(s.x.shape[1], s.edge_attr.shape[1], 1, seed=0, num_mp_layers=layers).cuda()
    with torch.no_grad():
        _, r = ref(s.x, s.edge_index, s.edge_attr)
        d = s.to("cuda")
        _, g = gpu(d.x, d.edge_index, d.edge_attr)
    print(layers, float((g.cpu() - r).abs().max()), float(r.abs().max()))
