"""GNN input samples (host-side input plumbing for the hot path).

``GraphSample`` carries the fields of the reference's PyG ``Data`` that the inference
path reads (``x, edge_index, edge_attr, mask, matrix_values, rsqrt_diag, ptr``);
``make_sample`` restates ``neural_cg/data.py:218-336`` (``make_data``) for one matrix,
including ``normalize_matrix='mean'`` (data.py:248-250) and the mean edge->node feature
aggregation used by the synthetic config (data.py:173-215).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import scipy.sparse as sp
import torch

from .problems import BlockGraph, to_block_graph


@dataclass
class GraphSample:
    x: torch.Tensor               # [N, F_in] fp32
    edge_index: torch.Tensor      # [2, E] int64, row-major sorted
    edge_attr: torch.Tensor       # [E, F_e] fp32
    mask: torch.Tensor            # [N, b] fp32
    matrix_values: Optional[torch.Tensor]  # [E, b, b] fp32 (scaled matrix)
    diagonal: Optional[torch.Tensor] = None
    inv_diag: Optional[torch.Tensor] = None
    rsqrt_diag: Optional[torch.Tensor] = None
    block_size: int = 1
    matrix_scale: float = 1.0
    ptr: torch.Tensor = field(default=None)
    gt: Optional[torch.Tensor] = None        # lhs / matrix_scale (training samples with a stored lhs)
    residual: Optional[torch.Tensor] = None  # rhs * mask (training samples)

    def __post_init__(self):
        if self.ptr is None:
            self.ptr = torch.tensor([0, self.x.shape[0]], dtype=torch.int64)

    @property
    def num_nodes(self) -> int:
        return int(self.x.shape[0])

    def to(self, device) -> "GraphSample":
        kw = {}
        for k, v in self.__dict__.items():
            kw[k] = v.to(device) if isinstance(v, torch.Tensor) and k != "ptr" else v
        return GraphSample(**kw)


def _mean_edge_to_node(edge_index: np.ndarray, edge_feat: np.ndarray, num_nodes: int) -> np.ndarray:
    """torch_geometric.utils.scatter(reduce='mean') at edge_index[1] (data.py:173-198)."""
    tgt = edge_index[1]
    out = np.zeros((num_nodes, edge_feat.shape[1]), dtype=np.float64)
    np.add.at(out, tgt, edge_feat.astype(np.float64))
    cnt = np.bincount(tgt, minlength=num_nodes).astype(np.float64)
    return (out / np.maximum(cnt, 1.0)[:, None]).astype(np.float32)


def make_sample(A: sp.spmatrix, mask: Optional[np.ndarray] = None, node_features: Optional[np.ndarray] = None,
                block_size: int = 1, use_mask_as_node_feature: bool = True,
                use_edge_features_as_node_feature: str = "disable", normalize_matrix="mean") -> GraphSample:
    """make_data (data.py:218-336) for an inference sample of matrix ``A``."""
    g: BlockGraph = to_block_graph(sp.csr_matrix(A), block_size)
    n_nodes = g.num_nodes
    if normalize_matrix is True or normalize_matrix == "mean":
        scale = 1.0 / np.mean(np.abs(g.block_values))
    elif normalize_matrix == "frob":
        scale = 1.0 / np.linalg.norm(g.block_values)
    elif normalize_matrix in ("none", False):
        scale = 1.0
    else:
        raise ValueError(f"normalize_matrix={normalize_matrix!r} not supported")
    if mask is None:
        mask = np.ones((n_nodes, block_size), dtype=np.float64)
    mask = np.asarray(mask, dtype=np.float64).reshape(n_nodes, block_size)
    nodes = []
    if node_features is not None:
        nodes.append(np.asarray(node_features, dtype=np.float32))
    if use_mask_as_node_feature:
        nodes.append(mask.astype(np.float32))
    edge_attr = torch.tensor(scale * g.block_values, dtype=torch.float32).flatten(1)
    if use_edge_features_as_node_feature == "mean":
        nodes.append(_mean_edge_to_node(g.edge_index, edge_attr.numpy(), n_nodes))
    elif use_edge_features_as_node_feature != "disable":
        raise ValueError("only 'disable' / 'mean' edge->node aggregation are restated")
    assert nodes, "No node feature found."
    x = torch.from_numpy(np.concatenate(nodes, axis=-1).astype(np.float32))
    diag = sp.csr_matrix(A).diagonal().reshape(-1, block_size) * scale
    return GraphSample(
        x=x,
        edge_index=torch.from_numpy(g.edge_index.astype(np.int64)),
        edge_attr=edge_attr,
        mask=torch.from_numpy(mask.astype(np.float32)),
        matrix_values=torch.tensor(g.block_values * scale, dtype=torch.float32),
        diagonal=torch.tensor(diag, dtype=torch.float32),
        inv_diag=torch.tensor(1.0 / (diag + 1e-7), dtype=torch.float32),
        rsqrt_diag=torch.tensor(1.0 / np.sqrt(diag + 1e-7), dtype=torch.float32),
        block_size=block_size,
        matrix_scale=float(scale),
    )
