"""GNN input samples (host-side input plumbing for the hot path).

``GraphSample`` carries the fields of the reference's PyG ``Data`` that the inference
path reads (``x, edge_index, edge_attr, mask, matrix_values, rsqrt_diag, ptr``);
``make_sample`` builds one inference sample of an in-memory matrix through
``dataset.make_data`` (the restatement of ``neural_cg/data.py:218-336``).
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


def make_sample(A: sp.spmatrix, mask: Optional[np.ndarray] = None, node_features: Optional[np.ndarray] = None,
                block_size: int = 1, use_mask_as_node_feature: bool = True,
                use_edge_features_as_node_feature: str = "disable", normalize_matrix="mean") -> GraphSample:
    """make_data (data.py:218-336) for an inference sample of an in-memory matrix ``A``: the
    block COO view of A (``FolderDataset.load``'s layout, data.py:471-572) fed to
    ``dataset.make_data`` -- the one restatement of make_data, golden-checked for every option."""
    from .dataset import RawData, make_data

    g: BlockGraph = to_block_graph(sp.csr_matrix(A), block_size)
    n_nodes = g.num_nodes
    if mask is None:
        mask = np.ones((n_nodes, block_size), dtype=np.float64)
    raw = RawData(block_values=g.block_values, diagonals=sp.csr_matrix(A).diagonal().reshape(-1, block_size),
                  edge_index=g.edge_index, node_features=None if node_features is None else np.asarray(node_features),
                  lhs=None, rhs=None, mask=np.asarray(mask, dtype=np.float64).reshape(n_nodes, block_size),
                  num_nodes=n_nodes, block_size=block_size)
    return make_data(raw, use_matrix_as_edge_feature=True, use_mask_as_node_feature=use_mask_as_node_feature,
                     use_node_features_as_edge_feature=False,
                     use_edge_features_as_node_feature=use_edge_features_as_node_feature, use_random_rhs=True,
                     normalize_matrix=normalize_matrix, is_inference=True)
