"""torch-CPU restatement of the reference GNN -- TEST INFRASTRUCTURE ONLY.

Follows ``/root/reference/neural_cg/nn/gnns.py:9-97`` (NodeEdgeProcessing) and
``/root/reference/neural_cg/nn/basic_layers.py:13-44`` (activations / norms), ``:73-109``
(FeedForward) and ``:145-225`` (MPLayer) with torch_geometric 2.6.1 ``MessagePassing``
semantics restated explicitly (PyG is not installed):

* flow ``source_to_target``: ``x_j = x[edge_index[0]]``, ``x_i = x[edge_index[1]]``,
  messages summed (``aggr='add'``) at ``edge_index[1]`` with ``dim_size = N``;
* ``update(aggr_out, x) = node_mlp(aggr_out)``; ``edge_update`` uses the OLD node state;
* ``hasattr(self, "msg_norm")`` is False (the module is stored as ``node_msg_norm``,
  basic_layers.py:190-201), so MessageNorm is never applied.

Module names, construction order and ``self.apply(weight_init)`` match the reference so a
seeded construction (``torch.manual_seed``) yields the same parameters and a reference
checkpoint's ``gnn.*`` state_dict loads with ``strict=True``.  Parity of the forward
arithmetic with PyG itself is UNPINNED (no PyG, no reference test vectors).
"""
from __future__ import annotations

import torch
from torch import nn


def get_activation(activation: str):
    a = activation.lower()
    table = {"relu": nn.ReLU, "tanh": nn.Tanh, "sigmoid": nn.Sigmoid, "gelu": nn.GELU, "elu": nn.ELU,
             "leaky_relu": nn.LeakyReLU, "none": nn.Identity}
    if a not in table:
        raise ValueError(f"Activation {activation} not supported.")
    return table[a]()


def get_normalization(normalization: str, channels: int):
    n = normalization.lower()
    if n == "none":
        return nn.Identity()
    if n in ["batch", "batchnorm", "batch_norm", "rms", "rmsnorm", "rms_norm"]:
        return nn.RMSNorm(channels)
    if n in ["layer", "layernorm", "layer_norm"]:
        return nn.LayerNorm(channels)
    raise ValueError(f"Normalization {normalization} not supported.")


class FeedForward(nn.Module):
    """basic_layers.py:73-109."""

    def __init__(self, in_channels, out_channels, hidden_channels, num_layers, pre_norm="none",
                 activation="gelu", out_activation="none"):
        super().__init__()
        self.pre_norm = get_normalization(pre_norm, in_channels)
        self.lift = nn.Sequential(nn.Linear(in_channels, hidden_channels), get_activation(activation))
        self.body = nn.ModuleList()
        for _ in range(1, num_layers):
            self.body.append(nn.Sequential(nn.Linear(hidden_channels, hidden_channels), get_activation(activation)))
        self.proj = nn.Sequential(nn.Linear(hidden_channels, out_channels), get_activation(out_activation))

    def forward(self, x):
        x = self.pre_norm(x)
        x = self.lift(x)
        for layer in self.body:
            x = layer(x)
        return self.proj(x)


class _MessageNorm(nn.Module):
    """Parameter holder with PyG MessageNorm's state (``scale``); never applied (see header)."""

    def __init__(self, learn_scale: bool = False):
        super().__init__()
        self.scale = nn.Parameter(torch.empty(1), requires_grad=learn_scale)
        self.reset_parameters()

    def reset_parameters(self):
        self.scale.data.fill_(1.0)


class MPLayer(nn.Module):
    """basic_layers.py:145-225 with PyG source_to_target / add semantics."""

    def __init__(self, node_channels, edge_channels, node_residual, edge_residual, node_mlp, edge_mlp, msg_mlp,
                 aggr="add", msg_norm=True):
        super().__init__()
        assert aggr == "add", "only aggr='add' (gnn.yaml) is restated"
        self.node_mlp = FeedForward(in_channels=node_channels, out_channels=node_channels, **node_mlp)
        self.edge_mlp = FeedForward(in_channels=2 * node_channels + edge_channels, out_channels=edge_channels,
                                    **edge_mlp)
        self.msg_mlp = FeedForward(in_channels=edge_channels + 2 * node_channels, out_channels=node_channels,
                                   **msg_mlp)
        self.node_residual = node_residual
        self.edge_residual = edge_residual
        if msg_norm:
            self.node_msg_norm = _MessageNorm()

    def forward(self, node_attr, edge_index, edge_attr):
        src, dst = edge_index[0], edge_index[1]
        x_i, x_j = node_attr[dst], node_attr[src]
        feat = torch.cat([x_i, x_j, edge_attr], dim=-1)
        msg = self.msg_mlp(feat)
        aggr = torch.zeros(node_attr.shape[0], msg.shape[1], dtype=msg.dtype).index_add_(0, dst, msg)
        node_new = self.node_mlp(aggr)
        node_out = node_attr + node_new if self.node_residual else node_new
        edge_new = self.edge_mlp(feat)
        edge_out = edge_attr + edge_new if self.edge_residual else edge_new
        return node_out, edge_out


def weight_init(m: nn.Module):
    """neural_cg/utils/weight_init.py:2-4."""
    if hasattr(m, "reset_parameters"):
        m.reset_parameters()


class NodeEdgeProcessing(nn.Module):
    """gnns.py:9-97."""

    def __init__(self, node_in_features, node_out_features, node_encoder, node_decoder, edge_in_features,
                 edge_out_features, edge_encoder, edge_decoder, num_mp_layers, node_features, edge_features,
                 node_residual, edge_residual, node_mlp, edge_mlp, msg_mlp, msg_norm, aggr="add"):
        super().__init__()
        self.node_enc = FeedForward(in_channels=node_in_features, out_channels=node_features, **node_encoder)
        if node_out_features is None:
            self.node_dec = nn.Identity()
        else:
            self.node_dec = FeedForward(in_channels=node_features, out_channels=node_out_features, **node_decoder)
        self.edge_enc = FeedForward(in_channels=edge_in_features, out_channels=edge_features, **edge_encoder)
        self.edge_dec = FeedForward(in_channels=edge_features + 2 * node_features, out_channels=edge_out_features,
                                    **edge_decoder)
        self.mp_layers = nn.ModuleList()
        for _ in range(num_mp_layers):
            self.mp_layers.append(MPLayer(node_features, edge_features, node_residual, edge_residual, node_mlp,
                                          edge_mlp, msg_mlp, aggr=aggr, msg_norm=msg_norm))
        self.apply(weight_init)

    def forward(self, node_attr, edge_index, edge_attr):
        node_attr = self.node_enc(node_attr)
        edge_attr = self.edge_enc(edge_attr)
        for mp in self.mp_layers:
            node_attr, edge_attr = mp(node_attr, edge_index, edge_attr)
        dec_in = torch.cat([edge_attr, node_attr[edge_index[0]], node_attr[edge_index[1]]], dim=-1)
        return self.node_dec(node_attr), self.edge_dec(dec_in)


def default_gnn_config(features: int = 16, mlp_layers: int = 2, num_mp_layers: int = 4) -> dict:
    """config/gnn.yaml."""
    ff = lambda norm: {"pre_norm": norm, "hidden_channels": features, "num_layers": mlp_layers}
    return dict(node_encoder=ff("none"), edge_encoder=ff("none"), node_decoder=ff("none"), edge_decoder=ff("none"),
                num_mp_layers=num_mp_layers, node_residual=True, edge_residual=True, node_features=features,
                edge_features=features, node_mlp=ff("layer"), edge_mlp=ff("layer"), msg_mlp=ff("layer"),
                msg_norm=True, aggr="add")


def build(node_in: int, edge_in: int, block_size: int, seed: int = 0, **over) -> NodeEdgeProcessing:
    """Seeded construction, like SimpleTrainingWorkspace.__init__ (workspace.py:70-76)."""
    cfg = default_gnn_config()
    cfg.update(over)
    torch.manual_seed(seed)
    return NodeEdgeProcessing(node_in_features=node_in, node_out_features=None, edge_in_features=edge_in,
                              edge_out_features=block_size * block_size, **cfg)


# ---------------------------------------------------------------------------
# basic_layers.py:112-142 GraphSpmv and :228-261 AATPE, PyG semantics restated in fp64
# ---------------------------------------------------------------------------
def graph_spmv(X, edge_index, A, mask=None, transpose=False):
    """flow target_to_source (transpose=False): message A_e x[ei[1]] summed at ei[0];
    source_to_target (transpose=True): message A_eᵀ x[ei[0]] summed at ei[1]; then * mask."""
    X = torch.as_tensor(X, dtype=torch.float64)
    A = torch.as_tensor(A, dtype=torch.float64)
    if A.ndim == 1:
        A = A.reshape(-1, 1, 1)
    X2 = X.reshape(X.shape[0], -1)
    src, dst = (edge_index[0], edge_index[1]) if transpose else (edge_index[1], edge_index[0])
    blk = A.transpose(-1, -2) if transpose else A
    msg = torch.bmm(blk, X2[src].unsqueeze(-1)).squeeze(-1)
    out = torch.zeros_like(X2).index_add_(0, dst, msg)
    if mask is not None:
        out = out * torch.as_tensor(mask, dtype=torch.float64).reshape(out.shape)
    return out.reshape(X.shape)


def aatpe(x, edge_index, boo_values, epsilon, mask=None, diag=None):
    x = torch.as_tensor(x, dtype=torch.float64)
    at_x = graph_spmv(x, edge_index, boo_values, mask, transpose=True)
    eps_x = epsilon * x
    if diag is not None:
        d = torch.as_tensor(diag, dtype=torch.float64)
        at_x = at_x * d
        eps_x = eps_x * d
    return eps_x + graph_spmv(at_x, edge_index, boo_values, mask, transpose=False)
