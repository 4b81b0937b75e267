"""The SPAI-emitting GNN (``NodeEdgeProcessing``) with a HIP forward pass.

Parameter layout, module names and seeded initialisation follow the reference
(``neural_cg/nn/gnns.py:9-97``, ``neural_cg/nn/basic_layers.py:73-225``,
``neural_cg/utils/weight_init.py``), so ``state_dict()`` keys are the reference's and a
reference checkpoint's ``gnn.*`` tensors load directly.  The modules here are parameter
containers; the forward pass is ``lspcg_gnn_forward`` (csrc/lspcg_gnn.hip) -- there is no
torch compute path.

Packed weight blob (fp32, ``pack_weights``), each FeedForward as
``[W1 (16 x in) | b1 | W2 (16 x 16) | b2 | W3 (out x 16) | b3]``::

    node_enc | edge_enc | per MPLayer: [node LN γ,β (16) | node_mlp]
                                      [edge LN γ,β (48) | edge_mlp]
                                      [msg  LN γ,β (48) | msg_mlp ] | edge_dec
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch
from torch import nn

from . import _lib
from .sparse import Context, _ptr


def _act(name: str):
    table = {"relu": nn.ReLU, "tanh": nn.Tanh, "sigmoid": nn.Sigmoid, "gelu": nn.GELU, "elu": nn.ELU,
             "leaky_relu": nn.LeakyReLU, "none": nn.Identity}
    return table[name.lower()]()


def _norm(name: str, channels: int):
    n = name.lower()
    if n == "none":
        return nn.Identity()
    if n in ("layer", "layernorm", "layer_norm"):
        return nn.LayerNorm(channels)
    if n in ("batch", "batchnorm", "batch_norm", "rms", "rmsnorm", "rms_norm"):
        return nn.RMSNorm(channels)
    raise ValueError(f"Normalization {name} not supported.")


class FeedForward(nn.Module):
    """Parameters of basic_layers.py:73-109 FeedForward."""

    def __init__(self, in_channels, out_channels, hidden_channels, num_layers, pre_norm="none", activation="gelu",
                 out_activation="none"):
        super().__init__()
        self.pre_norm = _norm(pre_norm, in_channels)
        self.lift = nn.Sequential(nn.Linear(in_channels, hidden_channels), _act(activation))
        self.body = nn.ModuleList()
        for _ in range(1, num_layers):
            self.body.append(nn.Sequential(nn.Linear(hidden_channels, hidden_channels), _act(activation)))
        self.proj = nn.Sequential(nn.Linear(hidden_channels, out_channels), _act(out_activation))
        self.activation = activation
        self.out_activation = out_activation

    def linears(self):
        return [self.lift[0]] + [b[0] for b in self.body] + [self.proj[0]]


class _MessageNormParams(nn.Module):
    def __init__(self):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(1), requires_grad=False)

    def reset_parameters(self):
        self.scale.data.fill_(1.0)


class MPLayer(nn.Module):
    """Parameters of basic_layers.py:145-191 MPLayer."""

    def __init__(self, node_channels, edge_channels, node_residual, edge_residual, node_mlp, edge_mlp, msg_mlp,
                 aggr="add", msg_norm=True):
        super().__init__()
        if aggr != "add":
            raise NotImplementedError("only aggr='add' (config/gnn.yaml) is implemented")
        self.node_mlp = FeedForward(in_channels=node_channels, out_channels=node_channels, **node_mlp)
        self.edge_mlp = FeedForward(in_channels=2 * node_channels + edge_channels, out_channels=edge_channels,
                                    **edge_mlp)
        self.msg_mlp = FeedForward(in_channels=edge_channels + 2 * node_channels, out_channels=node_channels,
                                   **msg_mlp)
        self.node_residual = node_residual
        self.edge_residual = edge_residual
        if msg_norm:
            self.node_msg_norm = _MessageNormParams()


def _weight_init(m: nn.Module):
    if hasattr(m, "reset_parameters"):
        m.reset_parameters()


def default_gnn_config(features: int = 16, mlp_layers: int = 2, num_mp_layers: int = 4) -> dict:
    """config/gnn.yaml."""
    ff = lambda norm: {"pre_norm": norm, "hidden_channels": features, "num_layers": mlp_layers}
    return dict(node_encoder=ff("none"), edge_encoder=ff("none"), node_decoder=ff("none"), edge_decoder=ff("none"),
                num_mp_layers=num_mp_layers, node_residual=True, edge_residual=True, node_features=features,
                edge_features=features, node_mlp=ff("layer"), edge_mlp=ff("layer"), msg_mlp=ff("layer"),
                msg_norm=True, aggr="add")


class NodeEdgeProcessing(nn.Module):
    """gnns.py:9-97 -- forward runs on MI355X through ``lspcg_gnn_forward``."""

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
        self.apply(_weight_init)
        self.node_in_features = node_in_features
        self.edge_in_features = edge_in_features
        self.edge_out_features = edge_out_features
        self.hidden = node_features
        self.num_mp_layers = num_mp_layers
        self.node_residual = node_residual
        self.edge_residual = edge_residual
        self._check_supported(node_features, edge_features, node_encoder, edge_encoder, edge_decoder, node_mlp,
                              edge_mlp, msg_mlp)
        self._handle = None
        self._ctx = None
        self._packed_version = None
        self._graph = None  # (key, edge_index tensor) of the structure analysed by lspcg_gnn_set_graph

    @staticmethod
    def _check_supported(nf, ef, *ffs):
        if nf != 16 or ef != 16:
            raise NotImplementedError("the HIP GNN kernel is specialised for gnn_features = 16 (config/gnn.yaml)")
        for cfg in ffs:
            if cfg.get("num_layers", 2) != 2 or cfg.get("hidden_channels", 16) != 16:
                raise NotImplementedError("the HIP GNN kernel is specialised for gnn_mlp_layers = 2, hidden = 16")
            if cfg.get("activation", "gelu") != "gelu" or cfg.get("out_activation", "none") != "none":
                raise NotImplementedError("the HIP GNN kernel implements GELU hidden / identity output activations")

    # ---- packing
    def pack_weights(self) -> torch.Tensor:
        parts = []

        def ff(m: FeedForward):
            for lin in m.linears():
                parts.append(lin.weight.detach().reshape(-1))
                parts.append(lin.bias.detach().reshape(-1))

        def ln(m: FeedForward):
            if not isinstance(m.pre_norm, nn.LayerNorm):
                raise NotImplementedError("MPLayer MLPs must use pre_norm 'layer' (config/gnn.yaml)")
            parts.append(m.pre_norm.weight.detach().reshape(-1))
            parts.append(m.pre_norm.bias.detach().reshape(-1))

        for enc in (self.node_enc, self.edge_enc):
            if not isinstance(enc.pre_norm, nn.Identity):
                raise NotImplementedError("encoders must use pre_norm 'none' (config/gnn.yaml)")
            ff(enc)
        for mp in self.mp_layers:
            for sub in (mp.node_mlp, mp.edge_mlp, mp.msg_mlp):
                ln(sub)
                ff(sub)
        if not isinstance(self.edge_dec.pre_norm, nn.Identity):
            raise NotImplementedError("edge decoder must use pre_norm 'none' (config/gnn.yaml)")
        ff(self.edge_dec)
        return torch.cat([p.float().cpu() for p in parts]).contiguous()

    def _version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def _ensure_handle(self, device: torch.device):
        ctx = Context.get(device)
        if self._handle is not None and self._ctx is ctx and self._packed_version == self._version():
            return
        self._free()
        self._graph = None
        blob = self.pack_weights()
        desc = _lib.lspcg_gnn_desc(node_in=self.node_in_features, edge_in=self.edge_in_features, hidden=self.hidden,
                                   mlp_layers=2, num_mp_layers=self.num_mp_layers,
                                   edge_out=self.edge_out_features, node_residual=int(self.node_residual),
                                   edge_residual=int(self.edge_residual))
        h = C.c_void_p()
        _lib.call("lspcg_gnn_create", ctx.handle, C.byref(desc), blob.data_ptr(), blob.numel(), C.byref(h))
        self._handle, self._ctx, self._packed_version = h, ctx, self._version()

    def precision(self, device=None) -> dict:
        """Which GEMM kernels ``lspcg_gnn_create`` chose for the current weights:
        ``{"f32": False}`` = split-f16 MFMAs (the default), ``True`` = fp32 MFMAs (weights whose
        LayerNorm-fed hidden activations could pass f16's range, or LSPCG_GNN_F32=1), with the
        weights' hidden-activation bound that decided it (``lspcg_gnn_precision``)."""
        self._ensure_handle(torch.device(device) if device is not None else torch.device("cuda"))
        f32, hb = C.c_int(), C.c_double()
        _lib.call("lspcg_gnn_precision", self._handle, C.byref(f32), C.byref(hb))
        return {"f32": bool(f32.value), "hidden_bound": hb.value}

    def _free(self):
        if self._handle is not None and _lib._lib is not None:
            _lib._lib.lspcg_gnn_destroy(self._handle)
        self._handle = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._packed_version = None
        return res

    def invalidate_graph(self):
        """Forget the cached graph analysis and release the edge_index tensor it holds (the next
        forward re-analyses).  Needed after an in-place change of edge_index that torch's version
        counter does not see (.data, DLPack / CuPy views); also frees the held tensor."""
        self._graph = None

    @torch.no_grad()
    def forward(self, node_attr: torch.Tensor, edge_index: torch.Tensor, edge_attr: torch.Tensor):
        """Returns ``(None, edge_out [E, b*b])``; the reference's node output is the identity
        node decoder of the final node state, which the hot path discards (workspace.py:93)."""
        if not node_attr.is_cuda:
            raise _lib.LspcgUnavailable("NodeEdgeProcessing.forward runs on the GPU only (HIP)")
        dev = node_attr.device
        self._ensure_handle(dev)
        x = node_attr.to(torch.float32).contiguous()
        ea = edge_attr.to(device=dev, dtype=torch.float32).contiguous()
        ei = edge_index.to(device=dev, dtype=torch.int64).contiguous()
        N, E = x.shape[0], ei.shape[1]
        assert x.shape[1] == self.node_in_features, (x.shape, self.node_in_features)
        assert ea.shape == (E, self.edge_in_features), (ea.shape, self.edge_in_features)
        out = torch.empty(E, self.edge_out_features, dtype=torch.float32, device=dev)
        # the graph's CSC is analysed once per edge_index (the tensor is held, so its address cannot
        # be reused by another one while cached; an in-place torch op bumps its version -- writes
        # that bypass the version counter, through .data, DLPack or CuPy views, must be followed by
        # invalidate_graph(), as lspcg_gnn.h asks for lspcg_gnn_set_graph)
        key = (ei.data_ptr(), ei._version, N, E)
        if self._graph is None or self._graph[0] != key or self._graph[1].data_ptr() != ei.data_ptr():
            _lib.call("lspcg_gnn_set_graph", self._handle, N, E, _ptr(ei))
            self._graph = (key, ei)
        _lib.call("lspcg_gnn_forward", self._handle, N, E, _ptr(x), _ptr(ei), _ptr(ea), _ptr(out))
        return None, out


def build_gnn(node_in: int, edge_in: int, block_size: int, seed: Optional[int] = 0, **over) -> NodeEdgeProcessing:
    """Seeded construction with the reference's config (workspace.py:70-76, config/gnn.yaml)."""
    cfg = default_gnn_config()
    cfg.update(over)
    if seed is not None:
        torch.manual_seed(seed)
    return NodeEdgeProcessing(node_in_features=node_in, node_out_features=None, edge_in_features=edge_in,
                              edge_out_features=block_size * block_size, **cfg)


# ---------------------------------------------------------------------------
# GraphSpmv / AATPE / LLT (basic_layers.py:112-142, 228-275) on lspcg_graph_* (HIP)
# ---------------------------------------------------------------------------
class _GraphCache:
    """lspcg_graph handles keyed on the edge_index tensor (held, so its address cannot be reused
    by another tensor while cached), its in-place version, N and the block size."""

    def __init__(self, size: int = 8):
        self.size = size
        self.items = []  # [(key, edge_index tensor, handle)]

    def get(self, edge_index: torch.Tensor, N: int, bs: int) -> C.c_void_p:
        ctx = Context.get(edge_index.device)
        key = (edge_index.data_ptr(), tuple(edge_index.shape), edge_index._version, N, bs, ctx.device)
        for i, (k, t, h) in enumerate(self.items):
            if k == key and t.data_ptr() == edge_index.data_ptr():
                self.items.append(self.items.pop(i))
                return h
        ei = edge_index.to(torch.int64).contiguous()
        h = C.c_void_p()
        _lib.call("lspcg_graph_create", ctx.handle, int(N), int(ei.shape[1]), int(bs), _ptr(ei), C.byref(h))
        self.items.append((key, edge_index, h))
        while len(self.items) > self.size:
            _, _, old = self.items.pop(0)
            if _lib._lib is not None:
                _lib._lib.lspcg_graph_destroy(old)
        return h


_GRAPHS = _GraphCache()


def _graph_args(X: torch.Tensor, edge_index: torch.Tensor, A: torch.Tensor, *opt):
    if not X.is_cuda:
        raise _lib.LspcgUnavailable("GraphSpmv / AATPE run on the GPU only (HIP)")
    if X.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"unsupported dtype {X.dtype}")
    N = X.shape[0]
    bs = X.shape[1] if X.ndim == 2 else 1
    assert A.shape[0] == edge_index.shape[1] and tuple(A.shape[1:]) in ((bs, bs),) + (((1,),) if bs == 1 else ()), \
        (tuple(A.shape), bs)
    dev = X.device
    x = X.contiguous()
    vals = A.to(device=dev, dtype=X.dtype).contiguous()
    out = []
    for o in opt:
        if o is None:
            out.append(None)
        else:
            o = o.to(device=dev, dtype=X.dtype).contiguous()
            assert o.numel() == N * bs, (tuple(o.shape), N, bs)
            out.append(o)
    return N, bs, x, vals, out, _lib.F32 if X.dtype == torch.float32 else _lib.F64


class GraphSpmv(nn.Module):
    """basic_layers.py:112-142: ``y_i = Σ_j A_ij x_j`` over the blocks of an edge list
    (``use_transpose``: ``y = Aᵀ x``), then ``y * mask``.  X is [N, b], A is [E, b, b]."""

    def __init__(self, use_transpose: bool = False):
        super().__init__()
        self.transpose = use_transpose

    @torch.no_grad()
    def forward(self, X, edge_index, A, mask=None):
        N, bs, x, vals, (m,), code = _graph_args(X, edge_index, A, mask)
        h = _GRAPHS.get(edge_index.to(x.device), N, bs)
        y = torch.empty_like(x)
        _lib.call("lspcg_graph_spmv", h, _ptr(vals), code, int(self.transpose), _ptr(x),
                  _ptr(m) if m is not None else None, _ptr(y))
        return y


class AATPE(nn.Module):
    """basic_layers.py:228-261: ``y = ε x + A Aᵀ x`` (``diag``: ``ε diag x + A diag Aᵀ x``), the
    mask applied after each SpMV -- the ext_spai apply on the GNN's own edge-list output."""

    def __init__(self, epsilon):
        super().__init__()
        self.epsilon = float(epsilon)
        self.spmv = GraphSpmv()
        self.spmv_t = GraphSpmv(use_transpose=True)

    @torch.no_grad()
    def forward(self, x, edge_index, boo_values, mask=None, diag=None):
        N, bs, xx, vals, (m, d), code = _graph_args(x, edge_index, boo_values, mask, diag)
        if diag is not None:
            assert tuple(diag.shape) == tuple(x.shape), "diag must have AT_x's shape (basic_layers.py:253)"
        h = _GRAPHS.get(edge_index.to(xx.device), N, bs)
        t = torch.empty_like(xx)
        y = torch.empty_like(xx)
        _lib.call("lspcg_graph_aatpe", h, _ptr(vals), code, self.epsilon, _ptr(xx), _ptr(m) if m is not None else None,
                  _ptr(d) if d is not None else None, _ptr(t), _ptr(y))
        return y


class LLT(nn.Module):
    """basic_layers.py:264-275: ``L Lᵀ x`` with the mask after each SpMV (AATPE with ε = 0)."""

    def __init__(self):
        super().__init__()
        self._op = AATPE(0.0)

    def forward(self, x, edge_index, boo_values, mask=None):
        return self._op(x, edge_index, boo_values, mask)
