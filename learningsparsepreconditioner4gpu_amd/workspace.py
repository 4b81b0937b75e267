"""Inference workspace: GNN -> L in HBM, the hot half of ``SimpleTrainingWorkspace``.

Mirrors ``neural_cg/workspace.py`` (``forward`` :92-94, ``inference_step`` :195-205) and
``neural_cg/scaled_workspace.py`` (``inference_step`` :199-212) without Lightning: the
GNN runs as HIP kernels and L is assembled on the GPU with ``to_csr_cpu`` semantics
(``lspcg_assemble``), so nothing is copied back to the host.  ``dt`` has the reference's
meaning: wall time of the GNN forward until its result is available (the reference stops
the clock after ``.cpu()``, i.e. after a device sync).
"""
from __future__ import annotations

from time import time
from typing import Optional, Tuple, Union

import numpy as np
import scipy.sparse as sp
import torch

from .data import GraphSample
from .nn import NodeEdgeProcessing, build_gnn, default_gnn_config
from .sparse import DeviceMatrix, assemble


# ---- weights-only loading of Lightning checkpoints with OmegaConf hparams ------------------------
# The reference trains with Hydra: train.py:56-60 builds the workspace with ``**cfg`` (a DictConfig),
# and workspace.py:52 ``save_hyperparameters()`` stores those arguments, so ``hyper_parameters``
# holds omegaconf containers (``gnn``, ``optimizer``, ...).  torch's weights-only unpickler refuses
# their classes.  Instead of unpickling them (``weights_only=False`` would run whatever the file
# names), the names below are allowlisted to INERT stand-ins: plain attribute holders that only
# receive the pickled state (NEWOBJ = ``object.__new__``, BUILD = ``__dict__.update``), which
# ``_plain`` then folds into plain dicts / lists / values.  Nothing of omegaconf or lightning is
# imported or executed; any other global in the file is still refused.
class _OmegaContainer:
    """Stand-in for an omegaconf DictConfig / ListConfig: pickled state {_metadata, _parent, _content}."""


class _OmegaValueNode:
    """Stand-in for an omegaconf value node (AnyNode, StringNode, ...): state {_metadata, _parent, _val}."""


class _OmegaMetadata:
    """Stand-in for omegaconf.base.Metadata / ContainerMetadata (ignored by _plain)."""


class _AttributeDict:
    """Stand-in for Lightning's AttributeDict (a dict subclass): NEWOBJ makes a plain dict, which
    the unpickler's SETITEMS then fills."""

    def __new__(cls, *args):
        return {}


class _TypeRef:
    """Stand-in for a type object named in omegaconf metadata (typing.Any, builtins.dict, ...)."""

    def __init__(self, name: str):
        self.name = name


def _defaultdict_standin(*_args):  # collections.defaultdict(factory) in omegaconf's resolver cache
    return {}


_OMEGA_NODES = ("AnyNode", "StringNode", "IntegerNode", "FloatNode", "BooleanNode", "BytesNode", "PathNode")
_TYPE_NAMES = ("typing.Any", "typing.Dict", "typing.List", "typing.Optional", "typing.Union", "builtins.dict",
               "builtins.list", "builtins.str", "builtins.int", "builtins.float", "builtins.bool", "builtins.object",
               "builtins.NoneType", "builtins.bytes")


def _checkpoint_safe_globals():
    g = [(_OmegaContainer, "omegaconf.dictconfig.DictConfig"), (_OmegaContainer, "omegaconf.listconfig.ListConfig"),
         (_OmegaMetadata, "omegaconf.base.Metadata"), (_OmegaMetadata, "omegaconf.base.ContainerMetadata"),
         (_defaultdict_standin, "collections.defaultdict")]
    g += [(_OmegaValueNode, f"omegaconf.nodes.{n}") for n in _OMEGA_NODES]
    g += [(_AttributeDict, n) for n in ("lightning.fabric.utilities.data.AttributeDict",
                                        "lightning_fabric.utilities.data.AttributeDict",
                                        "pytorch_lightning.utilities.parsing.AttributeDict")]
    g += [(_TypeRef(n), n) for n in _TYPE_NAMES]
    return g


def _plain(o):
    """Fold the stand-ins into plain Python: containers by their ``_content``, nodes by their
    ``_val`` (``_parent`` back references and metadata are dropped)."""
    if isinstance(o, _OmegaContainer):
        c = o.__dict__.get("_content")
        if isinstance(c, dict):
            return {k: _plain(v) for k, v in c.items()}
        if isinstance(c, (list, tuple)):
            return [_plain(v) for v in c]
        return c  # None or a "???" / interpolation string
    if isinstance(o, _OmegaValueNode):
        return _plain(o.__dict__.get("_val"))
    if isinstance(o, dict):
        return {k: _plain(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_plain(v) for v in o)
    return o


def load_checkpoint_weights_only(path: str):
    """``torch.load(path, weights_only=True)`` with the OmegaConf / Lightning hparam classes
    allowlisted to inert stand-ins (above); returns the checkpoint with ``hyper_parameters``
    as plain dicts."""
    with torch.serialization.safe_globals(_checkpoint_safe_globals()):
        ck = torch.load(path, map_location="cpu", weights_only=True)
    if "hyper_parameters" in ck:
        ck["hyper_parameters"] = _plain(ck["hyper_parameters"])
    return ck


class SimpleInferenceWorkspace:
    def __init__(self, node_features: int, edge_features: int, block_size: int = 1, epsilon: float = 3e-3,
                 gnn: Optional[dict] = None, seed: Optional[int] = 0, device: Union[str, torch.device] = "cuda"):
        self.block_size = block_size
        self.epsilon = float(epsilon)
        cfg = default_gnn_config() if gnn is None else dict(gnn)
        if seed is not None:
            torch.manual_seed(seed)
        self.gnn = NodeEdgeProcessing(node_in_features=node_features, node_out_features=None,
                                      edge_in_features=edge_features, edge_out_features=block_size * block_size,
                                      **cfg)
        self.device = torch.device(device)

    # ---- checkpoints (workspace.py:52 save_hyperparameters; infer.py:237 load_from_checkpoint)
    @classmethod
    def load_from_checkpoint(cls, path: str, device="cuda", trusted: bool = False) -> "SimpleInferenceWorkspace":
        """Load a Lightning checkpoint of the reference: ``hyper_parameters`` (block_size, epsilon,
        node_features, edge_features, gnn) and ``state_dict['gnn.*']``.  Loaded weights-only
        (``load_checkpoint_weights_only``: the reference's OmegaConf hparams come back as plain
        dicts through inert stand-ins) unless ``trusted=True`` (only for files you produced
        yourself, with omegaconf installed)."""
        ck = (torch.load(path, map_location="cpu", weights_only=False) if trusted
              else load_checkpoint_weights_only(path))
        hp = ck.get("hyper_parameters", {})
        gnn_cfg = hp.get("gnn")
        ws = cls(node_features=int(hp["node_features"]), edge_features=int(hp["edge_features"]),
                 block_size=int(hp.get("block_size", 1)), epsilon=float(hp.get("epsilon", 3e-3)),
                 gnn=None if gnn_cfg is None else {k: (dict(v) if hasattr(v, "items") else v)
                                                    for k, v in dict(gnn_cfg).items()},
                 seed=None, device=device)
        sd = {k[len("gnn."):]: v for k, v in ck["state_dict"].items() if k.startswith("gnn.")}
        ws.gnn.load_state_dict(sd, strict=True)
        return ws

    def to(self, device) -> "SimpleInferenceWorkspace":
        self.device = torch.device(device)
        return self

    def eval(self) -> "SimpleInferenceWorkspace":
        return self

    # ---- workspace.py:92-94
    def forward(self, node_attr, edge_index, edge_attr) -> torch.Tensor:
        _, boo = self.gnn(node_attr, edge_index, edge_attr)
        return boo.reshape(-1, self.block_size, self.block_size)

    __call__ = forward

    def _assemble(self, sample: GraphSample, boo: torch.Tensor, block_output: Optional[bool]) -> DeviceMatrix:
        n = sample.num_nodes * self.block_size
        bo = (self.block_size > 1) if block_output is None else block_output
        return assemble(sample.edge_index, boo, n, sample.mask, dtype=torch.float64, block_output=bo)

    # ---- workspace.py:195-205
    def inference_step(self, sample: GraphSample, time_beg: Optional[float] = None, block_output: Optional[bool] = None,
                       return_scipy: bool = False) -> Tuple[Union[DeviceMatrix, sp.csr_matrix], float]:
        s = sample if sample.x.is_cuda else sample.to(self.device)
        # the reference's clock starts with no device work pending (its to_csr_cpu is synchronous);
        # here a previous call's assembly may still be queued
        torch.cuda.synchronize(s.x.device)
        time_beg = time()
        boo = self.forward(s.x, s.edge_index, s.edge_attr)
        torch.cuda.synchronize(boo.device)
        dt = time() - time_beg
        L = self._assemble(s, boo, block_output)
        return (L.to_scipy().tocsr() if return_scipy else L), dt

    def inference_step_batch(self, samples, block_output: Optional[bool] = None):
        """inference_step over a window of graphs as ONE GNN forward on their disjoint union (not in
        the reference, which runs one forward per sample, infer.py:280): node ids offset per graph,
        so the union keeps row-major sorted edges and every node aggregates exactly its own graph's
        messages in the same order -- each L equals the single forward's bit for bit.  Returns
        ``([L_k], dt)`` with dt the wall time of the one forward (the reference's clock)."""
        ss = [s if s.x.is_cuda else s.to(self.device) for s in samples]
        offs, off = [], 0
        for s in ss:
            offs.append(off)
            off += s.num_nodes
        x = torch.cat([s.x for s in ss])
        ei = torch.cat([s.edge_index + o for s, o in zip(ss, offs)], dim=1)
        ea = torch.cat([s.edge_attr for s in ss])
        torch.cuda.synchronize(x.device)
        time_beg = time()
        boo = self.forward(x, ei, ea)
        torch.cuda.synchronize(boo.device)
        dt = time() - time_beg
        Ls, e0 = [], 0
        for s in ss:
            E = s.edge_index.shape[1]
            Ls.append(self._assemble(s, boo[e0:e0 + E], block_output))
            e0 += E
        return Ls, dt

    def system_matrix(self, sample: GraphSample, block_output: Optional[bool] = None) -> DeviceMatrix:
        """``to_csr_cpu(edge_index, matrix_values, n, mask)`` (infer.py:282) on the device."""
        s = sample if sample.x.is_cuda else sample.to(self.device)
        return self._assemble(s, s.matrix_values, block_output)


class ScaledInferenceWorkspace(SimpleInferenceWorkspace):
    """scaled_workspace.py:199-212: L <- L · diag(rsqrt(diag(A) + 1e-7)), solved with ext_spai_scaled."""

    def inference_step(self, sample: GraphSample, time_beg: Optional[float] = None, block_output: Optional[bool] = None,
                       return_scipy: bool = False):
        s = sample if sample.x.is_cuda else sample.to(self.device)
        # the reference's clock starts with no device work pending (its to_csr_cpu is synchronous);
        # here a previous call's assembly may still be queued
        torch.cuda.synchronize(s.x.device)
        time_beg = time()
        boo = self.forward(s.x, s.edge_index, s.edge_attr)
        torch.cuda.synchronize(boo.device)
        dt = time() - time_beg
        L = self._assemble(s, boo, block_output)
        L.scale_columns_(s.rsqrt_diag.reshape(-1).to(torch.float64))
        return (L.to_scipy().tocsr() if return_scipy else L), dt
