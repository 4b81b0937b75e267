"""On-disk dataset reader + GNN feature builder (host-side input plumbing).

Restates ``neural_cg/data.py``:

* ``FolderDataset`` (:339-640) -- the folder format written by ``neural_cg/datagen_helper.py``
  (:230-356): ``mat/NNNNNN.mtx`` (or ``mat/NNNNNN.npy`` value vectors + ``demo.mtx`` for a fixed
  topology), ``mask/``, ``features/``, ``rhs/`` and ``lhs/`` ``.npy`` files, ``shared_features.npy``.
  Same constructor arguments, ``len()``, ``get(idx)``, ``get_internal(idx)``, feature counts and
  (rhs column -> sample) enumeration; ``get`` returns a :class:`GraphSample` instead of a PyG
  ``Data`` (same field names).
* ``to_bcoo_components`` (:15-64) -- block COO in the reference's first-appearance order.
* ``make_data`` (:218-336) -- every option: matrix / node-feature edge features, mask node
  feature, edge->node aggregation (sum / mean / max / min, PyG ``scatter`` semantics: nodes
  without incoming edges get 0), ``normalize_matrix`` mean / frob / l1 / none, rhs / gt.
* ``FolderWriter`` -- the writer side (``datagen_helper.py:230-356``) so stand-in systems can be
  stored and read back through the same path.

Only numpy / scipy / torch on the host; the outputs feed the HIP GNN via ``GraphSample.to``.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import List, Literal, Optional, Sequence, Tuple, Union

import numpy as np
import scipy.sparse as sp
import torch
from scipy.io import mmread, mmwrite

from .data import GraphSample

Reduce = Literal["disable", "sum", "mean", "max", "min"]


@dataclass
class RawData:
    """data.py:159-170."""

    block_values: Optional[np.ndarray]  # [E, b, b]
    diagonals: Optional[np.ndarray]     # [N, b]
    edge_index: np.ndarray              # [2, E] int64
    node_features: Optional[np.ndarray]
    lhs: Optional[np.ndarray]
    rhs: Optional[np.ndarray]
    mask: np.ndarray                    # [N, b]
    num_nodes: int
    block_size: int


def to_bcoo_components(coo: sp.coo_matrix, block_size: int):
    """data.py:15-64: blocks ordered by the first scalar COO entry that touches them (the
    reference fills a dict in COO order); entries not present stay 0."""
    if not isinstance(coo, sp.coo_matrix):
        raise TypeError("Input must be a scipy.sparse.coo_matrix")
    if block_size <= 0:
        raise ValueError("Block size must be positive")
    rows, cols, data = coo.row.astype(np.int64), coo.col.astype(np.int64), coo.data
    br, bc = rows // block_size, cols // block_size
    ncb = int(bc.max()) + 1 if bc.size else 1
    key = br * ncb + bc
    uniq, first, inv = np.unique(key, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")          # blocks in first-appearance order
    rank = np.empty_like(order)
    rank[order] = np.arange(order.size)
    slot = rank[inv]
    vals = np.zeros((uniq.size, block_size, block_size))
    # later duplicates overwrite earlier ones, like the dict assignment
    vals[slot, rows % block_size, cols % block_size] = data
    ku = uniq[order]
    return vals, ku // ncb, ku % ncb


def _scatter(edge_index: torch.Tensor, src: torch.Tensor, num_nodes: int, reduce: str) -> torch.Tensor:
    """torch_geometric.utils.scatter(src, edge_index[1], dim=0, dim_size, reduce) (data.py:173-198)."""
    idx = edge_index[1]
    out = torch.zeros((num_nodes, src.shape[1]), dtype=src.dtype)
    if reduce in ("sum", "add"):
        return out.index_add_(0, idx, src)
    if reduce == "mean":
        s = out.index_add_(0, idx, src)
        cnt = torch.zeros(num_nodes, dtype=src.dtype).index_add_(0, idx, torch.ones_like(idx, dtype=src.dtype))
        return s / cnt.clamp(min=1).unsqueeze(-1)
    if reduce in ("max", "min", "amax", "amin"):
        r = "amax" if reduce in ("max", "amax") else "amin"
        return out.scatter_reduce_(0, idx.unsqueeze(-1).expand_as(src), src, reduce=r, include_self=False)
    raise ValueError(f"unknown reduce {reduce!r}")


def make_bsr_from_coo_inds(values: np.ndarray, rowinds, colinds, block_size: int, block_rows: int,
                           block_cols: int) -> sp.bsr_matrix:
    """data.py:134-156: the CSR structure of the (row, col) pairs with the values taken in the
    given order (i.e. the pairs must already be row-major sorted)."""
    assert values.ndim == 3 and values.shape[1] == values.shape[2] == block_size
    rowinds, colinds = np.asarray(rowinds), np.asarray(colinds)
    assert rowinds.size == colinds.size == values.shape[0]
    csr = sp.csr_matrix((np.ones(rowinds.size), (rowinds, colinds)), shape=(block_rows, block_cols), copy=True)
    return sp.bsr_matrix((values, csr.indices, csr.indptr), blocksize=(block_size, block_size),
                         shape=(block_rows * block_size, block_cols * block_size), copy=True)


def make_data(raw: RawData, use_matrix_as_edge_feature: bool = True, use_mask_as_node_feature: bool = True,
              use_node_features_as_edge_feature: bool = False, use_edge_features_as_node_feature: Reduce = "disable",
              use_random_rhs: bool = True, normalize_matrix: Union[bool, str] = "mean",
              is_inference: bool = True) -> GraphSample:
    """data.py:218-336 -> GraphSample (field names of the reference's Data)."""
    assert not (use_node_features_as_edge_feature and use_edge_features_as_node_feature != "disable")
    edge_index = torch.tensor(raw.edge_index, dtype=torch.long)
    scale = 1.0
    if normalize_matrix is True or normalize_matrix == "mean":
        scale = 1.0 / np.mean(np.abs(raw.block_values))
    elif normalize_matrix == "frob":
        scale = 1.0 / np.linalg.norm(raw.block_values)
    elif normalize_matrix == "l1":
        # as written in data.py:257-264 (block_rows = num_nodes // block_size: valid for b = 1 only,
        # the reference fails the same way for b > 1)
        nbr = raw.num_nodes // raw.block_size
        bsr = make_bsr_from_coo_inds(np.abs(raw.block_values), raw.edge_index[0], raw.edge_index[1], raw.block_size,
                                     nbr, nbr)
        scale = 1.0 / (np.max(bsr @ np.ones(bsr.shape[1])) + 1e-7)
    elif normalize_matrix in ("none", False):
        scale = 1.0
    nodes: List[torch.Tensor] = []
    if raw.node_features is not None:
        nodes.append(torch.tensor(raw.node_features, dtype=torch.float32))
    mask = torch.tensor(raw.mask, dtype=torch.float32)
    if use_mask_as_node_feature:
        nodes.append(mask)
    edges: List[torch.Tensor] = []
    if use_matrix_as_edge_feature:
        edges.append(torch.tensor(scale * raw.block_values, dtype=torch.float32).flatten(1))
    if use_node_features_as_edge_feature:
        assert raw.node_features is not None
        nf = torch.cat(nodes, dim=-1)
        edges += [nf[edge_index[i]] for i in (0, 1)]
    assert edges, "No edge feature found."
    edge_attr = torch.cat(edges, dim=-1)
    if use_edge_features_as_node_feature != "disable":
        nodes.append(_scatter(edge_index, edge_attr, raw.num_nodes, use_edge_features_as_node_feature))
    assert nodes, "No node feature found."
    x = torch.cat(nodes, dim=-1)
    kw = dict(x=x, edge_index=edge_index, edge_attr=edge_attr, mask=mask, block_size=raw.block_size,
              matrix_scale=float(scale))
    assert raw.block_values is not None or not is_inference, "Training depends on matrix values."
    kw["matrix_values"] = (torch.tensor(raw.block_values * scale, dtype=torch.float32)
                           if raw.block_values is not None else None)
    if raw.diagonals is not None:
        diag = raw.diagonals * scale
        kw["diagonal"] = torch.tensor(diag, dtype=torch.float32)
        kw["inv_diag"] = torch.tensor(1.0 / (diag + 1e-7), dtype=torch.float32)
        kw["rsqrt_diag"] = torch.tensor(1.0 / np.sqrt(diag + 1e-7), dtype=torch.float32)
    if not is_inference:
        rhs = torch.randn(raw.num_nodes, raw.block_size, dtype=torch.float32)
        if not use_random_rhs:
            assert raw.rhs is not None
            rhs = torch.tensor(raw.rhs, dtype=torch.float32)
            if raw.lhs is not None:
                kw["gt"] = torch.tensor(raw.lhs, dtype=torch.float32) / scale
        kw["residual"] = rhs * mask
    return GraphSample(**kw)


class FolderDataset:
    """data.py:339-640 (same constructor, enumeration and per-sample semantics)."""

    def __init__(self, is_fixed_topology: bool, load_into_memory: bool, block_size: int, has_shared_features: bool,
                 use_node_features: bool, use_matrix_as_edge_feature: bool, use_mask_as_node_feature: bool,
                 use_node_features_as_edge_feature: bool, use_edge_features_as_node_feature: Reduce,
                 use_random_rhs: bool, normalize_matrix: Union[bool, str], prefix: str):
        self.is_fixed_topology = is_fixed_topology
        self.prefix = prefix
        self.block_size = block_size
        self.path = Path(prefix)
        if is_fixed_topology:
            mats = list((self.path / "mat").glob("*.npy"))
        else:
            mats = list((self.path / "mat").glob("*.mtx")) + list((self.path / "mat").glob("*.npz"))
        self.all_matrices = sorted(mats)
        self.all_lhs = sorted((self.path / "lhs").glob("*.npy"))
        self.all_rhs = sorted((self.path / "rhs").glob("*.npy"))
        self.all_masks = sorted(self.path.glob("mask/*.npy"))
        self.all_features = sorted((self.path / "features").glob("*.npy"))
        self.has_shared_features = has_shared_features
        self.shared_features = np.load(self.path / "shared_features.npy") if has_shared_features else None
        assert len(self.all_matrices) > 0, f"no matrices under {self.path / 'mat'}"
        if self.all_lhs:
            assert len(self.all_lhs) == len(self.all_matrices)
        if self.all_rhs:
            assert len(self.all_rhs) == len(self.all_matrices)
        # one sample per rhs column (data.py:394-400)
        self.samples: List[Tuple[int, int]] = []
        for idx, f in enumerate(self.all_rhs):
            b = np.load(f)
            for i in range(b.shape[1]):
                self.samples.append((idx, i))
        self.use_node_features = use_node_features
        self.use_matrix_as_edge_feature = use_matrix_as_edge_feature
        self.use_mask_as_node_feature = use_mask_as_node_feature
        self.use_node_features_as_edge_feature = use_node_features_as_edge_feature
        self.use_edge_features_as_node_feature = use_edge_features_as_node_feature
        self.use_random_rhs = use_random_rhs
        self.normalize_matrix = normalize_matrix
        # feature counts (data.py:415-433)
        nnf = 0
        if use_node_features:
            assert len(self.all_features) == len(self.all_matrices)
            nnf = np.load(self.all_features[0]).shape[1]
            if has_shared_features:
                nnf += self.shared_features.shape[1]
        if use_mask_as_node_feature:
            nnf += block_size
        if use_node_features_as_edge_feature and use_edge_features_as_node_feature != "disable":
            raise ValueError("You cannot enable both feature enhancers")
        nef = 0
        if use_matrix_as_edge_feature:
            nef += block_size * block_size
        if use_node_features_as_edge_feature:
            nef += nnf * 2
        if use_edge_features_as_node_feature != "disable":
            nnf += nef
        self.num_node_features_, self.num_edge_features_ = nnf, nef
        if is_fixed_topology:  # data.py:437-454
            topo = self.path / "demo.mtx"
            assert topo.exists()
            self.topo_mat_dofs = sp.csr_matrix(mmread(topo)).sorted_indices()
            g = sp.bsr_matrix(self.topo_mat_dofs.tobsr((block_size, block_size))).sorted_indices()
            nn = g.shape[0] // block_size
            graph = sp.coo_matrix(sp.csr_matrix((np.ones(g.indptr[-1]), g.indices, g.indptr), shape=(nn, nn)))
            self.topo_mat_graph = graph
            self.edge_index = np.vstack((graph.row, graph.col)).astype(np.int64)
        self.loaded: List[RawData] = []
        if load_into_memory:
            self.loaded = [self.get_internal(i) for i in range(self.len())]

    def len(self) -> int:
        return max(len(self.all_matrices), len(self.samples))

    __len__ = len

    @property
    def num_node_features(self) -> int:
        return self.num_node_features_

    @property
    def num_edge_features(self) -> int:
        return self.num_edge_features_

    def load(self, mat_file: Path, lhs_file: Optional[Path], rhs_file: Optional[Path], feature_file: Optional[Path],
             mask_file: Optional[Path], dtype=np.float64) -> RawData:
        """data.py:471-572."""
        bs = self.block_size
        if str(mat_file).endswith(".npy"):
            assert self.is_fixed_topology
            values = np.load(mat_file)
            edge_index = self.edge_index
            num_nodes = self.topo_mat_graph.shape[0]
            csr = sp.csr_matrix((values, self.topo_mat_dofs.indices, self.topo_mat_dofs.indptr),
                                shape=self.topo_mat_dofs.shape)
            matrix = sp.bsr_matrix(csr.tobsr((bs, bs))).sorted_indices()
            block_values = matrix.data.astype(dtype).copy()
        else:
            if not str(mat_file).endswith(".mtx"):
                raise ValueError(f"unsupported matrix file {mat_file} (the reference asserts on .npz)")
            matrix = sp.csr_matrix(mmread(mat_file))
            coo = sp.coo_matrix(matrix)
            if bs == 1:
                block_values = coo.data.astype(dtype).reshape(-1, 1, 1).copy()
                edge_index = np.vstack((coo.row, coo.col)).astype(np.int64)
                num_nodes = matrix.shape[0]
            else:
                block_values, brows, bcols = to_bcoo_components(coo, bs)
                edge_index = np.vstack((brows, bcols)).astype(np.int64)
                num_nodes = matrix.shape[0] // bs
        diagonals = matrix.diagonal().reshape(-1, bs)
        lhs = rhs = node_features = None
        if rhs_file is not None:
            rhs = np.load(rhs_file)
            if rhs.ndim == 1:
                rhs = rhs.reshape(-1, 1)
            elif rhs.ndim > 2:
                raise ValueError(f"Unexpected RHS shape: {rhs.shape}")
            assert rhs.shape[0] == num_nodes
            if lhs_file is not None:
                lhs = np.load(lhs_file)
                if lhs.ndim == 1:
                    lhs = lhs.reshape(-1, 1)
                elif lhs.ndim > 2:
                    raise ValueError(f"Unexpected LHS shape: {lhs.shape}")
                assert lhs.shape == rhs.shape
        if self.use_node_features:
            parts = []
            if feature_file is not None:
                feat = np.load(feature_file)
                assert feat.ndim == 2 and feat.shape[0] == num_nodes
                parts.append(feat)
            if self.has_shared_features:
                parts.append(self.shared_features)
            node_features = np.concatenate(parts, axis=-1)
        mask = np.ones((num_nodes, bs), dtype=dtype)
        if mask_file is not None:
            m = np.load(mask_file)
            assert m.shape == mask.shape
            mask = m
        return RawData(block_values, diagonals, edge_index, node_features, lhs, rhs, mask, num_nodes, bs)

    def get_internal(self, idx: int) -> RawData:
        """data.py:584-626: the sub_id-th rhs/lhs column of matrix mat_id."""
        if self.loaded:
            return self.loaded[idx]
        mat_id, sub_id = self.samples[idx] if self.samples else (idx, 0)
        raw = self.load(self.all_matrices[mat_id], self.all_lhs[mat_id] if self.all_lhs else None,
                        self.all_rhs[mat_id] if self.all_rhs else None,
                        self.all_features[mat_id] if self.all_features else None,
                        self.all_masks[mat_id] if self.all_masks else None)
        bs = self.block_size
        return RawData(raw.block_values, raw.diagonals, raw.edge_index, raw.node_features,
                       raw.lhs[:, sub_id].reshape(-1, bs) if raw.lhs is not None else None,
                       raw.rhs[:, sub_id].reshape(-1, bs) if raw.rhs is not None else None,
                       raw.mask, raw.num_nodes, raw.block_size)

    def get(self, idx: int, is_inference: bool = False) -> GraphSample:
        """data.py:628-640."""
        d = make_data(self.get_internal(idx), self.use_matrix_as_edge_feature, self.use_mask_as_node_feature,
                      self.use_node_features_as_edge_feature, self.use_edge_features_as_node_feature,
                      self.use_random_rhs, self.normalize_matrix, is_inference=is_inference)
        assert d.x.shape[-1] == self.num_node_features
        assert d.edge_attr.shape[-1] == self.num_edge_features
        return d

    __getitem__ = get


class FolderWriter:
    """The folder format of datagen_helper.py:230-356 (prepare / append / topology files)."""

    def __init__(self, prefix: str, block_size: int = 1, is_fixed_topology: bool = False, save_rhs: int = 1,
                 save_lhs: bool = False, seed: int = 0):
        self.path = Path(prefix)
        self.block_size = block_size
        self.is_fixed_topology = is_fixed_topology
        self.save_rhs = save_rhs
        self.save_lhs = save_lhs
        self.current_count = 0
        self.rng = np.random.default_rng(seed)
        for d in ("mask", "mat", "features") + (("rhs",) if save_rhs else ()) + (("lhs",) if save_lhs else ()):
            (self.path / d).mkdir(parents=True, exist_ok=True)

    def write_topology(self, topo: sp.spmatrix):
        mmwrite(self.path / "demo.mtx", sp.csr_matrix(topo).sorted_indices())

    def write_shared(self, shared: np.ndarray):
        np.save(self.path / "shared_features.npy", shared)

    def append(self, mat: sp.spmatrix, mask: Optional[np.ndarray] = None, features: Optional[np.ndarray] = None,
               rhs: Union[np.ndarray, Sequence[np.ndarray], None] = None):
        mat = sp.csr_matrix(mat)
        rows = mat.shape[0]
        tag = f"{self.current_count:06d}"
        if self.is_fixed_topology:
            np.save(self.path / "mat" / f"{tag}.npy", mat.sorted_indices().data)
        else:
            mmwrite(self.path / "mat" / f"{tag}.mtx", mat)
        if features is not None:
            features = features.reshape(-1, 1) if features.ndim == 1 else features
            assert features.shape[0] == rows // self.block_size
            np.save(self.path / "features" / f"{tag}.npy", features)
        if mask is not None:
            mask = mask.reshape(-1, 1) if mask.ndim == 1 else mask
            assert mask.shape[0] == rows // self.block_size
            np.save(self.path / "mask" / f"{tag}.npy", mask)
        if self.save_rhs:
            if isinstance(rhs, np.ndarray):
                rhs = [rhs.ravel()]
            elif rhs is not None:
                rhs = [b.ravel() for b in rhs]
            else:
                rhs = []
                for _ in range(int(self.save_rhs)):
                    b = self.rng.standard_normal(rows)
                    b /= np.linalg.norm(b)
                    if mask is not None:
                        b = b * mask.ravel()
                    rhs.append(b)
            np.save(self.path / "rhs" / f"{tag}.npy", np.stack(rhs, 0).T)
            if self.save_lhs:
                from scipy.sparse.linalg import splu

                lu = splu(sp.csc_matrix(mat))
                np.save(self.path / "lhs" / f"{tag}.npy", np.stack([lu.solve(b) for b in rhs], 0).T)
        self.current_count += 1
        return mat
