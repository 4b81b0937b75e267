"""Device-resident sparse matrices (CSR / BSR3) on MI355X, owned by liblspcg_hip.so handles.

``DeviceMatrix`` is the handle the solver consumes; ``Context`` pins a device and the
stream the library issues on (the default stream, shared with PyTorch).
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple, Optional, Union

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib

_TORCH = {_lib.F32: torch.float32, _lib.F64: torch.float64}
_NP = {_lib.F32: np.float32, _lib.F64: np.float64}


def lspcg_dtype(dtype) -> int:
    if isinstance(dtype, torch.dtype):
        table = {torch.float32: _lib.F32, torch.float64: _lib.F64}
    else:
        dtype = np.dtype(dtype)
        table = {np.dtype(np.float32): _lib.F32, np.dtype(np.float64): _lib.F64}
    if dtype not in table:
        raise TypeError(f"unsupported dtype {dtype} (float32 / float64 only)")
    return table[dtype]


def _ptr(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


class Context:
    """One library context per device (the default stream of that device)."""

    _cache = {}

    def __init__(self, device: int = 0):
        if not torch.cuda.is_available():
            raise _lib.LspcgUnavailable("no ROCm GPU visible: the lspcg HIP path needs an MI355X (gfx950)")
        lib = _lib.load()
        self.device = int(device)
        h = C.c_void_p()
        _lib.check(lib.lspcg_ctx_create(self.device, None, C.byref(h)))
        self.handle = h

    @classmethod
    def get(cls, device: Optional[Union[int, torch.device, str]] = None) -> "Context":
        if not torch.cuda.is_available():
            raise _lib.LspcgUnavailable("no ROCm GPU visible: the lspcg HIP path needs an MI355X (gfx950)")
        if device is None:
            dev = torch.cuda.current_device()
        elif isinstance(device, (torch.device, str)):
            d = torch.device(device)
            dev = d.index if d.index is not None else torch.cuda.current_device()
        else:
            dev = int(device)
        if dev not in cls._cache:
            cls._cache[dev] = Context(dev)
        return cls._cache[dev]

    @property
    def torch_device(self) -> torch.device:
        return torch.device("cuda", self.device)

    def synchronize(self):
        _lib.call("lspcg_ctx_synchronize", self.handle)


class DeviceMatrix:
    """A square sparse matrix in HBM: scalar CSR (block_size 1) or BSR with 3x3 blocks."""

    def __init__(self, handle: C.c_void_p, ctx: Context):
        self.handle = handle
        self.ctx = ctx
        n, nnzb, bs, dt = C.c_int64(), C.c_int64(), C.c_int(), C.c_int()
        _lib.call("lspcg_mat_info", handle, C.byref(n), C.byref(nnzb), C.byref(bs), C.byref(dt))
        self.n, self.nnzb, self.block_size, self.dtype_code = n.value, nnzb.value, bs.value, dt.value
        self.version = 0  # bumped by in-place value changes (solvers key their installed L on it)

    # ---- construction
    @classmethod
    def from_scipy(cls, A, dtype=np.float64, block_size: int = 1, ctx: Optional[Context] = None,
                   keep_order: bool = False) -> "DeviceMatrix":
        """``keep_order`` (scalar CSR): upload each row's entries in their stored order (the
        SpMV sums a row in stored order; dist_pcg's extended matrices rely on it)."""
        ctx = ctx or Context.get()
        code = lspcg_dtype(dtype)
        npdt = _NP[code]
        if block_size == 1:
            A = sp.csr_matrix(A)
            if not keep_order and not A.has_sorted_indices:
                A = A.sorted_indices()
            indptr = np.ascontiguousarray(A.indptr, dtype=np.int32)
            indices = np.ascontiguousarray(A.indices, dtype=np.int32)
            vals = np.ascontiguousarray(A.data, dtype=npdt)
            nb, nnzb = A.shape[0], indices.size
        else:
            B = A if isinstance(A, sp.bsr_matrix) and A.blocksize == (block_size, block_size) else \
                sp.bsr_matrix(sp.csr_matrix(A), blocksize=(block_size, block_size))
            B.sort_indices()
            indptr = np.ascontiguousarray(B.indptr, dtype=np.int32)
            indices = np.ascontiguousarray(B.indices, dtype=np.int32)
            vals = np.ascontiguousarray(B.data, dtype=npdt)
            nb, nnzb = B.shape[0] // block_size, indices.size
        h = C.c_void_p()
        _lib.call("lspcg_mat_create_bsr", ctx.handle, nb, nnzb, block_size,
                  indptr.ctypes.data_as(C.c_void_p), indices.ctypes.data_as(C.c_void_p),
                  vals.ctypes.data_as(C.c_void_p), code, C.byref(h))
        return cls(h, ctx)

    @classmethod
    def from_device_csr(cls, indptr: torch.Tensor, indices: torch.Tensor, vals: torch.Tensor, n: int,
                        block_size: int = 1, ctx: Optional[Context] = None) -> "DeviceMatrix":
        ctx = ctx or Context.get(vals.device)
        code = lspcg_dtype(vals.dtype)
        h = C.c_void_p()
        _lib.call("lspcg_mat_create_bsr", ctx.handle, n // block_size, indices.numel(), block_size,
                  _ptr(indptr.int().contiguous()), _ptr(indices.int().contiguous()), _ptr(vals.contiguous()),
                  code, C.byref(h))
        return cls(h, ctx)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.lspcg_mat_destroy(h)
            self.handle = None

    # ---- properties
    @property
    def shape(self):
        return (self.n, self.n)

    @property
    def nnz(self) -> int:
        return self.nnzb * self.block_size * self.block_size

    @property
    def dtype(self) -> torch.dtype:
        return _TORCH[self.dtype_code]

    def empty_vector(self) -> torch.Tensor:
        return torch.empty(self.n, dtype=self.dtype, device=self.ctx.torch_device)

    # ---- operations
    def to_scipy(self):
        nb = self.n // self.block_size
        indptr = np.empty(nb + 1, np.int32)
        indices = np.empty(self.nnzb, np.int32)
        vals = np.empty(self.nnzb * self.block_size ** 2, _NP[self.dtype_code])
        _lib.call("lspcg_mat_copy_out", self.handle, indptr.ctypes.data_as(C.c_void_p),
                  indices.ctypes.data_as(C.c_void_p), vals.ctypes.data_as(C.c_void_p))
        if self.block_size == 1:
            return sp.csr_matrix((vals, indices, indptr), shape=self.shape)
        b = self.block_size
        return sp.bsr_matrix((vals.reshape(-1, b, b), indices, indptr), shape=self.shape, blocksize=(b, b))

    def transpose(self) -> "DeviceMatrix":
        h = C.c_void_p()
        _lib.call("lspcg_mat_transpose", self.handle, C.byref(h))
        return DeviceMatrix(h, self.ctx)

    @property
    def T(self) -> "DeviceMatrix":
        return self.transpose()

    def ic0(self) -> Tuple["DeviceMatrix", float]:
        """IC(0) factor L (tril pattern, A ≈ L Lᵀ) on the device; returns (L, setup seconds)."""
        h, ms = C.c_void_p(), C.c_double()
        _lib.call("lspcg_ic0", self.handle, C.byref(h), C.byref(ms))
        return DeviceMatrix(h, self.ctx), ms.value / 1e3

    def ainv0(self) -> Tuple["DeviceMatrix", float]:
        """AINV(0) factor L = Z D^{-1/2} (L Lᵀ ≈ A⁻¹) on the device; returns (L, setup seconds)."""
        h, ms = C.c_void_p(), C.c_double()
        _lib.call("lspcg_ainv0", self.handle, C.byref(h), C.byref(ms))
        return DeviceMatrix(h, self.ctx), ms.value / 1e3

    def trsv(self, b: torch.Tensor, lower: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x = T⁻¹ b for a triangular matrix (lower: diagonal last per row; upper: first)."""
        b = b.to(device=self.ctx.torch_device, dtype=self.dtype).contiguous()
        x = self.empty_vector() if out is None else out
        _lib.call("lspcg_trsv", self.handle, int(bool(lower)), _ptr(b), _ptr(x))
        return x

    def rcm(self):
        """The solver's reordering analysis (lspcg_mat_rcm): (perm | None, mean |col - row| before,
        after) -- perm[i'] = the old block row placed at i' (reverse Cuthill-McKee), None when the
        graph is left in its order."""
        perm = torch.empty(self.n // self.block_size, dtype=torch.int32, device=self.ctx.torch_device)
        applied = C.c_int(0)
        before, after = C.c_double(0.0), C.c_double(0.0)
        _lib.call("lspcg_mat_rcm", self.handle, _ptr(perm), C.byref(applied), C.byref(before), C.byref(after))
        return (perm if applied.value else None), before.value, after.value

    def diagonal(self) -> torch.Tensor:
        d = self.empty_vector()
        _lib.call("lspcg_mat_diagonal", self.handle, _ptr(d))
        return d

    def scale_columns_(self, d: torch.Tensor) -> "DeviceMatrix":
        d = d.to(device=self.ctx.torch_device, dtype=self.dtype).contiguous()
        assert d.numel() == self.n
        _lib.call("lspcg_mat_scale_columns", self.handle, _ptr(d))
        self.version += 1
        return self

    def matvec(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        x = x.to(device=self.ctx.torch_device, dtype=self.dtype).contiguous()
        assert x.numel() == self.n, f"x has {x.numel()} entries, matrix has {self.n} columns"
        y = self.empty_vector() if out is None else out
        _lib.call("lspcg_spmv", self.ctx.handle, self.handle, _ptr(x), _ptr(y))
        return y

    __matmul__ = matvec

    def prepare_spmv(self) -> int:
        """Analysis step: attach a SELL-64 copy that :meth:`matvec` then uses (same bits).
        Returns the column storage (1 = SELL-DIA, 16 = 16-bit offsets, 17 = SELL-64J, 18 = SELL-64X,
        32 = int32) or 0 when the CSR kernel stays in use.  A numbering far from banded is analysed
        on its reverse-Cuthill-McKee permutation (:attr:`spmv_reorder_info`)."""
        kind = C.c_int()
        _lib.call("lspcg_mat_prepare_spmv", self.handle, C.byref(kind))
        return kind.value

    @property
    def spmv_reorder_info(self) -> dict:
        """The analysis step's reordering: applied, mean |col - row| before / after (lspcg_mat_spmv_reorder_info)."""
        ap, before, after = C.c_int(), C.c_double(), C.c_double()
        _lib.call("lspcg_mat_spmv_reorder_info", self.handle, C.byref(ap), C.byref(before), C.byref(after))
        return {"applied": bool(ap.value), "mean_offset_before": before.value, "mean_offset_after": after.value}

    def spmv_timed(self, x: torch.Tensor, y: torch.Tensor, reps: int, flush_bytes: int = 0) -> float:
        """Average device ms of one SpMV launch: ``reps`` back-to-back launches (warm), or with
        ``flush_bytes`` > 0 each launch timed alone after an Infinity-Cache-evicting memset (cold)."""
        ms = C.c_double()
        _lib.call("lspcg_spmv_timed", self.ctx.handle, self.handle, _ptr(x), _ptr(y), int(reps), int(flush_bytes),
                  C.byref(ms))
        return ms.value


def dot(x: torch.Tensor, y: torch.Tensor, ctx: Optional[Context] = None) -> float:
    """Compensated deterministic dot product of two device vectors (HIP)."""
    ctx = ctx or Context.get(x.device)
    assert x.dtype == y.dtype and x.numel() == y.numel()
    out = C.c_double()
    _lib.call("lspcg_dot", ctx.handle, x.numel(), lspcg_dtype(x.dtype), _ptr(x.contiguous()),
              _ptr(y.contiguous()), C.byref(out))
    return out.value


def assemble(edge_index: torch.Tensor, blocks: torch.Tensor, n: int, mask: Optional[torch.Tensor] = None,
             dtype=torch.float64, block_output: bool = False, ctx: Optional[Context] = None) -> DeviceMatrix:
    """``to_csr_cpu`` on the GPU (validate.py:22-51): COO block edges -> masked CSR/BSR in HBM.

    ``blocks`` is ``[E]`` / ``[E,1,1]`` (scalar) or ``[E,b,b]``; ``n`` is the scalar size.
    ``block_output=False`` reproduces to_csr_cpu exactly (scalar CSR, zeros dropped);
    ``block_output=True`` keeps b x b blocks for the BSR kernels.
    """
    ctx = ctx or Context.get(blocks.device if blocks.is_cuda else None)
    dev = ctx.torch_device
    if blocks.ndim == 1:
        blocks = blocks.reshape(-1, 1, 1)
    assert blocks.ndim == 3 and blocks.shape[1] == blocks.shape[2]
    bs = blocks.shape[-1]
    ei = edge_index.to(device=dev, dtype=torch.int64).contiguous()
    bl = blocks.to(device=dev).contiguous()
    if bl.dtype not in (torch.float32, torch.float64):
        bl = bl.double()
    m = None
    mcode = _lib.F64
    if mask is not None:
        m = mask.to(device=dev).reshape(-1).contiguous()
        if m.dtype not in (torch.float32, torch.float64):
            m = m.double()
        mcode = lspcg_dtype(m.dtype)
        assert m.numel() == n
    h = C.c_void_p()
    _lib.call("lspcg_assemble", ctx.handle, n // bs, ei.shape[1], bs, _ptr(ei), _ptr(bl), lspcg_dtype(bl.dtype),
              _ptr(m) if m is not None else None, mcode, lspcg_dtype(dtype), int(block_output), C.byref(h))
    return DeviceMatrix(h, ctx)
