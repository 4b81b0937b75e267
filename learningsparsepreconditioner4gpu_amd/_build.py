"""Build liblspcg_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

``python -m learningsparsepreconditioner4gpu_amd._build`` or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "liblspcg_hip.so"
SOURCES = ["lspcg_core.hip", "lspcg_pcg.hip", "lspcg_assemble.hip", "lspcg_gnn.hip", "lspcg_factor.hip"]
HEADERS = ["lspcg_internal.hpp", "lspcg_spmv.hpp", "lspcg_factor.hpp"]
ARCH = os.environ.get("LSPCG_ARCH", "gfx950")

# -ffp-contract=off: products are rounded before they are added, exactly like
# scipy's csr_matvec and numpy's ufuncs (bit-identical SpMV / AXPY, DESIGN.md "Parity").
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-Wall", "-Wno-unused-result", "-munsafe-fp-atomics"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build liblspcg_hip.so)")


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + HEADERS] + [ROOT / "include" / "lspcg.h"]
    return any(p.exists() and p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and not _stale():
        return LIB
    srcs = [str(CSRC / s) for s in SOURCES if (CSRC / s).exists()]
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), *FLAGS, f"-I{ROOT / 'include'}", *srcs, "-o", str(tmp)]
    if verbose:
        print("[lspcg build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
