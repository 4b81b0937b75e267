"""Build liblspcg_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

``python -m learningsparsepreconditioner4gpu_amd._build`` or ``__graft_entry__.build()``.
Each translation unit compiles to its own object under build/ (in parallel, only when stale),
then hipcc links the shared library.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "liblspcg_hip.so"
OBJ = ROOT / "build" / "lspcg"
SOURCES = ["lspcg_core.hip", "lspcg_pcg.hip", "lspcg_assemble.hip", "lspcg_gnn.hip", "lspcg_factor.hip",
           "lspcg_sell.hip", "lspcg_graph.hip", "lspcg_part.hip"]
HEADERS = ["lspcg_internal.hpp", "lspcg_spmv.hpp", "lspcg_factor.hpp", "lspcg_sell.hpp"]
ARCH = os.environ.get("LSPCG_ARCH", "gfx950")

# -ffp-contract=off: products are rounded before they are added, exactly like
# scipy's csr_matvec and numpy's ufuncs (bit-identical SpMV / AXPY, DESIGN.md "Parity").
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
          "-Wall", "-Wno-unused-result", "-munsafe-fp-atomics"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build liblspcg_hip.so)")


def _mtime(p: Path) -> float:
    return p.stat().st_mtime if p.exists() else 0.0


def _hdr_time() -> float:
    return max(_mtime(p) for p in [CSRC / h for h in HEADERS] + [ROOT / "include" / "lspcg.h"])


def _obj(src: str) -> Path:
    return OBJ / (Path(src).stem + ".o")


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return _hdr_time() > t or any(_mtime(CSRC / s) > t for s in SOURCES)


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and not _stale():
        return LIB
    OBJ.mkdir(parents=True, exist_ok=True)
    hdr = _hdr_time()
    todo = [s for s in SOURCES if force or _mtime(_obj(s)) < max(hdr, _mtime(CSRC / s))]

    def compile_one(src: str) -> None:
        cmd = [hipcc(), *CFLAGS, f"-I{ROOT / 'include'}", "-c", str(CSRC / src), "-o", str(_obj(src))]
        if verbose:
            print("[lspcg build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, todo))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), "-shared", f"--offload-arch={ARCH}", *[str(_obj(s)) for s in SOURCES], "-o", str(tmp)]
    if verbose:
        print("[lspcg build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
