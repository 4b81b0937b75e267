"""Build liblspcg_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

``python -m learningsparsepreconditioner4gpu_amd._build`` or ``__graft_entry__.build()``.
Each translation unit compiles to its own object under build/ (in parallel), then hipcc links
the shared library.

Provenance: ``tree_hash()`` hashes every source and header, the C ABI header, the compiler flags
and the target arch; the hash is compiled into the library (``lspcg_build_id()``, plus a
``LSPCG_BUILD_ID=<hash>`` marker string), and the library is rebuilt whenever the marker in the
binary differs from the tree's hash (not on file times).  ``__graft_entry__.smoke()`` asserts the
loaded library's id equals the tree's.
"""
from __future__ import annotations

import hashlib
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
           "lspcg_sell.hip", "lspcg_graph.hip", "lspcg_part.hip", "lspcg_reorder.hip"]
HEADERS = ["lspcg_internal.hpp", "lspcg_spmv.hpp", "lspcg_factor.hpp", "lspcg_sell.hpp"]
ARCH = os.environ.get("LSPCG_ARCH", "gfx950")

# -ffp-contract=off: products are rounded before they are added, exactly like
# scipy's csr_matvec and numpy's ufuncs (bit-identical SpMV / AXPY, DESIGN.md "Parity").
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
          "-Wall", "-Wno-unused-result", "-munsafe-fp-atomics"]
MARKER = b"LSPCG_BUILD_ID="


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build liblspcg_hip.so)")


def _inputs():
    return [CSRC / s for s in SOURCES] + [CSRC / h for h in HEADERS] + [ROOT / "include" / "lspcg.h"]


def tree_hash() -> str:
    """16 hex digits of SHA-256 over (name, bytes) of every input, the flags and the arch."""
    h = hashlib.sha256()
    for p in _inputs():
        h.update(p.name.encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(" ".join(CFLAGS).encode() + b"\0" + ARCH.encode())
    return h.hexdigest()[:16]


def binary_id(path: Path = LIB) -> str:
    """The build id recorded in a built library (its marker string), or '' if absent."""
    if not path.exists():
        return ""
    data = path.read_bytes()
    i = data.find(MARKER)
    return data[i + len(MARKER): i + len(MARKER) + 16].decode(errors="replace") if i >= 0 else ""


def _stale() -> bool:
    return binary_id() != tree_hash()


def _obj(src: str) -> Path:
    return OBJ / (Path(src).stem + ".o")


def _cmd(src: str, bid: str):
    extra = [f'-DLSPCG_BUILD_ID="{bid}"'] if src == "lspcg_core.hip" else []  # the id lives in one TU
    return [hipcc(), *CFLAGS, *extra, f"-I{ROOT / 'include'}", "-c", str(CSRC / src), "-o", str(_obj(src))]


def _obj_hash(src: str, bid: str) -> str:
    """An object is reused only if it was compiled from the same source, headers and command."""
    h = hashlib.sha256(" ".join(_cmd(src, bid)).encode())
    for p in [CSRC / src] + [CSRC / x for x in HEADERS] + [ROOT / "include" / "lspcg.h"]:
        h.update(p.read_bytes())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and not _stale():
        return LIB
    bid = tree_hash()
    OBJ.mkdir(parents=True, exist_ok=True)
    stamp = lambda src: _obj(src).with_suffix(".hash")
    todo = [s for s in SOURCES if force or not _obj(s).exists() or not stamp(s).exists()
            or stamp(s).read_text() != _obj_hash(s, bid)]

    def compile_one(src: str) -> None:
        if stamp(src).exists():
            stamp(src).unlink()
        cmd = _cmd(src, bid)
        if verbose:
            print("[lspcg build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        stamp(src).write_text(_obj_hash(src, bid))

    jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, todo))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), "-shared", f"--offload-arch={ARCH}", *[str(_obj(s)) for s in SOURCES], "-o", str(tmp)]
    if verbose:
        print("[lspcg build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    assert binary_id() == bid, "build id marker missing from the linked library"
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
