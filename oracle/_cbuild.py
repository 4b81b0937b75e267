"""Build / load the oracle's C restatements (oracle/*.c) -- TEST INFRASTRUCTURE ONLY.

``gcc -O2 -ffp-contract=off -shared`` into ``oracle/liboracle.so`` (git-ignored; it travels to
the GPU box with the tree like the product's library).  ``__graft_entry__.build()`` calls
``build()``; ``lib()`` builds on first use when the .so is missing or older than a source.
"""
from __future__ import annotations

import ctypes as C
import shutil
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SOURCES = ["openblas_ddot.c"]
LIB = HERE / "liboracle.so"
_lib = None


def _stale() -> bool:
    return not LIB.exists() or any((HERE / s).stat().st_mtime > LIB.stat().st_mtime for s in SOURCES)


def build(force: bool = False) -> Path:
    if force or _stale():
        cc = shutil.which("gcc") or shutil.which("cc")
        if cc is None:
            raise RuntimeError("gcc not found: the oracle's C restatements cannot be built")
        tmp = LIB.with_suffix(".so.tmp")
        subprocess.run([cc, "-O2", "-ffp-contract=off", "-fPIC", "-shared", *[str(HERE / s) for s in SOURCES],
                        "-lm", "-o", str(tmp)], check=True)
        tmp.replace(LIB)
    return LIB


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = C.CDLL(str(build()))
        _lib.lspcg_oracle_openblas_ddot.restype = C.c_double
        _lib.lspcg_oracle_openblas_ddot.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_int]
    return _lib
