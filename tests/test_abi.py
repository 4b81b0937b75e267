"""CPU: the C-ABI library loads and exports exactly the entry points include/lspcg.h declares
(no compute calls -- there is no GPU here)."""
import re
import subprocess

import pytest

from tests.conftest import ROOT


def _header_functions():
    txt = (ROOT / "include" / "lspcg.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(lspcg_[a-z0-9_]+)\s*\(", txt))


def test_header_matches_binding_table():
    from learningsparsepreconditioner4gpu_amd import _lib

    assert _header_functions() == set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    from learningsparsepreconditioner4gpu_amd import _lib

    lib_path = _lib.LIB_PATH
    if not lib_path.exists():
        pytest.fail(f"{lib_path} not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib_path)], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (lspcg_[a-z0-9_]+)$", out.stdout, flags=re.M))
    missing = _header_functions() - exported
    assert not missing, missing
    lib = _lib.load()  # resolves and types every symbol via ctypes
    assert lib.lspcg_version() >= 10000


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from learningsparsepreconditioner4gpu_amd import _lib
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd import problems as P

    A = P.kuhn_laplacian(3)
    with pytest.raises(_lib.LspcgUnavailable):
        PreconditionedConjugateGradient(A, device="cuda", preconditioner="none")
    with pytest.raises(RuntimeError, match="pymathprim"):  # the reference's CPU backend, absent here
        PreconditionedConjugateGradient(A, device="cpu", preconditioner="none")
    with pytest.raises(ValueError, match="expected 'cuda'"):
        PreconditionedConjugateGradient(A, device="tpu", preconditioner="none")
    with pytest.raises(NotImplementedError):
        PreconditionedConjugateGradient(A, device="cuda", preconditioner="fsai")


def test_product_never_imports_oracle():
    """The product package must not import the CPU oracle (it is test infrastructure)."""
    pkg = ROOT / "learningsparsepreconditioner4gpu_amd"
    for f in pkg.rglob("*.py"):
        src = f.read_text()
        assert not re.search(r"^\s*(from|import)\s+oracle\b", src, flags=re.M), f


def test_host_solver_only_in_cpu_rows():
    """The only host (scipy) CG in the package is cpu_rows.py -- the reference's own scipy
    restatement behind infer's opt-in --cpu-rows comparison rows and the *_scipy names of
    validate.py; no device-path module calls it or falls back to it."""
    pkg = ROOT / "learningsparsepreconditioner4gpu_amd"
    users = []
    for f in sorted(pkg.rglob("*.py")):
        src = f.read_text()
        # a host CG solve (scipy's cg) or a route to one (cpu_rows); dataset.FolderWriter's splu is the
        # offline dataset writer's reference solution (datagen_helper.py), not a solver path
        if re.search(r"import[^\n]*\bcg\b|\bcg\(|\bcpu_rows\b", src):
            users.append(f.name)
    assert set(users) <= {"cpu_rows.py", "validate.py", "infer.py"}, users
    vsrc = (pkg / "validate.py").read_text()
    # validate only re-exports the host names; its device functions never reach them
    body = vsrc.split("from .cpu_rows import")[1]
    assert "get_pcg_iter_time_scipy" not in body.split(")", 1)[1]
    isrc = (pkg / "infer.py").read_text()
    assert len(re.findall(r"cpu_rows\.\w+\(", isrc)) == 2 and "if args.cpu_rows" in isrc
