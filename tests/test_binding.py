"""The documented binding runs the reference's UNCHANGED infer loop.

``/root/reference/infer.py:316-325`` calls ``get_cg_iter_time(..., device=d)`` for d in ("cpu",
"cuda") and ``pcg(..., device="cpu")`` / ``device="cuda"`` from one ``try`` whose handler is
``except RuntimeError`` (:363).  With the binding in place (validate.py's
``PreconditionedConjugateGradient`` = ours) the CPU device must still reach pymathprim -- the
reference's CPU backend, stubbed here because it is not installed -- and the CUDA device our
MI355X class (which, in this GPU-less container, raises ``LspcgUnavailable``).  Without
pymathprim the CPU row raises a ``RuntimeError`` (never ``ValueError``), which the reference's
loop catches.
"""
import sys
import types

import numpy as np
import pytest
import torch

from learningsparsepreconditioner4gpu_amd import _lib, linalg, validate
from learningsparsepreconditioner4gpu_amd import problems as P


class _StubPCG:
    """Records what the reference's validate.py hands to pymathprim; solves nothing (returns a
    fixed triple with x untouched), so the assertions are about dispatch only."""

    calls = []

    def __init__(self, matrix=None, device="cpu", preconditioner="none", dtype=np.float64):
        self.args = dict(matrix=matrix, device=device, preconditioner=preconditioner, dtype=dtype)

    def __call__(self, b, x, rtol, max_iter, ext_spai=None):
        _StubPCG.calls.append(dict(self.args, b=b, x=x, rtol=rtol, max_iter=max_iter, ext_spai=ext_spai))
        return 7, 0.25, 0.5


@pytest.fixture
def stub_pymathprim(monkeypatch):
    pm = types.ModuleType("pymathprim")
    pml = types.ModuleType("pymathprim.linalg")
    pml.PreconditionedConjugateGradient = _StubPCG
    pm.linalg = pml
    monkeypatch.setitem(sys.modules, "pymathprim", pm)
    monkeypatch.setitem(sys.modules, "pymathprim.linalg", pml)
    _StubPCG.calls = []
    return _StubPCG


def _gpu_absent():
    if torch.cuda.is_available():
        pytest.skip("GPU present: the cuda leg would solve")


def test_cpu_device_reaches_pymathprim(stub_pymathprim):
    A = P.kuhn_laplacian(4)
    n = A.shape[0]
    gt = np.ones(n)
    L = A.copy()
    s = linalg.PreconditionedConjugateGradient(A, device="cpu", preconditioner="ext_spai")
    assert isinstance(s, _StubPCG) and s.args["device"] == "cpu"
    # the reference's default device is "cpu" (validate.py:61, 98, 133) and it means pymathprim
    assert validate.get_cg_iter_time(A, gt, rtol=1e-8, method="diagonal") == (7.0, 0.25, 0.5)
    assert validate.get_pcg_iter_time(A, gt, L, 3e-3, rtol=1e-8, repeat=2) == (7.0, 0.25, 0.5)
    assert validate.get_pcg_scaled_iter_time(A, gt, L, 3e-3, rtol=1e-8, device="cpu") == (7.0, 0.25, 0.5)
    c = stub_pymathprim.calls
    assert len(c) == 4
    assert [x["preconditioner"] for x in c] == ["diagonal", "ext_spai", "ext_spai", "ext_spai_scaled"]
    assert all(x["device"] == "cpu" and x["max_iter"] == n and x["rtol"] == 1e-8 for x in c)
    assert np.array_equal(c[0]["b"], A @ gt) and c[0]["ext_spai"] is None
    assert c[1]["ext_spai"][1] == 3e-3 and (c[1]["ext_spai"][0] != L).nnz == 0
    assert all(isinstance(x["b"], np.ndarray) and isinstance(x["x"], np.ndarray) for x in c)


def test_cpu_row_reaching_max_iter_raises_runtime_error(stub_pymathprim):
    A = P.kuhn_laplacian(3)
    with pytest.raises(RuntimeError, match="CG did not converge"):  # validate.py:84-85
        validate.get_cg_iter_time(A, np.ones(A.shape[0]), max_iter=5, method="none")


def test_cuda_device_reaches_mi355x_class(stub_pymathprim):
    _gpu_absent()
    A = P.kuhn_laplacian(4)
    with pytest.raises(_lib.LspcgUnavailable):
        validate.get_pcg_iter_time(A, np.ones(A.shape[0]), A, 3e-3, device="cuda")
    with pytest.raises(_lib.LspcgUnavailable):
        linalg.PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai")
    assert stub_pymathprim.calls == []


def test_cpu_without_pymathprim_raises_runtime_error(monkeypatch):
    monkeypatch.setitem(sys.modules, "pymathprim", None)  # import fails like an absent package
    A = P.kuhn_laplacian(3)
    with pytest.raises(RuntimeError) as ei:
        validate.get_pcg_iter_time(A, np.ones(A.shape[0]), A, 3e-3)
    assert isinstance(ei.value, linalg.CpuBackendUnavailable) and not isinstance(ei.value, ValueError)


def test_reference_infer_loop_shape(stub_pymathprim):
    """The row loop of infer.py:310-331 as the reference writes it, on this package's names: the
    cpu rows come back from pymathprim, the cuda rows raise inside the same try, caught by the
    reference's ``except RuntimeError`` handler only if LspcgUnavailable is a RuntimeError."""
    _gpu_absent()
    A = P.kuhn_laplacian(3)
    r = np.ones(A.shape[0])
    rows = {}
    try:
        for m in ["none", "diagonal", "ainv", "ic"]:
            for d in ["cpu", "cuda"]:
                rows[f"PCG-{m}-{d}"] = validate.get_cg_iter_time(A, r, rtol=1e-8, repeat=1, method=m, device=d)
    except RuntimeError:
        pass
    assert rows == {"PCG-none-cpu": (7.0, 0.25, 0.5)}
    assert issubclass(_lib.LspcgUnavailable, RuntimeError)


def test_reference_quirks_rows():
    """--reference-quirks: the Neural rows take the last baseline's setup time and Neural+CUDA the
    host Neural row's count (infer.py:318, 330-331); the default keeps each row's own values."""
    from learningsparsepreconditioner4gpu_amd.distributed import SolveRecord
    from learningsparsepreconditioner4gpu_amd.infer import reference_quirks

    def rec(i, it, prec):
        return SolveRecord(index=i, iters=it, rel_res=0.0, t_prec=prec, t_solve=1.0, n=10, nnz=30)

    rows = {"PCG-none-cuda": [rec(0, 50, 0.0), rec(1, 60, 0.0)],
            "PCG-ic-cuda": [rec(1, 20, 0.7), rec(0, 21, 0.9)],
            "Neural+CUDA": [rec(0, 30, 0.01), rec(1, 31, 0.02)],
            "Neural": [rec(1, 33, 0.02), rec(0, 32, 0.01)]}
    q = reference_quirks(rows, "Neural+CUDA", ["none", "ic"])
    assert [(r.index, r.iters, r.t_prec) for r in q["Neural+CUDA"]] == [(0, 32, 0.9), (1, 33, 0.7)]
    assert [(r.index, r.iters, r.t_prec) for r in q["Neural"]] == [(1, 33, 0.7), (0, 32, 0.9)]
    assert q["PCG-ic-cuda"] is rows["PCG-ic-cuda"] and rows["Neural+CUDA"][0].iters == 30


def test_random_rhs_seeded_per_sample():
    from learningsparsepreconditioner4gpu_amd.infer import rhs_for

    m = np.ones(50)
    a = rhs_for("random", m, rng=np.random.default_rng(3))
    b = rhs_for("random", m, rng=np.random.default_rng(3))
    assert np.array_equal(a, b) and not np.array_equal(a, rhs_for("random", m, rng=np.random.default_rng(4)))


def test_cpu_device_rejects_device_only_options(stub_pymathprim):
    """info / dot_order / dot_threads belong to the HIP path; with device='cpu' (the
    reference's default, pymathprim's row) they raise a clear ValueError instead of leaving info empty."""
    A = P.kuhn_laplacian(4)
    gt = np.ones(A.shape[0])
    for kw in ({"info": {}}, {"dot_order": "openblas"}, {"dot_threads": 8}):
        with pytest.raises(ValueError, match="device='cuda' only"):
            validate.get_cg_iter_time(A, gt, method="none", **kw)
        with pytest.raises(ValueError, match="device='cuda' only"):
            validate.get_pcg_iter_time(A, gt, A.copy(), 1e-3, **kw)
    assert not stub_pymathprim.calls  # nothing reached the CPU backend
    validate.get_pcg_iter_time(A, gt, A.copy(), 1e-3)  # the reference's own call still goes through
    assert len(stub_pymathprim.calls) == 1
