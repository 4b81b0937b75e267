"""bench.py's JSON contract on a small system (GPU box): one line with the metric, value,
roofline (achieved / peak / frac / traffic) and cpu_baseline objects, rank-0 only."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def test_bench_json_line():
    env = dict(os.environ)
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--workload", "kuhn31", "--steps", "2", "--warmup",
                          "1", "--spmv-reps", "3", "--cpu-iters", "10"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=240, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["higher_is_better"] is True and d["dtype"] == "f64"
    assert d["value"] > 0 and d["config"]["iters_per_solve"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["value"] > 0 and c["nproc"] >= 1 and c["cores"] in (1, c["nproc"])
    assert set(c["by_threads"]) == {"1"} and c["cores"] == 1 and "cpu_model" in c
    v = d["time_to_rtol_variants"]
    assert set(v) == {"ext_spai", "none", "diagonal"} and all(set(r) == {"mask", "random"} for r in v.values())
    c1 = d["c1_synthetic"]
    assert c1["gpu"]["compensated"]["iters"] > 0 and c1["cpu"]["1"]["it_per_s"] > 0
    assert c1["gpu"]["openblas"]["iters"] == 3236  # the reference's count at 1 OpenBLAS thread
    assert d["gnn_tflops"] > 0 and d["pcg_loop_kernels"]["frac_format"] > 0
