import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    from learningsparsepreconditioner4gpu_amd.sparse import Context

    return Context.get(0)


def pytest_collection_modifyitems(config, items):
    # make sure CPU-only runs never touch the GPU tests by accident
    markexpr = config.getoption("-m") or ""
    if "not gpu" in markexpr:
        return
