"""AINV(0) setup on one workload (argv[1], default kuhn41), twice: for rocprofv3 kernel traces."""
import json
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, ".")
from learningsparsepreconditioner4gpu_amd import problems as P  # noqa: E402
from learningsparsepreconditioner4gpu_amd.sparse import DeviceMatrix  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "kuhn41"
A, mask, *_ = P.workload(name)
Ad = DeviceMatrix.from_scipy(sp.csr_matrix(A))
for _ in range(2):
    L, t = Ad.ainv0()
    print(json.dumps({"w": name, "ainv_setup_ms": t * 1e3}), flush=True)
