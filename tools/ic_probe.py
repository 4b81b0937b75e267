"""PCG-IC on one workload (argv[1], default kuhn101), two solves: for rocprofv3 kernel traces of the
triangular solves (sync-free vs LSPCG_TRSV_LEVELS=1)."""
import json
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, ".")
from learningsparsepreconditioner4gpu_amd import problems as P  # noqa: E402
from learningsparsepreconditioner4gpu_amd.validate import get_cg_iter_time  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "kuhn101"
A, mask, *_ = P.workload(name)
A = sp.csr_matrix(A)
for _ in range(2):
    it, prec, solve = get_cg_iter_time(A, np.ones(A.shape[0]), rtol=1e-8, method="ic")
    print(json.dumps({"w": name, "iters": it, "prec_ms": prec * 1e3, "solve_ms": solve * 1e3,
                      "us_per_iter": solve * 1e6 / max(it, 1)}), flush=True)
