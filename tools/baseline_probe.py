import sys, json, time
sys.path.insert(0, ".")
import numpy as np
from learningsparsepreconditioner4gpu_amd import problems as P
from learningsparsepreconditioner4gpu_amd.validate import get_cg_iter_time
for name in ["kuhn41", "kuhn101"]:
    A, mask, *_ = P.workload(name)
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    gt = np.ones(A.shape[0])
    for m in ["none", "diagonal", "ic", "ainv"]:
        it, prec, solve = get_cg_iter_time(A, gt, rtol=1e-8, method=m, device="cuda")
        print(json.dumps({"w": name, "method": m, "iters": it, "prec_ms": prec * 1e3, "solve_ms": solve * 1e3,
                          "us_per_iter": solve * 1e6 / max(it, 1)}), flush=True)
