"""First solve of a fresh solver (the reference's per-sample methodology: validate.py:110 builds a
new PreconditionedConjugateGradient per solve) vs repeated solves on the same solver, over the
heat_batch8 systems and a Kuhn grid: shows the per-solver fixed costs inside the solve time."""
import json
import sys
import time

import numpy as np
import torch


def main():
    sys.path.insert(0, ".")
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.linalg import PreconditionedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    samples = synthetic_dataset("heat_batch8")
    A_raw, mask, feats, bs, e2n = P.workload("kuhn41")
    samples.append(make_sample(A_raw, mask, node_features=feats, block_size=bs, use_edge_features_as_node_feature=e2n))
    out = []
    for s in samples:
        ws = SimpleInferenceWorkspace(node_features=s.x.shape[1], edge_features=s.edge_attr.shape[1], seed=0)
        d = s.to("cuda")
        L, _ = ws.inference_step(d)
        A = ws.system_matrix(d)
        b = A.matvec(d.mask.reshape(-1).to(torch.float64))
        rec = {"n": A.n, "nnz": A.nnz}
        for trial in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            solver = PreconditionedConjugateGradient(A, device="cuda", preconditioner="ext_spai", dtype=np.float64)
            prec = solver.set_spai(L, ws.epsilon)
            x = torch.zeros_like(b)
            it, conv, s1 = solver.solve(b, x, rtol=1e-6)
            x.zero_()
            it2, conv2, s2 = solver.solve(b, x, rtol=1e-6)
            torch.cuda.synchronize()
            rec[f"t{trial}"] = {"iters": it, "first_solve_ms": s1 * 1e3, "second_solve_ms": s2 * 1e3,
                                "set_spai_ms": prec * 1e3, "wall_ms": (time.perf_counter() - t0) * 1e3}
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
