"""Kernel-level view of the batched lockstep solve (run under rocprofv3 --kernel-trace --stats):
the C5 heat batch and 8 x Poisson 256^2 as one BatchedConjugateGradient each, 5 solves at rtol
1e-8 after a warm-up; prints the host wall time per solve."""
import json
import sys
import time

import torch


def main():
    sys.path.insert(0, ".")
    from learningsparsepreconditioner4gpu_amd import problems as P
    from learningsparsepreconditioner4gpu_amd.data import make_sample
    from learningsparsepreconditioner4gpu_amd.infer import synthetic_dataset
    from learningsparsepreconditioner4gpu_amd.linalg import BatchedConjugateGradient
    from learningsparsepreconditioner4gpu_amd.workspace import SimpleInferenceWorkspace

    sets = {"heat_batch8": synthetic_dataset("heat_batch8")}
    A_raw, mask, feats, bs, e2n = P.workload("poisson256")
    sets["poisson256x8"] = [make_sample(A_raw, mask, node_features=feats, block_size=bs,
                                        use_edge_features_as_node_feature=e2n)] * 8
    which = sys.argv[1:] or list(sets)
    for name in which:
        samples = sets[name]
        ws = SimpleInferenceWorkspace(node_features=samples[0].x.shape[1], edge_features=samples[0].edge_attr.shape[1],
                                      seed=0)
        As, Ls, bs_ = [], [], []
        for s in samples:
            d = s.to("cuda")
            L, _ = ws.inference_step(d)
            A = ws.system_matrix(d)
            As.append(A)
            Ls.append(L)
            bs_.append(A.matvec(d.mask.reshape(-1).to(torch.float64)))
        B = BatchedConjugateGradient(As, Ls, ws.epsilon)
        xs = [torch.zeros_like(b) for b in bs_]
        B.solve(bs_, xs, rtol=1e-8)
        walls = []
        for _ in range(5):
            for x in xs:
                x.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res, dev = B.solve(bs_, xs, rtol=1e-8)
            walls.append(time.perf_counter() - t0)
        its = [r[0] for r in res]
        print(json.dumps({"set": name, "rows": sum(B.n), "max_iters": max(its), "wall_ms": min(walls) * 1e3,
                          "us_per_lockstep_iter": min(walls) * 1e6 / max(its)}), flush=True)


if __name__ == "__main__":
    main()
