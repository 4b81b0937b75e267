"""Debug: world-2 DistributedPCG on one GPU (gloo): full solve, first divergence from the oracle,
with and without a device synchronize after each host-staged exchange."""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp


def rank_main(rank, world, port, sync):
    sys.path.insert(0, ".")
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from learningsparsepreconditioner4gpu_amd import dist_pcg as D
    from oracle import linalg as O
    from tests.test_gpu_dist_pcg import EPS, _system

    if sync:
        orig = D.exchange

        def ex(*a, **k):
            torch.cuda.synchronize()
            orig(*a, **k)
            torch.cuda.synchronize()
        D.exchange = ex
    A, L, b = _system("kuhn")
    d = D.DistributedPCG(A, L, EPS)
    it, conv, x, hist = d.solve(b, rtol=1e-8, return_history=True)
    it_o, x_o, h_o = O.pcg(A, b, O.spai_operator(L, EPS), rtol=1e-8, dot="exact")
    m = min(len(hist), len(h_o))
    bad = np.nonzero(np.abs(hist[:m] - h_o[:m]) > 1e-12 * np.abs(h_o[:m]))[0]
    print(f"sync={sync} rank {rank}: it {it} oracle {it_o} first bad {bad[:5]} "
          f"{hist[bad[0]] if len(bad) else ''} vs {h_o[bad[0]] if len(bad) else ''}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    for sync, port in ((0, 29611), (1, 29612)):
        ps = [ctx.Process(target=rank_main, args=(r, 2, port, sync)) for r in range(2)]
        [x.start() for x in ps]
        [x.join(120) for x in ps]
        print("exit", [x.exitcode for x in ps], flush=True)
