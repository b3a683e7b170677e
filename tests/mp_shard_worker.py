"""Worker of tests/test_gpu_multiprocess.py: one process per column shard, libbrr session on the
GPU, residual deltas + statistics summed across processes with torch.distributed (gloo) -- the
exchange ncclAllReduce performs inside libbrr between GPUs.  argv: rank world port out_dir model
[order]."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    rank, world, port, out_dir, model = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5])
    order = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import torch.distributed as dist
    import bayesrrcpp_amd as brr
    from bayesrrcpp_amd import _lib as L
    from bayesrrcpp_amd.distributed import shard_columns
    from oracle import oracle as O
    from conftest import CVA, HYP
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, P, B = 300, 640, 128
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    c0, c1 = shard_columns(P, B, rank, world)
    K = 1 if model == L.MODEL_HORSESHOE else len(CVA) + 1
    s = brr.Session(model, N, c1 - c0, K=K, M_total=P, col_offset=c0, block_size=B, shard_rank=rank,
                    shard_count=world, order_mode=order)
    s.upload_x(X[:, c0:c1])
    s.set_y(Y)
    if model == L.MODEL_HORSESHOE:
        s.set_horseshoe(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    else:
        s.set_bayesr(**HYP, cva=CVA)
    s.init(9)
    s.exchange_buffers()
    # the library's default exchanges per sweep (automatic), driven by the host
    # protocol driver (local segment, gloo all-reduce of deltas + statistics + failure flag, finish)
    from bayesrrcpp_amd.distributed import HostExchange
    HostExchange(dist).sweep(s, 4)
    assert s.iteration == 4
    np.save(os.path.join(out_dir, f"E{rank}.npy"), np.array([s.exchanges_per_sweep]))
    np.save(os.path.join(out_dir, f"beta{rank}.npy"), s.vector(L.BETA))
    np.save(os.path.join(out_dir, f"eps{rank}.npy"), s.vector(L.EPS))
    comp = s.vector(L.COMP) if model != L.MODEL_HORSESHOE else np.zeros(c1 - c0)
    np.save(os.path.join(out_dir, f"comp{rank}.npy"), comp)
    np.save(os.path.join(out_dir, f"sc{rank}.npy"), np.array([s.scalar(L.MU), s.scalar(L.SIGMAE)]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
