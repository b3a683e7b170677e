"""Multi-process (gloo, world_size 2) test of the column-sharded exchange protocol on CPU:
two processes, each sweeping its own shard and summing the residual deltas + statistics with
torch.distributed, reproduce the single-process 2-shard emulation bit for bit -- also with E
residual exchanges per sweep (brr_options.exchanges_per_sweep).  The GPU path
runs the same protocol with ncclAllReduce inside libbrr (tests/test_gpu_parity.py covers the
device side on one GPU)."""
import os
import socket

import numpy as np
import pytest

from conftest import CVA, HYP


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, model, out_dir, order=0, E=1):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from oracle import oracle as O
    from bayesrrcpp_amd.distributed import HostExchange
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, Y, _ = O.synth_cohort(11, 240, 384, n_causal=20)
    kw = dict(cva=CVA, **HYP) if model == O.V2 else dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1, vT=1,
                                                        c2=1, vC=10, sC=10)
    o = O.Oracle(model, X, Y, seed=3, block_size=64, n_shards=world, shard_only=rank, order_mode=order,
                 n_exchanges=E, **kw)
    HostExchange(dist).sweep(o, 3)
    np.save(os.path.join(out_dir, f"beta{rank}.npy"), o.vector(O.V_BETA))
    np.save(os.path.join(out_dir, f"eps{rank}.npy"), o.vector(O.V_EPS))
    np.save(os.path.join(out_dir, f"sc{rank}.npy"), np.array([o.scalar(O.S_MU), o.scalar(O.S_SIGMAE),
                                                             o.scalar(O.S_SIGMAG), o.scalar(O.S_TAU)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("model,order,E", [(0, 0, 1), (3, 0, 1), (0, 1, 1), (3, 1, 1),  # BLOCKED, REFERENCE
                                           (0, 0, 2), (3, 0, 3), (0, 1, 3)])  # E exchanges per sweep
def test_gloo_two_ranks_match_emulation(oracle_mod, tmp_path, model, order, E):
    import torch.multiprocessing as mp
    O = oracle_mod
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), model, str(tmp_path), order, E), nprocs=world, join=True)
    X, Y, _ = O.synth_cohort(11, 240, 384, n_causal=20)
    kw = dict(cva=CVA, **HYP) if model == O.V2 else dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1, vT=1,
                                                        c2=1, vC=10, sC=10)
    ref = O.Oracle(model, X, Y, seed=3, block_size=64, n_shards=world, order_mode=order, n_exchanges=E, **kw)
    ref.sweep(3)
    from bayesrrcpp_amd.distributed import shard_columns
    beta = np.zeros(384)
    for r in range(world):
        c0, c1 = shard_columns(384, 64, r, world)
        beta[c0:c1] = np.load(tmp_path / f"beta{r}.npy")[c0:c1]
        # replicated state identical on every rank and equal to the emulation, bit for bit
        assert np.array_equal(np.load(tmp_path / f"eps{r}.npy"), ref.vector(O.V_EPS))
        sc = np.load(tmp_path / f"sc{r}.npy")
        assert np.array_equal(sc, [ref.scalar(O.S_MU), ref.scalar(O.S_SIGMAE), ref.scalar(O.S_SIGMAG),
                                   ref.scalar(O.S_TAU)])
    assert np.array_equal(beta, ref.vector(O.V_BETA))


def test_shard_columns_partition():
    from bayesrrcpp_amd.distributed import shard_columns
    for P, B, W in [(500_000, 128, 8), (1000, 64, 3), (130, 128, 2)]:
        cover = []
        for r in range(W):
            c0, c1 = shard_columns(P, B, r, W)
            assert c0 % B == 0
            cover += list(range(c0, c1))
        assert cover == list(range(P))


class _FlakyShard:
    """Minimal protocol object (the session / oracle interface HostExchange drives) whose local
    sweep fails on one rank in one round."""

    exchanges_per_sweep = 2

    def __init__(self, rank, fail_round):
        self.rank, self.fail_round, self.round, self.finished = rank, fail_round, 0, 0

    def sweep_local(self):
        self.round += 1
        if self.round == self.fail_round:
            raise RuntimeError(f"sweep_local failed (rc=-3) on rank {self.rank}")

    def exchange_get(self):
        return np.full(4, float(self.rank + 1)), np.zeros(3)

    def exchange_set(self, e, s):
        assert np.array_equal(e, np.full(4, 3.0)) and s.shape == (3,)

    def sweep_finish(self):
        self.finished += 1


def _flaky_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from bayesrrcpp_amd.distributed import HostExchange
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = _FlakyShard(rank, fail_round=3 if rank == 1 else -1)
    msg = ""
    try:
        HostExchange(dist).sweep(sh, 4)
    except RuntimeError as ex:
        msg = str(ex)
    np.save(os.path.join(out_dir, f"flaky{rank}.npy"), np.array([sh.round, sh.finished]))
    with open(os.path.join(out_dir, f"flaky{rank}.txt"), "w") as f:
        f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


def test_host_exchange_failure_stops_every_rank(tmp_path):
    """A local sweep that fails on one rank (brr_session_sweep_local -> -3) still takes part in its
    round's all-reduce (failure flag appended to the statistics): every rank finishes that round and
    raises together instead of leaving its peers blocked in the collective."""
    import torch.multiprocessing as mp
    mp.spawn(_flaky_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"flaky{r}.npy"), [3, 3])  # round 3 exchanged + finished, none after
    assert "rank 1" in (tmp_path / "flaky1.txt").read_text()
    assert "other rank" in (tmp_path / "flaky0.txt").read_text()
