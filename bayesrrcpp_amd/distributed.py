"""Column-sharded multi-GPU driver helpers: one process per GPU, markers split
into contiguous ranges of whole blocks, the residual kept coherent by ONE all-reduce of the
residual deltas (and the marker statistics) per exchange segment: brr_options.exchanges_per_sweep =
E rounds per sweep (default: E = 8, at most the blocks per shard; 1 = one exchange per sweep).

Two exchange paths share the same session protocol (brr_session_sweep_local -> sum ->
brr_session_sweep_finish):
  * native: libbrr's own RCCL communicator (ncclAllReduce on the session stream, xGMI);
    `init_native_comm` only moves the 128-byte unique id through torch.distributed (gloo);
  * host:   `HostExchange` sums the exchange buffers with torch.distributed on CPU tensors
    (gloo) -- for debugging / CPU tests; any object with sweep_local / exchange_get /
    exchange_set / sweep_finish works (the oracle's per-shard mode implements the same).
torch's own HIP runtime is never initialised here (libbrr uses the system ROCm runtime).
"""
from __future__ import annotations


def shard_columns(P: int, B: int, rank: int, world: int) -> tuple[int, int]:
    """[c0, c1) of this rank: contiguous whole blocks of B markers, balanced by block count."""
    nb = (P + B - 1) // B
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    return b0 * B, min(P, b1 * B)


def init_native_comm(session, dist=None, rank: int = 0, world: int = 1):
    """Create libbrr's RCCL communicator: rank 0 makes the id, gloo broadcasts it."""
    from .session import comm_unique_id
    if world == 1:
        uid = [comm_unique_id()]
    else:
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
    session.comm_init(uid[0], world, rank)


class HostExchange:
    """Sweeps driven on the host: local sweep, gloo all-reduce of (deps, stats), finish.

    A local sweep that fails on one rank (a device pipeline timeout or a failed residency census,
    brr_session_sweep_local -> -3) must not leave its peers blocked in the collective: the failing
    rank still takes part in the round's all-reduce, with a failure flag appended to the
    statistics, and every rank finishes the round and then raises together."""

    def __init__(self, dist):
        self.dist = dist

    def sweep(self, shard, n: int = 1):
        """n sweeps; a sweep is `shard.exchanges_per_sweep` local / all-reduce / finish rounds."""
        import numpy as np
        import torch
        rounds = getattr(shard, "exchanges_per_sweep", 1)
        for _ in range(n * rounds):
            err = None
            try:
                shard.sweep_local()
            except Exception as ex:  # noqa: BLE001 -- re-raised on every rank below
                err = ex
            e, s = shard.exchange_get()
            te = torch.from_numpy(e)
            ts = torch.from_numpy(np.concatenate([s, [1.0 if err is not None else 0.0]]))
            self.dist.all_reduce(te)
            self.dist.all_reduce(ts)
            failed = int(ts[-1].item())
            shard.exchange_set(te.numpy(), ts[:-1].numpy())
            shard.sweep_finish()
            if failed:
                if err is not None:
                    raise err
                raise RuntimeError(f"column-shard sweep failed on {failed} other rank(s)")
