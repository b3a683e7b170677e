"""Column-sharded multi-GPU driver helpers: one process per GPU, markers split
into contiguous ranges of whole blocks, the residual kept coherent by ONE all-reduce of the
residual deltas (and the marker statistics) per sweep -- or per exchange segment, with
brr_options.exchanges_per_sweep = E > 1 (E rounds per sweep).

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
    """Sweeps driven on the host: local sweep, gloo all-reduce of (deps, stats), finish."""

    def __init__(self, dist):
        self.dist = dist

    def sweep(self, shard, n: int = 1):
        """n sweeps; a sweep is `shard.exchanges_per_sweep` local / all-reduce / finish rounds."""
        import torch
        rounds = getattr(shard, "exchanges_per_sweep", 1)
        for _ in range(n * rounds):
            shard.sweep_local()
            e, s = shard.exchange_get()
            te, ts = torch.from_numpy(e), torch.from_numpy(s)
            self.dist.all_reduce(te)
            self.dist.all_reduce(ts)
            shard.exchange_set(te.numpy(), ts.numpy())
            shard.sweep_finish()
