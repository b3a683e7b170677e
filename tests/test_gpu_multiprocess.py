"""Column shards in separate PROCESSES on the GPU (the driver's multi-GPU layout, on the one GPU
this pool gives a test): two worker processes (tests/mp_shard_worker.py, started as child
processes), each with its own libbrr session for its column shard, sum the residual deltas and
statistics with torch.distributed gloo after every sweep (libbrr does the same sum with
ncclAllReduce between GPUs).  The result equals the oracle's 2-shard emulation (identical
components, 1e-9) and every rank holds bit-identical replicated state."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,order", [(0, 0), (3, 0), (0, 1)])  # BLOCKED; REFERENCE
def test_two_processes_column_shards(oracle_mod, require_gpu, tmp_path, model, order):
    O = oracle_mod
    world, port = 2, str(_free_port())
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mp_shard_worker.py"), str(r), str(world), port,
                               str(tmp_path), str(model), str(order)]) for r in range(world)]
    try:
        rcs = [p.wait(timeout=180) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    N, P, B = 300, 640, 128
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    kw = dict(cva=CVA, **HYP) if model == O.V2 else dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0,
                                                        c2=1.0, vC=10.0, sC=10.0)
    E = int(np.load(tmp_path / "E0.npy")[0])
    assert E == 2 and int(np.load(tmp_path / "E1.npy")[0]) == E  # automatic: 8 capped at 5 blocks / 2 shards, same on every rank
    ref = O.Oracle(model, X, Y, seed=9, order_mode=order, block_size=B, n_shards=world, n_exchanges=E, **kw)
    ref.sweep(4)
    beta = np.concatenate([np.load(tmp_path / f"beta{r}.npy") for r in range(world)])
    scale = np.maximum(np.abs(ref.vector(O.V_BETA)), 1e-3 * np.abs(ref.vector(O.V_BETA)).max())
    assert np.max(np.abs(beta - ref.vector(O.V_BETA)) / scale) < 1e-9
    if model == O.V2:
        comp = np.concatenate([np.load(tmp_path / f"comp{r}.npy") for r in range(world)])
        assert np.array_equal(comp, ref.vector(O.V_COMP))
    e0 = np.load(tmp_path / "eps0.npy")
    for r in range(world):  # replicated state: bit-identical on every rank
        assert np.array_equal(np.load(tmp_path / f"eps{r}.npy"), e0)
        assert np.array_equal(np.load(tmp_path / f"sc{r}.npy"), np.load(tmp_path / "sc0.npy"))
    eo = ref.vector(O.V_EPS)
    assert np.max(np.abs(e0 - eo)) / np.max(np.abs(eo)) < 1e-9
    sc = np.load(tmp_path / "sc0.npy")
    assert abs(sc[1] - ref.scalar(O.S_SIGMAE)) / ref.scalar(O.S_SIGMAE) < 1e-9
