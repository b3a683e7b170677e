"""GPU parity of the column-sharded protocol with E residual exchanges per sweep
(brr_options.exchanges_per_sweep): two shard sessions on one GPU, each sweep
split into E local / host-summed exchange / finish rounds (the role ncclAllReduce plays across
GPUs), against the oracle's 2-shard emulation with the same E (oracle/brr_oracle.c
marker_segment).  Segments are whole blocks, one-block segments included; the fused persistent
sweep (lag 1 and 2) and the per-block kernels; V2, Groups with a fixed effect, and the Horseshoe.

Tolerance as tests/test_gpu_parity.py: identical component assignments, beta / epsilon / sigmaE /
pi within relative 1e-9 after every sweep.
"""
import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu

RTOL = 1e-9


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.maximum(np.abs(b), np.max(np.abs(b)) * 1e-3 + 1e-300)
    return float(np.max(np.abs(a - b) / scale)) if a.size else 0.0


@pytest.mark.parametrize("model,E,per_block,lag", [
    (0, 2, False, None), (0, 4, False, None), (0, 3, False, "1"), (0, 4, True, None),
    (1, 3, False, None), (3, 3, False, None), (3, 2, True, None),
    # lag 2 with segments of one block (E = 6) and of one or two blocks (E = 4): the cross-Gram
    # corrections and the streamers' list prefetch must stop at the segment start
    (0, 6, False, "2"), (0, 4, False, "2"),
])
def test_exchange_segments_match_oracle(brr, oracle_mod, require_gpu, monkeypatch, model, E, per_block, lag):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    if per_block:
        monkeypatch.setenv("BRR_PER_BLOCK", "1")
    if lag:
        monkeypatch.setenv("BRR_LAG", lag)
    N, P, B = 300, 1536, 128  # two shards of 6 blocks
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=40)
    G = 2 if model == L.MODEL_GROUPS else 1
    F = 1 if model == L.MODEL_GROUPS else 0
    fixed = np.linspace(-1.0, 1.0, N).reshape(N, 1) if F else None
    gA = (np.arange(P) * G // P).astype(np.int32) if G > 1 else None
    cva = np.tile(CVA, (G, 1))
    hs = dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    sess = []
    for r, c0 in enumerate((0, 768)):
        s = brr.Session(model, N, 768, K=1 if model == L.MODEL_HORSESHOE else 4, groups=G, F=F, M_total=P,
                        col_offset=c0, block_size=B, shard_rank=r, shard_count=2, exchanges_per_sweep=E)
        assert s.exchanges_per_sweep == E
        if lag == "2":
            assert s.scalar(106) == 2  # the fused sweep's pipeline lag
        s.upload_x(X[:, c0:c0 + 768])
        s.set_y(Y)
        if model == L.MODEL_HORSESHOE:
            s.set_horseshoe(**hs)
        else:
            s.set_bayesr(**HYP, cva=cva, gAssign=gA[c0:c0 + 768] if G > 1 else None)
        if F:
            s.set_fixed(fixed)
        s.init(9)
        s.exchange_buffers()
        sess.append(s)
    if model == L.MODEL_HORSESHOE:
        orc = O.Oracle(O.HORSESHOE, X, Y, seed=9, order_mode=0, block_size=B, n_shards=2, n_exchanges=E, **hs)
    else:
        orc = O.Oracle({0: O.V2, 1: O.GROUPS}[model], X, Y, cva=cva, G=G, gAssign=gA, fixed=fixed, seed=9,
                       order_mode=0, block_size=B, n_shards=2, n_exchanges=E, **HYP)
    for it in range(3):
        for _ in range(E):
            for s in sess:
                s.sweep_local()
            parts = [s.exchange_get() for s in sess]
            te, ts = parts[0][0] + parts[1][0], parts[0][1] + parts[1][1]
            for s in sess:
                s.exchange_set(te, ts)
                s.sweep_finish()
        assert all(s.iteration == it + 1 for s in sess)
        orc.sweep(1)
        beta = np.concatenate([s.vector(L.BETA) for s in sess])
        if model != L.MODEL_HORSESHOE:
            comp = np.concatenate([s.vector(L.COMP) for s in sess])
            assert np.array_equal(comp, orc.vector(O.V_COMP)), f"it={it}"
            for s in sess:
                assert _rel(s.vector(L.PI), orc.vector(O.V_PI)) < RTOL
        assert _rel(beta, orc.vector(O.V_BETA)) < RTOL, f"it={it} {_rel(beta, orc.vector(O.V_BETA))}"
        for s in sess:
            assert _rel(s.vector(L.EPS), orc.vector(O.V_EPS)) < RTOL
            assert _rel([s.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < RTOL
    for s in sess:
        s.close()


def test_exchange_segments_one_equals_default(brr, oracle_mod, require_gpu):
    """E = 1 is the one-exchange protocol; E > 1 on an unsharded session is ignored (one round)."""
    from bayesrrcpp_amd import _lib as L
    s = brr.Session(L.MODEL_V2, 300, 512, K=4, block_size=128, exchanges_per_sweep=4)
    assert s.exchanges_per_sweep == 1
    s.close()
