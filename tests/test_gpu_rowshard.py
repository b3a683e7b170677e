"""GPU parity of the exact row-sharded sampler against the single-shard oracle.

Each row shard holds rows [row_offset, row_offset + N_r) of the cohort and every marker; per
marker block the partial dots are summed across the shards before the replicated block solve
(src/BayesRv2.cpp:186-245 run exactly, not the column shards' stale-residual approximation).
Here the shards are sessions of one in-process brr_group on one GPU, whose cross-shard sums run
on the device in rank order; the multi-process RCCL path shares every step but the sum itself.

Tolerance as tests/test_gpu_parity.py: component assignments identical to the unsharded
oracle chain; beta, epsilon (shards concatenated), mu and the hyper-parameters within relative
1e-9; and every shard holds bit-identical replicated state (beta, comps, sigmas).
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


def _build(brr, O, model, X, Y, cuts, order, B=128, G=1, gAssign=None, fixed=None, cva=CVA,
           seed=7, restart=None, hs=None, x_storage=0):
    from bayesrrcpp_amd import _lib as L
    N, P = X.shape
    R = len(cuts) - 1
    K = 1 if model == L.MODEL_HORSESHOE else np.atleast_2d(cva).shape[-1] + 1
    F = 0 if fixed is None else np.asarray(fixed).reshape(N, -1).shape[1]
    cva2 = None
    if model != L.MODEL_HORSESHOE:
        cva2 = np.tile(np.asarray(cva, float), (G, 1)) if np.ndim(cva) == 1 else np.asarray(cva)
    members = []
    for r in range(R):
        a, b = cuts[r], cuts[r + 1]
        s = brr.Session(model, b - a, P, K=K, groups=G, F=F, block_size=B, order_mode=order,
                        row_shard_rank=r, row_shard_count=R, row_offset=a, N_total=N, x_storage=x_storage)
        s.upload_x(X[a:b])
        if model != L.MODEL_RESTART:
            s.set_y(Y[a:b])
        if model == L.MODEL_HORSESHOE:
            s.set_horseshoe(**hs)
        else:
            s.set_bayesr(HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], cva2, gAssign)
        if fixed is not None:
            s.set_fixed(np.asarray(fixed).reshape(N, -1)[a:b])
        if restart is not None:
            s.set_restart(restart["mu0"], restart["beta0"], restart["sigmaE0"], restart["sigmaGG0"],
                          restart["eps0"][a:b], restart["comp0"])
        members.append(s)
    g = brr.Group(members).init(seed)
    okw = {}
    if model == L.MODEL_HORSESHOE:
        okw.update(hs)
    else:
        okw.update(HYP)
        okw.update(cva=cva2, G=G)
        if gAssign is not None:
            okw["gAssign"] = gAssign
    if fixed is not None:
        okw["fixed"] = fixed
    if restart is not None:
        okw.update(restart)
    orc = O.Oracle(model, X, None if model == L.MODEL_RESTART else Y, seed=seed, order_mode=order,
                   block_size=B, N=N, **okw)
    return g, members, orc


def _compare(members, orc, O, L, model, tag):
    s0 = members[0]
    eps = np.concatenate([m.vector(L.EPS) for m in members])
    assert _rel(eps, orc.vector(O.V_EPS)) < RTOL, f"{tag} eps rel err {_rel(eps, orc.vector(O.V_EPS))}"
    bo = orc.vector(O.V_BETA)
    for m in members:  # replicated state: identical bits on every shard
        assert np.array_equal(m.vector(L.BETA), s0.vector(L.BETA)), tag
        assert m.scalar(L.SIGMAE) == s0.scalar(L.SIGMAE) and m.scalar(L.MU) == s0.scalar(L.MU), tag
    assert _rel(s0.vector(L.BETA), bo) < RTOL, f"{tag} beta rel err {_rel(s0.vector(L.BETA), bo)}"
    assert abs(s0.scalar(L.MU) - orc.scalar(O.S_MU)) <= RTOL * (1 + abs(orc.scalar(O.S_MU))), tag
    assert _rel([s0.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < RTOL, tag
    if model == L.MODEL_HORSESHOE:
        for a, b in ((L.TAU, O.S_TAU), (L.ETA, O.S_ETA), (L.C2, O.S_C2)):
            assert _rel([s0.scalar(a)], [orc.scalar(b)]) < RTOL, f"{tag} scalar {a}"
        assert _rel(s0.vector(L.LAMBDA), orc.vector(O.V_LAMBDA)) < RTOL, tag
    else:
        cg, co = s0.vector(L.COMP), orc.vector(O.V_COMP)
        assert np.array_equal(cg, co), f"{tag} comps differ at {np.nonzero(cg != co)[0][:10]}"
        for m in members:
            assert np.array_equal(m.vector(L.COMP), cg), tag
        assert _rel(s0.vector(L.SIGMAGG), orc.vector(O.V_SIGMAGG)) < RTOL, tag
        assert _rel(s0.vector(L.PI), orc.vector(O.V_PI)) < RTOL, tag
        assert np.array_equal(s0.vector(L.VCOUNT), orc.vector(O.V_VCOUNT)), tag


@pytest.mark.parametrize("order", [0, 1, 2])  # BLOCKED, REFERENCE, IDENTITY
@pytest.mark.parametrize("R", [2, 3])
def test_rowshard_v2_matches_unsharded_oracle(brr, oracle_mod, require_gpu, order, R):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 1100, 700
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=40)
    cuts = [0, 300, N] if R == 2 else [0, 257, 700, N]  # ragged shards, one not a multiple of 4
    g, ms, orc = _build(brr, O, L.MODEL_V2, X, Y, cuts, order)
    for it in range(4):
        g.sweep(1)
        orc.sweep(1)
        _compare(ms, orc, O, L, L.MODEL_V2, f"v2 R={R} order={order} it={it}")
    g.close()


def test_rowshard_groups_fixed_effects(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, G = 600, 500, 4
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    gA = (np.arange(P) * G // P).astype(np.int32)
    fixed = np.random.default_rng(3).normal(size=(N, 2))
    cva = np.array([[1e-4, 1e-3, 1e-2]] * G) * (1 + np.arange(G))[:, None]
    for order in (0, 1):
        g, ms, orc = _build(brr, O, L.MODEL_GROUPS, X, Y, [0, 250, N], order, G=G, gAssign=gA,
                            fixed=fixed, cva=cva)
        for it in range(4):
            g.sweep(1)
            orc.sweep(1)
            tag = f"groups order={order} it={it}"
            _compare(ms, orc, O, L, L.MODEL_GROUPS, tag)
            assert _rel(ms[0].vector(L.ALPHA), orc.vector(O.V_ALPHA)) < RTOL, tag
            assert _rel([ms[0].scalar(L.SIGMAF)], [orc.scalar(O.S_SIGMAF)]) < RTOL, tag
        g.close()


def test_rowshard_horseshoe(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 500, 450
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    A = (1 / np.sqrt(N)) * 150 / (P - 150)
    hs = dict(A=A, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    g, ms, orc = _build(brr, O, L.MODEL_HORSESHOE, X, Y, [0, 200, N], 0, hs=hs)
    for it in range(4):
        g.sweep(1)
        orc.sweep(1)
        _compare(ms, orc, O, L, L.MODEL_HORSESHOE, f"hs it={it}")
    g.close()


def test_rowshard_restart(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, G = 420, 300, 3
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=20)
    gA = (np.arange(P) % G).astype(np.int32)
    prev = O.Oracle(O.GROUPS, X, Y, cva=np.tile(CVA, (G, 1)), G=G, gAssign=gA, seed=3,
                    order_mode=0, block_size=128, **HYP)
    prev.sweep(4)
    st = dict(mu0=prev.scalar(O.S_MU), beta0=prev.vector(O.V_BETA), sigmaE0=prev.scalar(O.S_SIGMAE),
              sigmaGG0=prev.vector(O.V_SIGMAGG), eps0=prev.vector(O.V_EPS), comp0=prev.vector(O.V_COMP))
    g, ms, orc = _build(brr, O, L.MODEL_RESTART, X, None, [0, 211, N], 0, G=G, gAssign=gA, restart=st)
    assert _rel(ms[0].vector(L.PI), orc.vector(O.V_PI)) < RTOL
    for it in range(4):
        g.sweep(1)
        orc.sweep(1)
        _compare(ms, orc, O, L, L.MODEL_RESTART, f"restart it={it}")
    g.close()


def test_rowshard_2bit_storage_identical(brr, oracle_mod, require_gpu):
    """2-bit genotype storage in row shards: the same chain bit for bit as f32 row shards."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 900, 640
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    ga, ma, _ = _build(brr, O, L.MODEL_V2, X, Y, [0, 333, N], 0)
    gb, mb, _ = _build(brr, O, L.MODEL_V2, X, Y, [0, 333, N], 0, x_storage=L.X_2BIT)
    ga.sweep(3)
    gb.sweep(3)
    for a, b in zip(ma, mb):
        assert np.array_equal(a.vector(L.BETA), b.vector(L.BETA))
        assert np.array_equal(a.vector(L.EPS), b.vector(L.EPS))
    ga.close()
    gb.close()


def test_rowshard_synthetic_cohort_matches_unsharded(brr, oracle_mod, require_gpu):
    """On-device synthetic genotypes of row shards (statistics over the whole cohort, each shard
    storing its rows) give the unsharded cohort: same column norms, same Y, same chain."""
    from bayesrrcpp_amd import _lib as L
    N, P, R = 1000, 512, 2
    cuts = [0, 420, N]
    one = brr.Session(L.MODEL_V2, N, P, K=4, block_size=128)
    one.synthesize(20261015, 0.5, 40)
    one.set_bayesr(HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], np.asarray(CVA)[None, :])
    one.init(5)
    ms = []
    for r in range(R):
        s = brr.Session(L.MODEL_V2, cuts[r + 1] - cuts[r], P, K=4, block_size=128, row_shard_rank=r,
                        row_shard_count=R, row_offset=cuts[r], N_total=N)
        s.synthesize(20261015, 0.5, 40)
        ms.append(s)
    gsum = np.concatenate([m.synth_partial_y() for m in ms])
    for m in ms:
        m.synth_y(gsum, 20261015, 0.5)
        m.set_bayesr(HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], np.asarray(CVA)[None, :])
    g = brr.Group(ms).init(5)
    assert _rel(ms[0].vector(L.XSQ), one.vector(L.XSQ)) < 1e-12
    one.sweep(3)
    g.sweep(3)
    assert np.array_equal(ms[0].vector(L.COMP), one.vector(L.COMP))
    assert _rel(ms[0].vector(L.BETA), one.vector(L.BETA)) < RTOL
    assert _rel(np.concatenate([m.vector(L.EPS) for m in ms]), one.vector(L.EPS)) < RTOL
    g.close()


def test_rowshard_automatic_block_size_from_cohort(brr, oracle_mod, require_gpu):
    """block_size = 0 picks B from the cohort's N_total on every shard: a cohort split
    across the N = 32,768 boundary (40k + 24k rows) runs B = 512 on both shards, as the unsharded
    chain does, and matches the unsharded oracle."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 64_000, 600
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    cuts = [0, 40_000, N]
    g, ms, orc = _build(brr, O, L.MODEL_V2, X, Y, cuts, 0, B=0)
    assert [m.block_size for m in ms] == [512, 512]
    for it in range(2):
        g.sweep(1)
        orc.sweep(1)
        _compare(ms, orc, O, L, L.MODEL_V2, f"auto-B it={it}")
    g.close()


def test_rowshard_set_state_then_read_then_sweep(brr, oracle_mod, require_gpu):
    """set_vector(EPS) / set_scalar(MU) on every shard, a state read (which used to reduce the
    residual sums over this shard's rows only and mark them final), then a group sweep: the
    residual sums must still be summed across the shards."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 900, 512
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=30)
    cuts = [0, 380, N]
    g, ms, orc = _build(brr, O, L.MODEL_V2, X, Y, cuts, 0)
    g.sweep(2)
    orc.sweep(2)
    eps = orc.vector(O.V_EPS) + 0.01 * np.sin(np.arange(N))
    mu = orc.scalar(O.S_MU) + 0.05
    orc.set_vector(O.V_EPS, eps)
    orc.set_scalar(O.S_MU, mu)
    for m, a, b in zip(ms, cuts[:-1], cuts[1:]):
        m.set_vector(L.EPS, eps[a:b])
        m.set_scalar(L.MU, mu)
    ms[0].scalar(L.MU)  # a read between the setters and the sweep
    ms[1].vector(L.BETA)
    for it in range(2):
        g.sweep(1)
        orc.sweep(1)
        _compare(ms, orc, O, L, L.MODEL_V2, f"set-eps it={it}")
    g.close()
