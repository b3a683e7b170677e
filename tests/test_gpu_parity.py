"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same seeded
inputs, the same Philox draws and the same visit order.

Tolerance (BASELINE north_star "within a stated floating-point tolerance"): component
assignments identical; beta, epsilon, mu, sigmaE, sigmaG, pi, tau, lambda within relative
1e-9 (f64 on both sides; the only differences are summation order and libm ulps).
"""
import os
import tempfile

import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu

RTOL = 1e-9


def _cohort(O, N, P, seed=20261015, n_causal=None):
    X, Y, b = O.synth_cohort(seed, N, P, h2=0.5, n_causal=n_causal)
    return X, Y, b


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nf = ~np.isfinite(b)
    if nf.any():
        # degenerate draws (e.g. sigmaG = inf from a scaled-inverse-chi^2 with v0G + m0 = 1e-4 degrees
        # of freedom): the same non-finite value on both sides, the finite rest compared as usual
        if not np.array_equal(a[nf], b[nf], equal_nan=True):
            return float("inf")
        a, b = a[~nf], b[~nf]
        if not a.size:
            return 0.0
    scale = np.maximum(np.abs(b), np.max(np.abs(b)) * 1e-3 + 1e-300)
    return float(np.max(np.abs(a - b) / scale)) if a.size else 0.0


def _compare(sess, orc, O, L, model, tag=""):
    bg, bo = sess.vector(L.BETA), orc.vector(O.V_BETA)
    eg, eo = sess.vector(L.EPS), orc.vector(O.V_EPS)
    assert _rel(bg, bo) < RTOL, f"{tag} beta rel err {_rel(bg, bo)}"
    assert _rel(eg, eo) < RTOL, f"{tag} eps rel err {_rel(eg, eo)}"
    assert abs(sess.scalar(L.MU) - orc.scalar(O.S_MU)) <= RTOL * (1 + abs(orc.scalar(O.S_MU))), tag
    assert _rel([sess.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < RTOL, tag
    if model == L.MODEL_HORSESHOE:
        for a, b in ((L.TAU, O.S_TAU), (L.ETA, O.S_ETA), (L.C2, O.S_C2)):
            assert _rel([sess.scalar(a)], [orc.scalar(b)]) < RTOL, f"{tag} scalar {a}"
        assert _rel(sess.vector(L.LAMBDA), orc.vector(O.V_LAMBDA)) < RTOL, tag
    else:
        cg, co = sess.vector(L.COMP), orc.vector(O.V_COMP)
        assert np.array_equal(cg, co), f"{tag} comps differ at {np.nonzero(cg != co)[0][:10]}"
        assert _rel(sess.vector(L.SIGMAGG), orc.vector(O.V_SIGMAGG)) < RTOL, tag
        assert _rel(sess.vector(L.PI), orc.vector(O.V_PI)) < RTOL, tag
        assert np.array_equal(sess.vector(L.VCOUNT), orc.vector(O.V_VCOUNT)), tag


def _make(brr, O, model, X, Y, order_mode, B=128, G=1, gAssign=None, fixed=None, cva=CVA,
          seed=7, restart=None, hs=None, xs="f32"):
    from bayesrrcpp_amd import _lib as L
    N, P = X.shape
    K = 1 if model == L.MODEL_HORSESHOE else np.atleast_2d(cva).shape[-1] + 1
    F = 0 if fixed is None else np.asarray(fixed).reshape(N, -1).shape[1]
    s = brr.Session(model, N, P, K=K, groups=G, F=F, block_size=B, order_mode=order_mode,
                    x_storage=L.X_2BIT if xs == "2bit" else L.X_F32)
    s.upload_x(X)
    okw = {}
    if model != L.MODEL_RESTART:
        s.set_y(Y)
    if model == L.MODEL_HORSESHOE:
        s.set_horseshoe(**hs)
        okw.update(hs)
    else:
        cva2 = np.tile(np.asarray(cva, float), (G, 1)) if np.ndim(cva) == 1 else np.asarray(cva)
        s.set_bayesr(HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], cva2, gAssign)
        okw.update(HYP)
        okw.update(cva=cva2, G=G)
        if gAssign is not None:
            okw["gAssign"] = gAssign
    if fixed is not None:
        s.set_fixed(fixed)
        okw["fixed"] = fixed
    if restart is not None:
        s.set_restart(restart["mu0"], restart["beta0"], restart["sigmaE0"], restart["sigmaGG0"],
                      restart["eps0"], restart["comp0"])
        okw.update(restart)
    s.init(seed)
    orc = O.Oracle(model, X, None if model == L.MODEL_RESTART else Y, seed=seed,
                   order_mode=order_mode, block_size=B, N=N, **okw)
    return s, orc


@pytest.mark.parametrize("order", [2, 0, 1])  # IDENTITY, BLOCKED, REFERENCE
def test_v2_trajectory(brr, oracle_mod, require_gpu, order):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 300, 500, n_causal=30)
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, order)
    # init state: sigmaE and xsquared
    assert _rel(s.vector(L.XSQ), orc.vector(O.V_XSQ)) < 1e-12
    assert _rel([s.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < 1e-12
    assert _rel([s.scalar(L.SIGMAG)], [orc.scalar(O.S_SIGMAG)]) == 0.0
    for it in range(6):
        s.sweep(1)
        orc.sweep(1)
        assert np.array_equal(s.vector(L.ORDER), orc.vector(O.V_ORDER)), f"visit order it={it}"
        _compare(s, orc, O, L, L.MODEL_V2, tag=f"order={order} it={it}")


def test_v2_block64_and_many_sweeps(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 257, 333, n_causal=20)
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0, B=64, cva=[1e-3, 1e-2])
    for it in range(20):
        s.sweep(1)
        orc.sweep(1)
    _compare(s, orc, O, L, L.MODEL_V2, tag="B=64 20 sweeps")


@pytest.mark.parametrize("cva", [[1e-3, 1e-2], [1e-4, 1e-3, 1e-2], [1e-4, 1e-3, 3e-3, 1e-2]])
def test_redecision_heavy_chain(brr, oracle_mod, require_gpu, cva):
    """Few rows, strong effects: a chain's nums move far and many positions leave their decision
    windows, so the serial chain re-decides often -- K = 4 through the compile-time quad form
    (decide_fast_quad, a re-decided change stepped at once), K = 3 and 5 through the runtime-K form --
    against the oracle, component choices identical, over several sweeps at B = 128."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 96, 640, n_causal=60)
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0, B=128, cva=cva)
    for it in range(8):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_V2, tag=f"K={len(cva) + 1} it={it}")


@pytest.mark.parametrize("xs", ["f32", "2bit"])
@pytest.mark.parametrize("B", [256, 512])
def test_v2_large_blocks(brr, oracle_mod, require_gpu, B, xs):
    """Multi-chunk streaming grid, a partial last block, Gram-row slot overflow (sweep 1 changes
    most markers: more candidates than LDS slots) and ragged N (not a multiple of 256 rows)."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 301, 1300, n_causal=40)
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0, B=B, xs=xs)
    for it in range(5):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_V2, tag=f"B={B} {xs} it={it}")


@pytest.mark.parametrize("mode", ["persistent", "persistent-cap7", "persistent-cap30", "persistent-lag1", "per-block"])
def test_pipeline_modes_midsize(brr, oracle_mod, require_gpu, monkeypatch, mode):
    """The sweep pipeline at a size with many streaming workgroups and reduction groups: the fused
    persistent sweep (256 rows per streaming workgroup; 7 workgroups of 12 passes; 27 workgroups
    of 768 rows -- f32 row ranges at B >= 256 are whole 256-row passes -- the last one ragged; lag 2
    and lag 1) and the per-block kernels, all against the oracle over several sweeps."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    cap = {"persistent-cap7": 7, "persistent-cap30": 30}.get(mode)
    if cap:
        monkeypatch.setenv("BRR_STREAM_WG", str(cap))
    if mode == "per-block":
        monkeypatch.setenv("BRR_PER_BLOCK", "1")
    if mode == "persistent-lag1":  # the fused sweep with the lag-1 pipeline (default: lag 2)
        monkeypatch.setenv("BRR_LAG", "1")
    N = 20000
    X, Y, _ = _cohort(O, N, 3000, n_causal=60)
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0, B=512)
    if mode.startswith("persistent"):
        rpw = max(256, (-(-N // cap) + 255) // 256 * 256) if cap else 256
        assert s.scalar(104) == -(-N // rpw)
    else:
        assert s.scalar(104) == 0
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_V2, tag=f"{mode} it={it}")


def test_list_prefetch_engaged_and_bit_identical(brr, require_gpu, monkeypatch):
    """The streamers' list prefetch (f32 storage: the change list of boundary s + 1 and its column rows
    fetched into LDS while block s streams) serves boundaries in a streaming-bound sweep, and the chain
    equals, bit for bit, that of a session with the prefetch switched off (BRR_LIST_PREFETCH=0: every
    list applied by the ordinary path, itself pinned to the oracle by the parity tests above).  C2's
    rows (100,000: two 256-row passes per streaming workgroup) on the on-device synthetic cohort with
    32 causal markers, 128 blocks of 512 markers, lag 2 in every sweep.  (A sweep is streaming-bound
    only when few markers change per block: a denser posterior keeps the solver the bound and its
    lists are published too late to prefetch -- C2 itself: 93 % of the boundaries served.)"""
    from bayesrrcpp_amd import _lib as L
    monkeypatch.setenv("BRR_LAG", "2")
    N, P = 100_000, 65_536

    def make():
        s = brr.Session(L.MODEL_V2, N, P, K=4, block_size=512)
        s.synthesize(20261015, 0.5, 32)
        s.set_bayesr(HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], np.asarray(CVA, float), None)
        s.init(3)
        return s

    s = make()
    assert s.scalar(104) > 0  # the fused sweep
    monkeypatch.setenv("BRR_LIST_PREFETCH", "0")
    s0 = make()
    for it in range(30):
        if it == 20:  # past the burn-in (solver-bound: lists published too late to prefetch)
            s.set_scalar(102, 1.0)  # diagnostics counters on (they count, nothing else changes)
        s.sweep(1)
        s0.sweep(1)
        for w in (L.BETA, L.EPS, L.COMP):
            assert np.array_equal(s.vector(w), s0.vector(w)), f"prefetch on/off differ ({w}) at sweep {it}"
        assert s.scalar(L.SIGMAE) == s0.scalar(L.SIGMAE)
    served = s.scalar(126)
    s.close()
    s0.close()
    assert served > 0, "no boundary was served by the list prefetch"


@pytest.mark.parametrize("B,xs", [(512, "f32"), (512, "2bit"), (256, "2bit")])
def test_horseshoe_block512(brr, oracle_mod, require_gpu, B, xs):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 260, 700
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    A = (1 / np.sqrt(N)) * 150 / (P - 150)
    hs = dict(A=A, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    s, orc = _make(brr, O, L.MODEL_HORSESHOE, X, Y, 0, B=B, hs=hs, xs=xs)
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_HORSESHOE, tag=f"hs B={B} {xs} it={it}")


@pytest.mark.parametrize("xs", ["f32", "2bit"])
def test_horseshoe_default_pipeline(brr, oracle_mod, require_gpu, monkeypatch, xs):
    """The Horseshoe's default marker loop: lag 2 in every sweep after the first (the burn-in included) with the
    cross-Gram corrections in the reducers, many blocks and several streaming workgroups, against
    the oracle."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    monkeypatch.setenv("BRR_STREAM_WG", "5")
    N, P, B = 1500, 1100, 128
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    A = (1 / np.sqrt(N)) * 150 / (P - 150)
    hs = dict(A=A, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    s, orc = _make(brr, O, L.MODEL_HORSESHOE, X, Y, 0, B=B, hs=hs, xs=xs)
    assert s.scalar(104) > 0 and s.scalar(106) == 2  # fused sweep, lag-2 pipeline
    for it in range(4):
        assert int(s.scalar(108)) == (1 if it == 0 else 2)  # this sweep's lag (the first from init: 1)
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_HORSESHOE, tag=f"hs default {xs} it={it}")
    s.close()


@pytest.mark.parametrize("model,B,xs", [(0, 512, "f32"), (0, 128, "2bit"), (3, 128, "f32")])
def test_solver_side_correction_matches_oracle(brr, oracle_mod, require_gpu, monkeypatch, model, B, xs):
    """The cross-Gram corrections summed by the solver instead of the reducers (BRR_RED_CORR=0; the
    default corrects in the reducers for every fused sweep) at lag 1 and 2, against the oracle."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    monkeypatch.setenv("BRR_STREAM_WG", "5")
    monkeypatch.setenv("BRR_RED_CORR", "0")
    N, P = 1500, 4 * B + 100
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    hs = None
    if model == L.MODEL_HORSESHOE:
        A = (1 / np.sqrt(N)) * 150 / (P - 150)
        hs = dict(A=A, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    for lag in ("1", "2"):
        monkeypatch.setenv("BRR_LAG", lag)
        s, orc = _make(brr, O, model, X, Y, 0, B=B, hs=hs, xs=xs)
        assert s.scalar(104) > 0
        for it in range(3):
            s.sweep(1)
            orc.sweep(1)
            _compare(s, orc, O, L, model, tag=f"solver-side correction lag {lag} it={it}")
        s.close()


def test_groups_fixed_effects(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, G = 280, 400, 5
    X, Y, _ = _cohort(O, N, P, n_causal=25)
    gA = (np.arange(P) * G // P).astype(np.int32)
    rng = np.random.default_rng(3)
    fixed = rng.normal(size=(N, 3))
    cva = np.array([[1e-4, 1e-3, 1e-2]] * G) * (1 + np.arange(G))[:, None]
    for order in (0, 1):
        s, orc = _make(brr, O, L.MODEL_GROUPS, X, Y, order, G=G, gAssign=gA, fixed=fixed, cva=cva)
        for it in range(5):
            s.sweep(1)
            orc.sweep(1)
            _compare(s, orc, O, L, L.MODEL_GROUPS, tag=f"groups order={order} it={it}")
            assert _rel(s.vector(L.ALPHA), orc.vector(O.V_ALPHA)) < RTOL
            assert _rel([s.scalar(L.SIGMAF)], [orc.scalar(O.S_SIGMAF)]) < RTOL
            assert _rel(s.vector(L.BETAACUM), orc.vector(O.V_BETAACUM)) < RTOL


@pytest.mark.parametrize("order,xs", [(0, "f32"), (1, "f32"), (0, "2bit"), (1, "2bit")])
def test_restart(brr, oracle_mod, require_gpu, order, xs):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, G = 250, 300, 3
    X, Y, _ = _cohort(O, N, P, n_causal=20)
    gA = (np.arange(P) % G).astype(np.int32)
    # a previous chain's last state (taken from the oracle)
    prev = O.Oracle(O.GROUPS, X, Y, cva=np.tile(CVA, (G, 1)), G=G, gAssign=gA, seed=3,
                    order_mode=0, block_size=128, **HYP)
    prev.sweep(4)
    st = dict(mu0=prev.scalar(O.S_MU), beta0=prev.vector(O.V_BETA), sigmaE0=prev.scalar(O.S_SIGMAE),
              sigmaGG0=prev.vector(O.V_SIGMAGG), eps0=prev.vector(O.V_EPS), comp0=prev.vector(O.V_COMP))
    s, orc = _make(brr, O, L.MODEL_RESTART, X, None, order, G=G, gAssign=gA, restart=st, xs=xs)
    assert _rel(s.vector(L.PI), orc.vector(O.V_PI)) < RTOL  # Dirichlet(v+1) from components
    for it in range(5):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_RESTART, tag=f"restart order={order} {xs} it={it}")


@pytest.mark.parametrize("order", [0, 1])
def test_horseshoe(brr, oracle_mod, require_gpu, order):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 300, 450
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    A = (1 / np.sqrt(N)) * 150 / (P - 150)  # HorseshoeR.cpp:317-318 recipe
    hs = dict(A=A, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    s, orc = _make(brr, O, L.MODEL_HORSESHOE, X, Y, order, hs=hs)
    assert _rel([s.scalar(L.TAU)], [orc.scalar(O.S_TAU)]) < RTOL
    for it in range(5):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_HORSESHOE, tag=f"hs order={order} it={it}")


def test_forced_state_single_sweep(brr, oracle_mod, require_gpu):
    """Identical injected state (beta, comps, pi, sigmas) -> one sweep -> identical result."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 200, 256, n_causal=20)
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0)
    rng = np.random.default_rng(11)
    beta = np.where(rng.random(256) < 0.3, rng.normal(0, 0.05, 256), 0.0)
    comp = np.where(beta != 0, rng.integers(1, 4, 256), 0).astype(float)
    pi = np.array([0.6, 0.2, 0.15, 0.05])
    eps = Y - X @ beta
    s.set_vector(L.BETA, beta); orc.set_vector(O.V_BETA, beta)
    s.set_vector(L.COMP, comp); orc.set_vector(O.V_COMP, comp)
    s.set_vector(L.PI, pi); orc.set_vector(O.V_PI, pi)
    s.set_vector(L.EPS, eps); orc.set_vector(O.V_EPS, eps)
    s.set_scalar(L.SIGMAE, 0.6); orc.set_scalar(O.S_SIGMAE, 0.6)
    s.set_scalar(L.SIGMAG, 0.3); orc.set_scalar(O.S_SIGMAG, 0.3)
    s.sweep(1)
    orc.sweep(1)
    _compare(s, orc, O, L, L.MODEL_V2, tag="forced")


def test_synthetic_x_bitwise(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 777, 100
    s = brr.Session(L.MODEL_V2, N, P, K=4)
    s.synthesize(20261015, 0.5, 10)
    s.set_bayesr(**HYP, cva=CVA)
    s.init(1)
    Xo = O.synth_x(20261015, N, P)
    xsq_o = (Xo * Xo).sum(0)
    # X identical bit for bit -> identical column norms up to summation order
    assert _rel(s.vector(L.XSQ), xsq_o) < 1e-12
    assert np.allclose(s.vector(L.XSQ), N - 1, rtol=1e-5)


def test_oneshot_csv_v2(brr, oracle_mod, require_gpu, tmp_path):
    """The drop-in entry point writes the reference CSV; it matches the oracle's CSV."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 120, 150, n_causal=10)
    p_gpu = str(tmp_path / "gpu.csv")
    p_orc = str(tmp_path / "orc.csv")
    brr.BayesRSamplerV2(p_gpu, 5, 30, 10, 4, X, Y, HYP["sigma0"], HYP["v0E"], HYP["s02E"],
                        HYP["v0G"], HYP["s02G"], CVA, log=lambda m: None)
    O.run_csv(p_orc, O.V2, X, Y, 30, 10, 4, cva=CVA, seed=5, order_mode=0, **HYP)
    g = open(p_gpu).read().splitlines()
    o = open(p_orc).read().splitlines()
    assert g[0] == o[0]  # header
    assert len(g) == len(o) == 1 + len([i for i in range(10, 30) if i % 4 == 0])
    for lg, lo in zip(g[1:], o[1:]):
        a = np.array([float(v) for v in lg.split(", ")])
        b = np.array([float(v) for v in lo.split(", ")])
        assert a.shape == b.shape
        assert np.allclose(a, b, rtol=2e-5, atol=1e-9)


def test_oneshot_validation(brr, require_gpu, tmp_path):
    p = str(tmp_path / "bad.csv")
    msgs = []
    X = np.ones((10, 5))
    brr.BayesRSamplerV2(p, 1, 10, 20, 1, X, np.ones(10), 0.01, 1e-4, 1e-3, 1e-4, 1e-3, CVA,
                        log=msgs.append)
    assert any("burn_in has to be a positive integer" in m for m in msgs)
    assert open(p).read().startswith("iteration,mu,beta[1]")  # header written before the check


@pytest.mark.parametrize("xs", ["f32", "2bit"])
def test_sharded_two_sessions_match_oracle(brr, oracle_mod, require_gpu, xs):
    """Column-sharded protocol: two sessions on one GPU, residual deltas and statistics summed
    on the host (the role ncclAllReduce plays across GPUs) == the oracle's 2-shard emulation."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, B = 260, 512, 128
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    shards = [(0, 256), (256, 256)]
    sess = []
    for r, (c0, pl) in enumerate(shards):
        s = brr.Session(L.MODEL_V2, N, pl, K=4, M_total=P, col_offset=c0, block_size=B,
                        shard_rank=r, shard_count=2, x_storage=L.X_2BIT if xs == "2bit" else L.X_F32,
                        exchanges_per_sweep=1)  # (E > 1: tests/test_gpu_exchange.py)
        s.upload_x(X[:, c0:c0 + pl])
        s.set_y(Y)
        s.set_bayesr(**HYP, cva=CVA)
        s.init(9)
        s.exchange_buffers()
        sess.append(s)
    orc = O.Oracle(O.V2, X, Y, cva=CVA, seed=9, order_mode=0, block_size=B, n_shards=2, **HYP)
    for it in range(4):
        for s in sess:
            s.sweep_local()
        parts = [s.exchange_get() for s in sess]
        te = parts[0][0] + parts[1][0]
        ts = parts[0][1] + parts[1][1]
        for s in sess:
            s.exchange_set(te, ts)
            s.sweep_finish()
        orc.sweep(1)
        beta = np.concatenate([s.vector(L.BETA) for s in sess])
        comp = np.concatenate([s.vector(L.COMP) for s in sess])
        assert np.array_equal(comp, orc.vector(O.V_COMP)), f"it={it}"
        assert _rel(beta, orc.vector(O.V_BETA)) < RTOL
        for s in sess:
            assert _rel(s.vector(L.EPS), orc.vector(O.V_EPS)) < RTOL
            assert _rel([s.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < RTOL
            assert _rel(s.vector(L.PI), orc.vector(O.V_PI)) < RTOL


@pytest.mark.parametrize("model,xs", [(0, "f32"), (1, "f32"), (3, "f32"), (0, "2bit")])
def test_sharded_reference_order_matches_oracle(brr, oracle_mod, require_gpu, model, xs):
    """REFERENCE visit order over two column shards: every shard draws the same global
    std::random_shuffle permutation (BayesRv2.cpp:182; Groups: fixedI first, :216) and visits its
    own columns in that order; host-summed exchange == the oracle's 2-shard emulation."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, B = 260, 512, 128
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    G = 2 if model == L.MODEL_GROUPS else 1
    gA = (np.arange(P) * G // P).astype(np.int32) if G > 1 else None
    F = 1 if model == L.MODEL_GROUPS else 0
    fixed = np.ones((N, 1)) if F else None
    cva = np.tile(CVA, (G, 1))
    hs = dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    sess = []
    for r, (c0, pl) in enumerate([(0, 256), (256, 256)]):
        s = brr.Session(model, N, pl, K=1 if model == L.MODEL_HORSESHOE else 4, groups=G, F=F, M_total=P,
                        col_offset=c0, block_size=B, shard_rank=r, shard_count=2, order_mode=L.ORDER_REFERENCE,
                        x_storage=L.X_2BIT if xs == "2bit" else L.X_F32, exchanges_per_sweep=1)
        s.upload_x(X[:, c0:c0 + pl])
        s.set_y(Y)
        if model == L.MODEL_HORSESHOE:
            s.set_horseshoe(**hs)
        else:
            s.set_bayesr(**HYP, cva=cva, gAssign=gA[c0:c0 + pl] if G > 1 else None)
        if F:
            s.set_fixed(fixed)
        s.init(9)
        s.exchange_buffers()
        sess.append(s)
    if model == L.MODEL_HORSESHOE:
        orc = O.Oracle(O.HORSESHOE, X, Y, seed=9, order_mode=O.ORDER_REFERENCE, block_size=B, n_shards=2, **hs)
    else:
        orc = O.Oracle({0: O.V2, 1: O.GROUPS}[model], X, Y, cva=cva, G=G, gAssign=gA, fixed=fixed, seed=9,
                       order_mode=O.ORDER_REFERENCE, block_size=B, n_shards=2, **HYP)
    for it in range(4):
        for s in sess:
            s.sweep_local()
        parts = [s.exchange_get() for s in sess]
        te = parts[0][0] + parts[1][0]
        ts = parts[0][1] + parts[1][1]
        for s in sess:
            s.exchange_set(te, ts)
            s.sweep_finish()
        orc.sweep(1)
        beta = np.concatenate([s.vector(L.BETA) for s in sess])
        if model != L.MODEL_HORSESHOE:
            comp = np.concatenate([s.vector(L.COMP) for s in sess])
            assert np.array_equal(comp, orc.vector(O.V_COMP)), f"it={it}"
        assert _rel(beta, orc.vector(O.V_BETA)) < RTOL
        for s in sess:
            assert _rel(s.vector(L.EPS), orc.vector(O.V_EPS)) < RTOL
            assert _rel([s.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < RTOL


def test_restart_column_shards(brr, oracle_mod, require_gpu):
    """Restart across two column shards: the pi init's component counts (BRv2Grstart.cpp:157-165)
    summed across shards through init_local / exchange / init_finish, then the column-sharded
    sweep, == the oracle's 2-shard emulation; a sharded restart without a communicator or the
    split init is refused."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, B, G = 260, 512, 128, 3
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    gA = (np.arange(P) % G).astype(np.int32)
    cva2 = np.tile(CVA, (G, 1))
    prev = O.Oracle(O.GROUPS, X, Y, cva=cva2, G=G, gAssign=gA, seed=3, order_mode=0, block_size=B, **HYP)
    prev.sweep(4)
    st = dict(mu0=prev.scalar(O.S_MU), beta0=prev.vector(O.V_BETA), sigmaE0=prev.scalar(O.S_SIGMAE),
              sigmaGG0=prev.vector(O.V_SIGMAGG), eps0=prev.vector(O.V_EPS), comp0=prev.vector(O.V_COMP))
    sess = []
    for r, c0 in enumerate((0, 256)):
        s = brr.Session(L.MODEL_RESTART, N, 256, K=len(CVA) + 1, groups=G, M_total=P, col_offset=c0,
                        block_size=B, shard_rank=r, shard_count=2, exchanges_per_sweep=1)
        s.upload_x(X[:, c0:c0 + 256])
        s.set_bayesr(HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], cva2, gA[c0:c0 + 256])
        s.set_restart(st["mu0"], st["beta0"][c0:c0 + 256], st["sigmaE0"], st["sigmaGG0"], st["eps0"],
                      st["comp0"][c0:c0 + 256])
        sess.append(s)
    with pytest.raises(RuntimeError, match="column shards"):
        sess[0].init(11)
    for s in sess:
        s.init_local(11)
    tot = sum(s.exchange_get()[1] for s in sess)
    for s in sess:
        s.exchange_set(None, tot)
        s.init_finish()
    orc = O.Oracle(O.RESTART, X, None, cva=cva2, G=G, gAssign=gA, seed=11, order_mode=0, block_size=B,
                   N=N, n_shards=2, **HYP, **st)
    for s in sess:
        assert _rel(s.vector(L.PI), orc.vector(O.V_PI)) < RTOL  # Dirichlet(v + 1) of the summed counts
    for it in range(4):
        for s in sess:
            s.sweep_local()
        parts = [s.exchange_get() for s in sess]
        te = parts[0][0] + parts[1][0]
        ts = parts[0][1] + parts[1][1]
        for s in sess:
            s.exchange_set(te, ts)
            s.sweep_finish()
        orc.sweep(1)
        comp = np.concatenate([s.vector(L.COMP) for s in sess])
        assert np.array_equal(comp, orc.vector(O.V_COMP)), f"it={it}"
        assert _rel(np.concatenate([s.vector(L.BETA) for s in sess]), orc.vector(O.V_BETA)) < RTOL
        for s in sess:
            assert _rel(s.vector(L.EPS), orc.vector(O.V_EPS)) < RTOL
            assert _rel([s.scalar(L.SIGMAE)], [orc.scalar(O.S_SIGMAE)]) < RTOL
            assert _rel(s.vector(L.PI), orc.vector(O.V_PI)) < RTOL
            assert _rel(s.vector(L.SIGMAGG), orc.vector(O.V_SIGMAGG)) < RTOL


def test_rccl_single_rank(brr, oracle_mod, require_gpu):
    """brr_session_comm_init + sweep with a 1-rank RCCL communicator runs the native path."""
    from bayesrrcpp_amd import _lib as L
    from bayesrrcpp_amd.session import comm_unique_id
    O = oracle_mod
    X, Y, _ = _cohort(O, 200, 256, n_causal=20)
    s = brr.Session(L.MODEL_V2, 200, 256, K=4, shard_rank=0, shard_count=1)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=CVA).init(3)
    s.comm_init(comm_unique_id(), 1, 0)
    s.sweep(3)
    orc = O.Oracle(O.V2, X, Y, cva=CVA, seed=3, order_mode=0, **HYP)
    orc.sweep(3)
    _compare(s, orc, O, L, L.MODEL_V2, tag="rccl 1 rank")


def test_recycled_device_memory(brr, oracle_mod, require_gpu):
    """Sessions of different shapes back to back: a later session gets the earlier one's
    freed device memory and must not read any of it before writing (regression: slab2 pad
    rows / member padding were once left uninitialised)."""
    import gc
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    for (N, P, B, cva) in [(257, 333, 64, [1e-3, 1e-2]), (257, 333, 128, [1e-3, 1e-2]),
                           (600, 333, 64, [1e-3, 1e-2]), (257, 333, 64, list(CVA))]:
        X, Y, _ = _cohort(O, N, P, n_causal=20)
        s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0, B=B, cva=cva)
        for it in range(3):
            s.sweep(1)
            orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_V2, tag=f"recycled N={N} B={B}")
        del s, orc
        gc.collect()


@pytest.mark.parametrize("xs", ["f32", "2bit"])
@pytest.mark.parametrize("lag", [1, 2, 3])
@pytest.mark.parametrize("model", [0, 1, 2, 3])  # V2, Groups, restart, Horseshoe
def test_pipeline_lag_all_models(brr, oracle_mod, require_gpu, monkeypatch, model, lag, xs):
    """Every pipeline lag (default: 2 for every model in BLOCKED order with nb >= 4 -- V2 / restart
    adaptively, lag 1 in sweeps after one that changed many markers; 3 is opt-in) for every model,
    against the oracle: many blocks, several streaming workgroups."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    monkeypatch.setenv("BRR_LAG", str(lag))
    monkeypatch.setenv("BRR_STREAM_WG", "5")
    N, P = 1500, 1100
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    kw = {}
    if model == L.MODEL_GROUPS:
        G = 3
        kw = dict(G=G, gAssign=(np.arange(P) * G // P).astype(np.int32),
                  fixed=np.linspace(-1, 1, N).reshape(N, 1))
    elif model == L.MODEL_RESTART:
        rng = np.random.default_rng(3)
        comp0 = rng.integers(0, 4, P).astype(np.float64)
        beta0 = np.where(comp0 > 0, rng.normal(0, 0.02, P), 0.0)
        kw = dict(restart=dict(mu0=0.01, beta0=beta0, sigmaE0=0.7, sigmaGG0=np.array([0.3]),
                               eps0=Y - X @ beta0 - 0.01, comp0=comp0))
    elif model == L.MODEL_HORSESHOE:
        kw = dict(hs=dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0))
    s, orc = _make(brr, O, model, X, Y, 0, B=128, xs=xs, **kw)
    assert s.scalar(104) > 1  # fused sweep
    assert s.scalar(106) == lag
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, model, tag=f"model={model} lag={lag} {xs} it={it}")


@pytest.mark.parametrize("lag", [1, 2])
def test_groups_22_c3_layout(brr, oracle_mod, require_gpu, monkeypatch, lag):
    """C3's group layout at a size the oracle runs in seconds: G = 22, gAssign = floor(22 j / P),
    identical cva rows, one all-zero fixed column (vignettes/BayesRR.Rmd:166); B = 128 (the
    automatic Groups block), several streaming workgroups (BayesRv2Groups.cpp:216-312)."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    monkeypatch.setenv("BRR_LAG", str(lag))
    N, P, G = 3000, 4400, 22
    X, Y, _ = _cohort(O, N, P, n_causal=60)
    gA = (np.arange(P) * G // P).astype(np.int32)
    s, orc = _make(brr, O, L.MODEL_GROUPS, X, Y, 0, B=128, G=G, gAssign=gA, fixed=np.zeros((N, 1)))
    assert s.scalar(104) > 1  # fused sweep
    for it in range(5):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, L.MODEL_GROUPS, tag=f"G=22 lag={lag} it={it}")
        assert _rel(s.vector(L.BETAACUM), orc.vector(O.V_BETAACUM)) < RTOL
        assert _rel([s.scalar(L.SIGMAF)], [orc.scalar(O.S_SIGMAF)]) < RTOL
    assert s.vector(L.SIGMAGG).size == G and len(set(s.vector(L.SIGMAGG))) == G


def _csv_rows(path):
    lines = open(path).read().splitlines()
    return lines


def _compare_csv(p_gpu, p_orc, header=True):
    g, o = _csv_rows(p_gpu), _csv_rows(p_orc)
    assert len(g) == len(o) and len(g) > int(header)
    if header:
        assert g[0] == o[0]
    for lg, lo in zip(g[int(header):], o[int(header):]):
        a = np.array([float(v) for v in lg.split(", ")])
        b = np.array([float(v) for v in lo.split(", ")])
        assert a.shape == b.shape
        assert np.allclose(a, b, rtol=2e-5, atol=1e-9)  # 6 significant digits on both sides


def test_oneshot_csv_groups(brr, oracle_mod, require_gpu, tmp_path):
    """brr_BayesRSamplerV2Groups writes the reference's Groups CSV (header and rows,
    BayesRv2Groups.cpp:25-54,314-318) equal to the oracle's."""
    O = oracle_mod
    N, P, G = 150, 260, 3
    X, Y, _ = _cohort(O, N, P, n_causal=15)
    gA = (np.arange(P) % G).astype(np.int32)
    cva = np.tile(CVA, (G, 1))
    fixed = np.linspace(-1, 1, 2 * N).reshape(N, 2)
    pg, po = str(tmp_path / "g.csv"), str(tmp_path / "o.csv")
    brr.BayesRSamplerV2Groups(pg, 4, 24, 8, 3, X, Y, HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"],
                              HYP["s02G"], cva, G, gA, fixed, block_size=128, log=lambda m: None)
    O.run_csv(po, O.GROUPS, X, Y, 24, 8, 3, cva=cva, G=G, gAssign=gA, fixed=fixed, seed=4, order_mode=0,
              block_size=128, **HYP)
    _compare_csv(pg, po)
    assert open(pg).readline().rstrip("\n").endswith("alpha[1],alpha[2],sigmaF")


def test_oneshot_csv_restart(brr, oracle_mod, require_gpu, tmp_path):
    """brr_BRV2Grstart: no header (BRv2Grstart.cpp:26 unused), rows as the reference's sample
    (BRv2Grstart.cpp:262-268), equal to the oracle's."""
    O = oracle_mod
    N, P, G = 140, 200, 2
    X, Y, _ = _cohort(O, N, P, n_causal=12)
    gA = (np.arange(P) % G).astype(np.int32)
    cva = np.tile(CVA, (G, 1))
    rng = np.random.default_rng(8)
    comp0 = rng.integers(0, 4, P).astype(np.float64)
    beta0 = np.where(comp0 > 0, rng.normal(0, 0.02, P), 0.0)
    eps0 = Y - X @ beta0 - 0.02
    pg, po = str(tmp_path / "g.csv"), str(tmp_path / "o.csv")
    brr.BRV2Grstart(pg, 6, 20, 5, 2, 0.02, beta0, 0.8, np.array([0.3, 0.2]), X, eps0, comp0, HYP["sigma0"],
                    HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"], cva, G, gA, block_size=512, log=lambda m: None)
    O.run_csv(po, O.RESTART, X, None, 20, 5, 2, cva=cva, G=G, gAssign=gA, seed=6, order_mode=0, block_size=512,
              mu0=0.02, beta0=beta0, sigmaE0=0.8, sigmaGG0=np.array([0.3, 0.2]), eps0=eps0, comp0=comp0, N=N, **HYP)
    _compare_csv(pg, po, header=False)
    first = open(pg).readline()
    assert not first.startswith("iteration") and len(first.split(", ")) == 2 + 2 * P + 1 + G + N


def test_oneshot_csv_horseshoe(brr, oracle_mod, require_gpu, tmp_path):
    """brr_HorseshoeR: header with the trailing comma (HorseshoeR.cpp:279-291) and every kept
    sample (2M+N+3 values plus the uninitialised last slot, HorseshoeR.cpp:157,258), equal to the
    oracle's."""
    O = oracle_mod
    N, P = 160, 240
    X, Y, _ = _cohort(O, N, P, n_causal=12)
    hs = dict(A=(1 / np.sqrt(N)) * 24 / (P - 24), v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    pg, po = str(tmp_path / "g.csv"), str(tmp_path / "o.csv")
    brr.HorseshoeR(pg, 2, 18, 6, 4, X, Y, hs["A"], hs["v0E"], hs["s02E"], hs["vL"], hs["vT"], hs["c2"], hs["vC"],
                   hs["sC"], block_size=128, log=lambda m: None)
    O.run_csv(po, O.HORSESHOE, X, Y, 18, 6, 4, seed=2, order_mode=0, block_size=128, **hs)
    _compare_csv(pg, po)
    assert open(pg).readline().rstrip("\n").endswith(f"epsilon[{N}],")


def test_f64_x_not_f32_representable(brr, oracle_mod, require_gpu):
    """The drop-in upload rounds the reference's f64 X to f32 on the device.
    On an X that is not f32-representable (scale()d dosages plus a 1e-4 jitter), the GPU chain
    equals the oracle run on the f32-rounded X (rtol 1e-9), and one sweep from the same state
    deviates from the oracle on the exact f64 X by at most rtol 1e-5 (the rounding of X,
    2^-24 relative, propagated through one sweep)."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 300, 400
    X, Y, _ = _cohort(O, N, P, n_causal=20)
    X64 = X.astype(np.float64) + 1e-4 * np.sin(np.arange(N * P, dtype=np.float64)).reshape(N, P)
    assert not np.array_equal(X64.astype(np.float32).astype(np.float64), X64)
    X32 = X64.astype(np.float32).astype(np.float64)
    s, orc32 = _make(brr, O, L.MODEL_V2, X64, Y, 0, B=128)  # session uploads f64 -> f32
    for it in range(3):
        s.sweep(1)
        orc32.sweep(1)
    orc32b = O.Oracle(O.V2, X32, Y, cva=CVA, seed=7, order_mode=0, block_size=128, **HYP)
    orc32b.sweep(3)
    _compare(s, orc32b, O, L, L.MODEL_V2, tag="f64 X vs oracle on f32(X)")
    # one sweep from the GPU's state, oracle on the exact f64 X
    o64 = O.Oracle(O.V2, X64, Y, cva=CVA, seed=7, order_mode=0, block_size=128, **HYP)
    o64.sweep(3)
    st = dict(beta=s.vector(L.BETA), comp=s.vector(L.COMP), pi=s.vector(L.PI), sigmaE=s.scalar(L.SIGMAE),
              sigmaG=s.scalar(L.SIGMAG), mu=s.scalar(L.MU))
    eps64 = Y - st["mu"] - X64 @ st["beta"]
    o64.set_vector(O.V_BETA, st["beta"]); o64.set_vector(O.V_COMP, st["comp"]); o64.set_vector(O.V_PI, st["pi"])
    o64.set_vector(O.V_EPS, eps64)
    o64.set_scalar(O.S_SIGMAE, st["sigmaE"]); o64.set_scalar(O.S_SIGMAG, st["sigmaG"]); o64.set_scalar(O.S_MU, st["mu"])
    s.sweep(1)
    o64.sweep(1)
    same = s.vector(L.COMP) == o64.vector(O.V_COMP)
    assert same.mean() > 0.99
    if same.all():
        assert _rel(s.vector(L.BETA), o64.vector(O.V_BETA)) < 1e-5
        assert _rel([s.scalar(L.SIGMAE)], [o64.scalar(O.S_SIGMAE)]) < 1e-5


def test_failed_census_exits_cleanly(brr, oracle_mod, require_gpu, monkeypatch):
    """A fused sweep whose residency census fails (forced: target above the grid) returns the
    protocol error without touching the chain's state; the session then goes on with the
    per-block kernels and keeps eps = Y - mu - X beta."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 2000, 1024
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    s, _ = _make(brr, O, L.MODEL_V2, X, Y, 0, B=128)
    s.sweep(2)
    assert s.scalar(104) > 0  # fused
    beta0, eps0 = s.vector(L.BETA), s.vector(L.EPS)
    monkeypatch.setenv("BRR_TEST_CENSUS_EXTRA", "100000")
    with pytest.raises(L.BrrError, match="site 5"):
        s.sweep(1)
    monkeypatch.delenv("BRR_TEST_CENSUS_EXTRA")
    assert np.array_equal(s.vector(L.BETA), beta0)  # the marker loop never ran
    assert s.scalar(104) == 0                       # per-block kernels from now on
    assert s.scalar(130) == 1                       # and the session counts the failure (bench.py reports it)
    s.sweep(3)
    resid = Y - s.scalar(L.MU) - X.astype(np.float64) @ s.vector(L.BETA)
    assert _rel(s.vector(L.EPS), resid) < 1e-9
    assert not np.array_equal(s.vector(L.EPS), eps0)


def test_failed_census_in_exchange_segment(brr, oracle_mod, require_gpu, monkeypatch):
    """A failed residency census in the FIRST of E = 4 exchange segments of a column shard: that
    segment's markers keep their values for the sweep, and the sweep's remaining segments -- on the
    per-block kernels, whose hand-over epochs are rebased past the failed segment -- and every later
    sweep complete without a protocol timeout; eps = Y - mu - X beta holds and the replicated residual
    stays bit-identical on both shards."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, B, E = 300, 1536, 128, 4
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=40)
    sess = []
    for r, c0 in enumerate((0, 768)):
        s = brr.Session(L.MODEL_V2, N, 768, K=4, M_total=P, col_offset=c0, block_size=B, shard_rank=r,
                        shard_count=2, exchanges_per_sweep=E)
        s.upload_x(X[:, c0:c0 + 768]).set_y(Y).set_bayesr(**HYP, cva=CVA).init(9)
        s.exchange_buffers()
        sess.append(s)
    assert all(s.scalar(104) > 0 for s in sess)

    def rounds(n, fail_first=False):
        for k in range(n):
            for i, s in enumerate(sess):
                if fail_first and k == 0 and i == 0:
                    monkeypatch.setenv("BRR_TEST_CENSUS_EXTRA", "100000")
                    with pytest.raises(L.BrrError, match="site 5"):
                        s.sweep_local()
                    monkeypatch.delenv("BRR_TEST_CENSUS_EXTRA")
                else:
                    s.sweep_local()
            parts = [s.exchange_get() for s in sess]
            te, ts = parts[0][0] + parts[1][0], parts[0][1] + parts[1][1]
            for s in sess:
                s.exchange_set(te, ts)
                s.sweep_finish()

    rounds(2 * E)
    rounds(E, fail_first=True)
    assert sess[0].scalar(104) == 0 and sess[1].scalar(104) > 0  # shard 0 on the per-block kernels now
    assert sess[0].scalar(130) == 1 and sess[1].scalar(130) == 0
    assert all(s.iteration == 3 for s in sess)
    rounds(2 * E)  # raises on a hand-over timeout
    assert all(s.iteration == 5 for s in sess)
    beta = np.concatenate([s.vector(L.BETA) for s in sess])
    mu = sess[0].scalar(L.MU)
    resid = Y - mu - X.astype(np.float64) @ beta
    assert _rel(sess[0].vector(L.EPS), resid) < 1e-9
    assert np.array_equal(sess[0].vector(L.EPS), sess[1].vector(L.EPS))
    for s in sess:
        s.close()


def test_adaptive_lag_switch_matches_oracle(brr, oracle_mod, require_gpu, monkeypatch):
    """The fused sweep's per-sweep pipeline lag (k_hyper: lag 1 while more markers change than
    Dev::lag_thresh, else lag 2) flips within a few sweeps when BRR_LAG_SWITCH puts the threshold
    inside the chain's own per-sweep change counts; both lags occur and the chain equals the oracle
    (identical components, 1e-9) in every sweep, across the flips."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, B, T = 2000, 4096, 256, 10
    X, Y, _ = _cohort(O, N, P, n_causal=40)
    orc = O.Oracle(O.V2, X, Y, cva=CVA, seed=5, order_mode=0, block_size=B, **HYP)
    nz = []
    for _ in range(T):
        b0 = orc.vector(O.V_BETA)
        orc.sweep(1)
        nz.append(int(np.count_nonzero(orc.vector(O.V_BETA) != b0)))
    # a threshold inside the burn-in's change counts: lag 1 while above it, lag 2 below
    thr = 0.5 * (max(nz[1:]) + min(nz[1:]))
    nb = P // B
    monkeypatch.setenv("BRR_LAG_SWITCH", repr(thr / (N / 1e5) / nb))
    s, orc = _make(brr, O, L.MODEL_V2, X, Y, 0, B=B, seed=5)
    assert s.scalar(104) > 0 and s.scalar(106) == 2
    lags = []
    for it in range(T):
        lags.append(int(s.scalar(108)))
        s.sweep(1)
        orc.sweep(1)
        assert np.array_equal(s.vector(L.COMP), orc.vector(O.V_COMP)), f"it={it} lags={lags}"
        assert _rel(s.vector(L.BETA), orc.vector(O.V_BETA)) < RTOL
        assert _rel(s.vector(L.EPS), orc.vector(O.V_EPS)) < RTOL
    assert 1 in lags and 2 in lags, (lags, nz, thr)


@pytest.mark.parametrize("depth", [1, 4])
def test_session_output_matches_oneshot(brr, oracle_mod, require_gpu, tmp_path, depth, monkeypatch):
    """The asynchronous sample pipeline (device snapshot -> pinned ring -> writer thread, SURVEY
    8f2): a session driving its own sweeps with brr_session_output_* writes the one-shot's file
    byte for byte, at any ring depth (depth 1 = the sampler waits for every row), and never has
    more rows in flight than the ring holds."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, 150, 200, n_causal=10)
    p1, p2 = str(tmp_path / "oneshot.csv"), str(tmp_path / "session.csv")
    monkeypatch.setenv("BRR_SAMPLE_RING", str(depth))
    brr.BayesRSamplerV2(p1, 5, 12, 2, 1, X, Y, HYP["sigma0"], HYP["v0E"], HYP["s02E"], HYP["v0G"], HYP["s02G"],
                        CVA, log=lambda m: None)
    s = brr.Session(L.MODEL_V2, 150, 200, K=4)
    s.upload_x(X).set_y(Y).set_bayesr(cva=CVA, **HYP).init(5)
    s.output_open(p2, ring_depth=depth)
    for it in range(12):
        s.sweep(1)
        if it >= 2:
            s.output_sample(it)
    assert 1 <= s.output_close() <= depth
    assert open(p1).read() == open(p2).read()


@pytest.mark.parametrize("model,N,P,order,kind", [
    (0, 7, 1, 1, "one marker, 7 rows"),
    (0, 64, 3, 0, "fewer markers than a wave"),
    (0, 300, 129, 0, "one full block and a one-marker block"),
    (0, 257, 200, 1, "K = 2 (one non-zero component)"),
    (0, 257, 200, 0, "an all-zero and a constant column"),
    (1, 90, 70, 1, "Groups: G = 3 with an empty group, fixed effect"),
    (3, 33, 5, 0, "Horseshoe, tiny"),
])
@pytest.mark.parametrize("xs", ["f32", "2bit"])
def test_edge_shapes(brr, oracle_mod, require_gpu, model, N, P, order, kind, xs):
    """Edge shapes against the oracle: a single marker, fewer markers or rows than a wave, a ragged
    one-marker last block, K = 2, degenerate columns (all zero: xsq = 0, BayesRv2.cpp:199; constant),
    an empty group, a tiny Horseshoe."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    X, Y, _ = _cohort(O, N, P, n_causal=max(1, min(5, P)))
    cva = CVA
    kw = {}
    if "K = 2" in kind:
        cva = [1e-2]
    if "degenerate" in kind or "all-zero" in kind:
        X = np.array(X)
        X[:, 3] = 0.0
        X[:, 7] = 0.5
    if model == L.MODEL_GROUPS:
        gA = np.where(np.arange(P) < P // 2, 0, 2).astype(np.int32)  # group 1 empty
        kw = dict(G=3, gAssign=gA, fixed=np.ones((N, 1)))
    if model == L.MODEL_HORSESHOE:
        kw = dict(hs=dict(A=1.0, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0))
    s, orc = _make(brr, O, model, X, Y, order, cva=cva, xs=xs, **kw)
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        _compare(s, orc, O, L, model, tag=f"{kind} {xs} it={it}")


@pytest.mark.parametrize("model", [0, 1, 3])
def test_2bit_reference_order_matches_oracle(brr, oracle_mod, require_gpu, model):
    """2-bit storage in the reference's own visit order: a REFERENCE block holds arbitrary
    columns, so the sweep runs the per-block kernels (each member column decoded by index; the
    fused streamers read whole column blocks in storage order) -- against the oracle."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P, B = 300, 400, 128
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    G = 3 if model == L.MODEL_GROUPS else 1
    gA = (np.arange(P) * G // P).astype(np.int32) if G > 1 else None
    hs = dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)
    s = brr.Session(model, N, P, K=1 if model == L.MODEL_HORSESHOE else 4, groups=G,
                    F=1 if model == L.MODEL_GROUPS else 0, block_size=B, order_mode=L.ORDER_REFERENCE,
                    x_storage=L.X_2BIT)
    s.upload_x(X)
    s.set_y(Y)
    okw = dict(hs)
    if model == L.MODEL_HORSESHOE:
        s.set_horseshoe(**hs)
    else:
        cva = np.tile(CVA, (G, 1))
        s.set_bayesr(**HYP, cva=cva, gAssign=gA)
        okw = dict(HYP, cva=cva, G=G, gAssign=gA)
        if model == L.MODEL_GROUPS:
            s.set_fixed(np.ones((N, 1)))
            okw["fixed"] = np.ones((N, 1))
    s.init(7)
    assert s.scalar(104) == 0  # per-block kernels
    orc = O.Oracle(model, X, Y, seed=7, order_mode=O.ORDER_REFERENCE, block_size=B, **okw)
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        assert np.array_equal(s.vector(L.ORDER), orc.vector(O.V_ORDER)), f"visit order it={it}"
        _compare(s, orc, O, L, model, tag=f"2bit reference model={model} it={it}")


@pytest.mark.parametrize("xs", ["f32", "2bit"])
@pytest.mark.parametrize("lag", [1, 2])
@pytest.mark.parametrize("ovs", [0, 1])
@pytest.mark.parametrize("model", [0, 1, 2])  # V2, Groups, restart
def test_overlapped_solver_both_ways(brr, oracle_mod, require_gpu, monkeypatch, model, ovs, lag, xs):
    """The overlapped solver workgroup (brr_ovsolve.hpp: block s+1's decisions, Gram triangle and every
    cross-Gram correction prepared while block s's chain runs; the default for Groups) and the round-5
    solver (the default for V2 / restart), each forced on every BayesR model, both pipeline lags and
    storages, against the oracle (BayesRv2.cpp:186-245, BayesRv2Groups.cpp:232-298)."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    monkeypatch.setenv("BRR_OVS", str(ovs))
    monkeypatch.setenv("BRR_LAG", str(lag))
    monkeypatch.setenv("BRR_STREAM_WG", "5")
    N, P = 1500, 1100
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    kw = {}
    if model == L.MODEL_GROUPS:
        G = 3
        kw = dict(G=G, gAssign=(np.arange(P) * G // P).astype(np.int32),
                  fixed=np.linspace(-1, 1, N).reshape(N, 1))
    elif model == L.MODEL_RESTART:
        rng = np.random.default_rng(3)
        comp0 = rng.integers(0, 4, P).astype(np.float64)
        beta0 = np.where(comp0 > 0, rng.normal(0, 0.02, P), 0.0)
        kw = dict(restart=dict(mu0=0.01, beta0=beta0, sigmaE0=0.7, sigmaGG0=np.array([0.3]),
                               eps0=Y - X @ beta0 - 0.01, comp0=comp0))
    s, orc = _make(brr, O, model, X, Y, 0, B=128, xs=xs, **kw)
    assert s.scalar(104) > 1  # fused sweep
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        assert s.scalar(132) == ovs
        _compare(s, orc, O, L, model, tag=f"model={model} ovs={ovs} lag={lag} {xs} it={it}")



@pytest.mark.parametrize("ovs", [0, 1])
@pytest.mark.parametrize("model", [0, 1, 2])  # V2, Groups, restart
def test_reference_order_lag2_matches_oracle(brr, oracle_mod, require_gpu, monkeypatch, model, ovs):
    """REFERENCE order on the fused sweep at pipeline lag 2 (BRR_LAG=2: a third Gram set per sweep, the
    layout's blocks two apart), with either solver, against the oracle's REFERENCE visit order
    (BayesRv2.cpp:182 random_shuffle; BayesRv2Groups.cpp:232-298)."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    monkeypatch.setenv("BRR_OVS", str(ovs))
    monkeypatch.setenv("BRR_LAG", "2")
    monkeypatch.setenv("BRR_STREAM_WG", "5")
    N, P = 1500, 1100
    X, Y, _ = _cohort(O, N, P, n_causal=30)
    kw = {}
    if model == L.MODEL_GROUPS:
        G = 3
        kw = dict(G=G, gAssign=(np.arange(P) * G // P).astype(np.int32),
                  fixed=np.linspace(-1, 1, N).reshape(N, 1))
    elif model == L.MODEL_RESTART:
        rng = np.random.default_rng(3)
        comp0 = rng.integers(0, 4, P).astype(np.float64)
        beta0 = np.where(comp0 > 0, rng.normal(0, 0.02, P), 0.0)
        kw = dict(restart=dict(mu0=0.01, beta0=beta0, sigmaE0=0.7, sigmaGG0=np.array([0.3]),
                               eps0=Y - X @ beta0 - 0.01, comp0=comp0))
    s, orc = _make(brr, O, model, X, Y, 1, B=128, **kw)
    assert s.scalar(104) > 1  # fused sweep
    assert s.scalar(106) == 2  # pipeline lag
    for it in range(4):
        s.sweep(1)
        orc.sweep(1)
        assert s.scalar(132) == ovs
        _compare(s, orc, O, L, model, tag=f"REFERENCE model={model} ovs={ovs} it={it}")
