"""Genotype storage: 2-bit codes + a per-column value table on the device.

The decoded values are the f32 values the dense storage holds, so a chain under BRR_X_2BIT must be
IDENTICAL (bit for bit) to the same chain under BRR_X_F32 -- every kernel sees the same inputs in
the same order -- and, like it, within the parity tolerance of the CPU oracle.  The PLINK .bed
loader is checked against a numpy restatement of its standardisation (same IEEE operations in the
same order, so the f32 values are identical) fed to the oracle.
"""
import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _same_lag(monkeypatch):
    # the automatic pipeline lag differs between the storages (f32 V2: 2, 2-bit: 1) and the two
    # lags order the floating-point corrections differently: compare the storages at one lag
    monkeypatch.setenv("BRR_LAG", "1")

RTOL = 1e-9


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.maximum(np.abs(b), np.max(np.abs(b)) * 1e-3 + 1e-300)
    return float(np.max(np.abs(a - b) / scale)) if a.size else 0.0


HS = dict(A=0.01, v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0)


def _session(brr, L, model, X, Y, B, x_storage, G=1, gA=None, seed=5, upload=None):
    N, P = X.shape
    K = 1 if model == L.MODEL_HORSESHOE else len(CVA) + 1
    F = 1 if model == L.MODEL_GROUPS else 0
    s = brr.Session(model, N, P, K=K, groups=G, F=F, block_size=B, x_storage=x_storage)
    if upload is None:
        s.upload_x(X)
    else:
        upload(s)
    s.set_y(Y)
    if model == L.MODEL_HORSESHOE:
        s.set_horseshoe(**HS)
    else:
        s.set_bayesr(**HYP, cva=np.tile(CVA, (G, 1)), gAssign=gA)
        if F:
            s.set_fixed(np.linspace(-1, 1, N).reshape(N, 1))
    return s.init(seed)


def _identical(a, b, L, model, tag):
    for v in (L.BETA, L.EPS, L.XSQ):
        assert np.array_equal(a.vector(v), b.vector(v)), f"{tag}: vector {v} differs"
    for sc in (L.MU, L.SIGMAE):
        assert a.scalar(sc) == b.scalar(sc), f"{tag}: scalar {sc} differs"
    if model != L.MODEL_HORSESHOE:
        assert np.array_equal(a.vector(L.COMP), b.vector(L.COMP)), tag
        assert np.array_equal(a.vector(L.PI), b.vector(L.PI)), tag


@pytest.mark.parametrize("model,B", [(0, 64), (0, 128), (0, 256), (0, 512), (1, 128), (3, 128)])
def test_2bit_chain_identical_to_f32(brr, oracle_mod, require_gpu, model, B):
    """Per-block path (B = 64), resident-Gram fused path (128) and the fused B = 512 path."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 1003, 1100
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=40)
    G = 4 if model == L.MODEL_GROUPS else 1
    gA = (np.arange(P) * G // P).astype(np.int32) if G > 1 else None
    a = _session(brr, L, model, X, Y, B, L.X_F32, G, gA)
    b = _session(brr, L, model, X, Y, B, L.X_2BIT, G, gA)
    for it in range(4):
        a.sweep(1)
        b.sweep(1)
        _identical(a, b, L, model, f"model={model} B={B} it={it}")
    okw = dict(HS) if model == L.MODEL_HORSESHOE else dict(HYP, cva=np.tile(CVA, (G, 1)), G=G)
    if gA is not None:
        okw["gAssign"] = gA
    if model == L.MODEL_GROUPS:
        okw["fixed"] = np.linspace(-1, 1, N).reshape(N, 1)
    orc = O.Oracle(model, X, Y, seed=5, order_mode=L.ORDER_BLOCKED, block_size=B, N=N, **okw)
    orc.sweep(4)
    assert _rel(b.vector(L.BETA), orc.vector(O.V_BETA)) < RTOL
    assert _rel(b.vector(L.EPS), orc.vector(O.V_EPS)) < RTOL


@pytest.mark.parametrize("B,cap", [(512, 4), (256, 2), (512, None)])
def test_2bit_wide_streamer_identical(brr, oracle_mod, require_gpu, monkeypatch, B, cap):
    """The 2-bit streaming kernel of 1,024-thread workgroups (B >= 256, four waves per SIMD) against
    the same kernel at 512 threads (BRR_STREAM_NT=512) and against the f32 chain: bit-identical over
    the burn-in's long change lists (split into parts across waves) and the steady state's short ones,
    with one and several 256-row passes per streaming workgroup."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 2000, 1536
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=60)
    if cap:
        monkeypatch.setenv("BRR_STREAM_WG", str(cap))
    wide = _session(brr, L, 0, X, Y, B, L.X_2BIT)
    assert wide.scalar(104) > 0 and wide.scalar(109) == 1024
    monkeypatch.setenv("BRR_STREAM_NT", "512")
    narrow = _session(brr, L, 0, X, Y, B, L.X_2BIT)
    assert narrow.scalar(109) == 512
    f32 = _session(brr, L, 0, X, Y, B, L.X_F32)
    for it in range(5):
        for s in (wide, narrow, f32):
            s.sweep(1)
        _identical(wide, narrow, L, 0, f"B={B} cap={cap} it={it} 1024 vs 512")
        _identical(wide, f32, L, 0, f"B={B} cap={cap} it={it} 2-bit vs f32")
    for s in (wide, narrow, f32):
        s.close()


def test_2bit_synthetic_cohort_identical(brr, require_gpu):
    """On-device synthetic genotypes written as codes decode to the f32 cohort exactly."""
    from bayesrrcpp_amd import _lib as L
    N, P = 2050, 1024
    ses = []
    for xs in (L.X_F32, L.X_2BIT):
        s = brr.Session(L.MODEL_V2, N, P, K=4, block_size=256, x_storage=xs)
        s.synthesize(20261015, 0.5, 30)
        s.set_bayesr(**HYP, cva=CVA)
        s.init(1)
        ses.append(s)
    assert np.array_equal(ses[0].vector(200), ses[1].vector(200))  # column |x| sums of the decoded X
    for it in range(3):
        for s in ses:
            s.sweep(1)
        _identical(ses[0], ses[1], L, L.MODEL_V2, f"synth it={it}")


def _bed_standardise(bed, N):
    """numpy restatement of brr_session_upload_bed (same operations, same order)."""
    M = bed.shape[0]
    codes = np.stack([(bed >> (2 * k)) & 3 for k in range(4)], axis=2).reshape(M, -1)[:, :N]
    gval = np.array([2.0, 0.0, 1.0, 0.0])
    X = np.zeros((N, M), dtype=np.float32)
    for j in range(M):
        c = codes[j]
        cnt = np.bincount(c, minlength=4)
        nobs = cnt[0] + cnt[2] + cnt[3]
        S = 2.0 * cnt[0] + cnt[2]
        Q = 4.0 * cnt[0] + cnt[2]
        mean = S / nobs if nobs > 0 else 0.0
        ss = Q - S * mean
        if nobs < 2 or not ss > 0.0:
            continue
        sd = np.sqrt(ss / (N - 1))
        lut = np.array([np.float32((gval[k] - mean) / sd) for k in range(4)], dtype=np.float32)
        lut[1] = 0.0
        X[:, j] = lut[c]
    return X


def test_upload_bed(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    rng = np.random.default_rng(17)
    N, P = 301, 384  # N not a multiple of 4: the last byte of every column is padded
    nbytes = (N + 3) // 4
    f = rng.uniform(0.05, 0.5, P)
    g = rng.binomial(2, f, size=(N, P))
    code = np.choose(g, [3, 2, 0])  # copies of allele 1: 2 -> 00, 1 -> 10, 0 -> 11
    code[rng.random((N, P)) < 0.02] = 1  # missing
    code[:, 5] = 0  # a column without variation
    pad = np.zeros((4 * nbytes, P), dtype=np.int64)
    pad[:N] = code
    bed = np.zeros((P, nbytes), dtype=np.uint8)
    for k in range(4):
        bed |= (pad[k::4].T << (2 * k)).astype(np.uint8)
    X = _bed_standardise(bed, N)
    Y = X[:, :20].astype(np.float64) @ rng.normal(0, 0.2, 20) + rng.normal(0, 1, N)
    Y = (Y - Y.mean()) / Y.std(ddof=1)
    a = _session(brr, L, L.MODEL_V2, X, Y, 128, L.X_2BIT, upload=lambda s: s.upload_bed(bed))
    b = _session(brr, L, L.MODEL_V2, X, Y, 128, L.X_F32, upload=lambda s: s.upload_bed(bed))
    c = _session(brr, L, L.MODEL_V2, X, Y, 128, L.X_F32)  # the numpy-standardised X, dense
    assert np.array_equal(a.vector(L.XSQ), c.vector(L.XSQ))
    orc = O.Oracle(O.V2, X.astype(np.float64), Y, seed=5, order_mode=L.ORDER_BLOCKED, block_size=128,
                   cva=CVA, **HYP)
    for it in range(4):
        for s in (a, b, c):
            s.sweep(1)
        orc.sweep(1)
        _identical(a, b, L, L.MODEL_V2, f"bed it={it}")
        _identical(a, c, L, L.MODEL_V2, f"bed vs dense it={it}")
        assert np.array_equal(a.vector(L.COMP), orc.vector(O.V_COMP))
        assert _rel(a.vector(L.BETA), orc.vector(O.V_BETA)) < RTOL


def test_2bit_rejects_non_genotype_columns(brr, require_gpu):
    from bayesrrcpp_amd import _lib as L
    N, P = 64, 8
    X = np.tile(np.array([0.0, 1.0, -1.0, 2.0]), N // 4)[:, None] * np.ones((1, P))
    s = brr.Session(L.MODEL_V2, N, P, K=4, x_storage=L.X_2BIT)
    s.upload_x(X)  # 3 non-zero values (+ zero) per column: encodable
    X[7, 3] = 0.5  # a fourth non-zero value in column 3
    with pytest.raises(L.BrrError, match="column 3"):
        s.upload_x(X)


@pytest.mark.parametrize("model,cap", [(0, None), (0, 30), (3, 30), (1, 7)])
def test_2bit_code_cache_midsize(brr, require_gpu, monkeypatch, model, cap):
    """The streamers' LDS cache of the last three blocks' code bytes (the change list of block s-2
    is applied from it): several row passes per workgroup, ragged last workgroup, every model.
    Identical to the f32 chain and to the 2-bit chain that re-reads the codes from HBM."""
    from bayesrrcpp_amd import _lib as L
    from oracle import oracle as O
    if cap:
        monkeypatch.setenv("BRR_STREAM_WG", str(cap))
    N, P, B = 20003, 1536, 128
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=60)
    G = 4 if model == L.MODEL_GROUPS else 1
    gA = (np.arange(P) * G // P).astype(np.int32) if G > 1 else None
    a = _session(brr, L, model, X, Y, B, L.X_F32, G, gA)
    b = _session(brr, L, model, X, Y, B, L.X_2BIT, G, gA)
    monkeypatch.setenv("BRR_NO_CODE_CACHE", "1")
    c = _session(brr, L, model, X, Y, B, L.X_2BIT, G, gA)
    assert a.scalar(104) > 0 and b.scalar(104) == a.scalar(104) == c.scalar(104)  # fused sweep
    # code cache on / off (12 row passes per workgroup at cap 7: three blocks of codes do not fit
    # in LDS, the apply re-reads them from HBM)
    assert b.scalar(105) == (0 if cap == 7 else 1) and c.scalar(105) == 0
    for it in range(3):
        for s in (a, b, c):
            s.sweep(1)
        _identical(a, b, L, model, f"cache model={model} cap={cap} it={it}")
        _identical(a, c, L, model, f"no cache model={model} cap={cap} it={it}")


@pytest.mark.parametrize("model", [1, 3])
def test_f32_class_code_cache_identical(brr, oracle_mod, require_gpu, model, monkeypatch):
    """f32 storage with every column class-coded (BLOCKED order, B = 128, BRR_F32_CODE_CACHE=1; the
    Horseshoe's and, since round 5, the Groups model's default): the streamers keep the streamed blocks' class codes in LDS and apply the
    change lists from them (k_sweep_stream<2>) instead of re-reading X.  Same values in the same
    order: the chain equals the f32 chain without the cache (BRR_F32_CODE_CACHE=0) bit for bit, and
    the oracle within the parity tolerance."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    N, P = 1003, 1100
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5, n_causal=40)
    G = 4 if model == L.MODEL_GROUPS else 1
    gA = (np.arange(P) * G // P).astype(np.int32) if G > 1 else None
    monkeypatch.setenv("BRR_F32_CODE_CACHE", "1")
    a = _session(brr, L, model, X, Y, 128, L.X_F32, G, gA)
    assert a.scalar(105) == 1 and a.scalar(104) > 0, "f32 code cache not in use"
    monkeypatch.setenv("BRR_F32_CODE_CACHE", "0")
    b = _session(brr, L, model, X, Y, 128, L.X_F32, G, gA)
    assert b.scalar(105) == 0
    monkeypatch.delenv("BRR_F32_CODE_CACHE")
    dflt = _session(brr, L, model, X, Y, 128, L.X_F32, G, gA)
    assert dflt.scalar(105) == 1, "the cache is the default of the Horseshoe and Groups models"
    del dflt
    for it in range(4):
        a.sweep(1)
        b.sweep(1)
        _identical(a, b, L, model, f"model={model} it={it}")
