"""Gram blocks (src/BayesRv2.cpp:170 xsq; the blocked chain's G = X_b^T X_b and cross-Gram blocks).

For class-coded columns (at most 4 distinct values: genotypes, in either storage) the device forms
every entry on the i8 matrix cores from class-pair counts and sums them exactly (k_gram_int): the
result must be the CORRECTLY ROUNDED dot product of the f32 columns, i.e. equal, bit for bit, to
math.fsum of the exact f64 products -- in both storages, for 2, 3 and 4 classes per column, ragged N
and a short last block.  Columns that are not class-coded take the FP64 matrix-core kernel, whose
sums are within a few ulps of the exact value.
"""
import math
import os

import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu

GRAM, XGRAM, GRAM_NP = 202, 203, 107


def _exact_block(X, cols_a, cols_b):
    Xa = X[:, cols_a].astype(np.float64)
    Xb = X[:, cols_b].astype(np.float64)
    out = np.zeros((len(cols_a), len(cols_b)))
    for i in range(len(cols_a)):
        prod = Xa[:, i:i + 1] * Xb  # exact (f32 x f32 in f64)
        for j in range(len(cols_b)):
            out[i, j] = math.fsum(prod[:, j])
    return out


def _session(brr, L, X, Y, B, storage):
    N, P = X.shape
    s = brr.Session(L.MODEL_V2, N, P, K=len(CVA) + 1, block_size=B, x_storage=storage)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=CVA)
    return s.init(3)


def _check(s, X, B, nblocks_checked=2):
    N, P = X.shape
    nb = (P + B - 1) // B
    G = s.vector(GRAM).reshape(nb, B, B)
    XG = s.vector(XGRAM).reshape(nb, B, B)
    for b in list(range(min(nblocks_checked, nb))) + [nb - 1]:
        ca = np.arange(b * B, min(P, (b + 1) * B))
        b2 = (b + 1) % nb
        cb = np.arange(b2 * B, min(P, (b2 + 1) * B))
        yield b, G[b][: len(ca), : len(ca)], _exact_block(X, ca, ca), XG[b][: len(ca), : len(cb)], _exact_block(X, ca, cb)


def _genotypes(rng, N, P, nclass, zero_class=False):
    """Standardised dosages (f32) with nclass distinct values per column."""
    f = rng.uniform(0.05, 0.5, P)
    g = (rng.random((N, P)) < f).astype(np.int64) + (rng.random((N, P)) < f)
    if nclass == 2:
        g = np.minimum(g, 1)
    X = ((g - g.mean(0)) / np.maximum(g.std(0, ddof=1), 1e-3)).astype(np.float32)
    if zero_class:  # a fourth value: missing genotypes imputed to 0
        X[rng.random((N, P)) < 0.03] = 0.0
    return X


@pytest.mark.parametrize("tile", ["128", "64"])
@pytest.mark.parametrize("storage", ["f32", "2bit"])
@pytest.mark.parametrize("nclass,zero,N,B", [(3, False, 1003, 128), (2, False, 517, 64), (3, True, 1000, 128),
                                             (3, False, 300, 256), (2, False, 517, 128), (3, False, 201, 512)])
def test_integer_gram_is_correctly_rounded(brr, require_gpu, monkeypatch, tile, storage, nclass, zero, N, B):
    """tile 128: k_gram_blk (whole 128-column tiles, at most 2 explicit planes, B a multiple of 128; the
    default there), 64: k_gram_int (BRR_GRAM_TILE64=1; every other case) -- both exact."""
    from bayesrrcpp_amd import _lib as L
    if tile == "64":
        monkeypatch.setenv("BRR_GRAM_TILE64", "1")
    rng = np.random.default_rng(nclass * 100 + N)
    P = 3 * B - 37  # a short last block
    X = _genotypes(rng, N, P, nclass, zero)
    Y = rng.standard_normal(N)
    s = _session(brr, L, X, Y, B, L.X_2BIT if storage == "2bit" else L.X_F32)
    want_np = nclass - 1 + (1 if zero else 0)
    assert int(s.scalar(GRAM_NP)) == want_np, "k_gram_int planes"
    for b, g, ge, xg, xge in _check(s, X, B):
        assert np.array_equal(g, ge), f"gram block {b}: max |diff| {np.max(np.abs(g - ge))}"
        assert np.array_equal(xg, xge), f"cross-Gram block {b}: max |diff| {np.max(np.abs(xg - xge))}"
    xsq = s.vector(L.XSQ)
    assert np.array_equal(xsq, np.array([math.fsum(X[:, j].astype(np.float64) ** 2) for j in range(P)]))
    s.close()


def test_unclassed_columns_use_fp64_kernel(brr, require_gpu):
    from bayesrrcpp_amd import _lib as L
    rng = np.random.default_rng(7)
    N, B = 700, 128
    X = rng.standard_normal((N, 2 * B)).astype(np.float32)
    s = _session(brr, L, X, rng.standard_normal(N), B, L.X_F32)
    assert int(s.scalar(GRAM_NP)) == 0
    for b, g, ge, xg, xge in _check(s, X, B):
        assert np.max(np.abs(g - ge)) <= 1e-13 * np.max(np.abs(ge))
        assert np.max(np.abs(xg - xge)) <= 1e-13 * np.max(np.abs(ge))
    s.close()


def test_fp64_and_integer_kernels_agree(brr, require_gpu, monkeypatch):
    """The same genotype cohort through both kernels: FP64 sums within a few ulps of the exact ones."""
    from bayesrrcpp_amd import _lib as L
    rng = np.random.default_rng(11)
    N, B = 2048, 128
    X = _genotypes(rng, N, 3 * B, 3)
    Y = rng.standard_normal(N)
    a = _session(brr, L, X, Y, B, L.X_F32)
    monkeypatch.setenv("BRR_GRAM_F64", "1")
    b = _session(brr, L, X, Y, B, L.X_F32)
    assert int(a.scalar(GRAM_NP)) == 2 and int(b.scalar(GRAM_NP)) == 0
    ga, gb = a.vector(GRAM), b.vector(GRAM)
    assert np.max(np.abs(ga - gb)) <= 1e-12 * np.max(np.abs(ga))
    a.close()
    b.close()


def _ref_session(brr, L, X, Y, B, storage):
    N, P = X.shape
    s = brr.Session(L.MODEL_V2, N, P, K=len(CVA) + 1, block_size=B, x_storage=storage, order_mode=L.ORDER_REFERENCE)
    s.upload_x(X).set_y(Y).set_bayesr(**HYP, cva=CVA)
    return s.init(3)


@pytest.mark.parametrize("storage", ["f32", "2bit"])
@pytest.mark.parametrize("nclass,N,B", [(3, 1003, 128), (2, 517, 128), (3, 300, 256)])
def test_reference_order_fp4_gram_is_correctly_rounded(brr, require_gpu, storage, nclass, N, B):
    """REFERENCE order reads the column-major class codes straight into fp4 planes (k_gram_fp4: planes c and
    c^2 on the block-scaled matrix cores, class-pair counts recovered exactly): every block of the sweep's
    layout (member order, vector ORDER) must again be the correctly rounded dot products, after init and
    after a sweep's re-layout."""
    from bayesrrcpp_amd import _lib as L
    rng = np.random.default_rng(nclass * 1000 + N)
    P = 3 * B - 37
    X = _genotypes(rng, N, P, nclass)
    Y = rng.standard_normal(N)
    s = _ref_session(brr, L, X, Y, B, L.X_2BIT if storage == "2bit" else L.X_F32)
    assert int(s.scalar(GRAM_NP)) == nclass - 1
    nb = (P + B - 1) // B
    for stage in range(2):
        if stage:
            s.sweep(1)
        order = s.vector(L.ORDER).astype(np.int64)
        G = s.vector(GRAM).reshape(nb, B, B)
        XG = s.vector(XGRAM).reshape(nb, B, B)
        blocks = [order[b * B:(b + 1) * B] for b in range(nb)]
        for b in (0, nb - 1):
            ca, cb = blocks[b], blocks[(b + 1) % nb]
            ge = _exact_block(X, ca, ca)
            assert np.array_equal(G[b][: len(ca), : len(ca)], ge), f"stage {stage} gram block {b}"
            xge = _exact_block(X, ca, cb)
            assert np.array_equal(XG[b][: len(ca), : len(cb)], xge), f"stage {stage} cross-Gram block {b}"
    s.close()


def test_reference_order_fp4_and_i8_chains_identical(brr, require_gpu, monkeypatch):
    """The fp4 Gram kernel (default in REFERENCE order) and the i8 kernels (BRR_GRAM_FP4=0, with the per-sweep
    layout encoding) give the same exact Gram blocks, so the chains are bit-identical."""
    from bayesrrcpp_amd import _lib as L
    rng = np.random.default_rng(5)
    N, B = 1500, 128
    X = _genotypes(rng, N, 5 * B - 9, 3)
    Y = rng.standard_normal(N)
    out = []
    for fp4 in ("1", "0"):
        monkeypatch.setenv("BRR_GRAM_FP4", fp4)
        s = _ref_session(brr, L, X, Y, B, L.X_F32)
        s.sweep(3)
        out.append((s.vector(L.BETA), s.vector(L.EPS), s.vector(GRAM)))
        s.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
