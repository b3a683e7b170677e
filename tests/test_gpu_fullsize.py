"""Parity at BASELINE.json's full single-GPU size (C2: N = 100,000 x P = 500,000, 200 GB of f32 X
on the device) through size-independent properties; the oracle cannot run this size in seconds.

* residual invariant: after k sweeps eps = Y - mu - X beta (BayesRv2.cpp:168,191,243), with Y the
  residual right after init (beta = 0, mu = 0) and X beta formed on the host from the oracle's
  bit-identical regeneration of the synthetic columns with non-zero beta;
* storage invariance: the chain under 2-bit genotype storage is bit-identical to the dense f32
  chain (same decoded values, same kernels' order of operations).
"""
import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu

N, P, DS = 100_000, 500_000, 20261015


def _c2_session(brr, L, x_storage):
    s = brr.Session(L.MODEL_V2, N, P, K=4, x_storage=x_storage)
    s.synthesize(DS, 0.5, -1)
    s.set_bayesr(**HYP, cva=CVA)
    return s.init(1)


def test_c2_residual_invariant(brr, oracle_mod, require_gpu):
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    with _c2_session(brr, L, L.X_F32) as s:  # the 200 GB of X go at the block's end, also on a failure
        Y = s.vector(L.EPS).copy()  # eps after init = Y - 0 - X 0
        s.sweep(10)
        beta, eps, mu = s.vector(L.BETA), s.vector(L.EPS), s.scalar(L.MU)
    nz = np.nonzero(beta)[0]
    assert 0 < nz.size < 20_000, nz.size
    xb = np.zeros(N)
    for j in nz:  # the synthetic column j, regenerated bit for bit on the host
        xb += O.synth_x(DS, N, 1, int(j))[:, 0] * beta[j]
    ref = Y - mu - xb
    err = np.max(np.abs(eps - ref)) / np.max(np.abs(ref))
    assert err < 1e-9, err


def test_c2_2bit_chain_identical(brr, require_gpu, monkeypatch):
    from bayesrrcpp_amd import _lib as L
    monkeypatch.setenv("BRR_LAG", "2")  # both storages on the f32 default pipeline (lag 2)
    traj = []
    with _c2_session(brr, L, L.X_F32) as s:  # frees the 200 GB of X before the next session
        for _ in range(4):
            s.sweep(1)
            traj.append((s.vector(L.BETA), s.vector(L.COMP), s.vector(L.EPS), s.scalar(L.SIGMAE), s.scalar(L.MU)))
    with _c2_session(brr, L, L.X_2BIT) as s:
        for it, (b, c, e, se, mu) in enumerate(traj):
            s.sweep(1)
            assert np.array_equal(s.vector(L.BETA), b), f"beta differs at sweep {it}"
            assert np.array_equal(s.vector(L.COMP), c), f"comp differs at sweep {it}"
            assert np.array_equal(s.vector(L.EPS), e), f"eps differs at sweep {it}"
            assert s.scalar(L.SIGMAE) == se and s.scalar(L.MU) == mu, f"scalars differ at sweep {it}"


def test_linear_predictor_small(brr, oracle_mod, require_gpu):
    """The validation product X beta + F alpha (used by the full-size invariants below) against numpy."""
    from bayesrrcpp_amd import _lib as L
    O = oracle_mod
    n, p, G = 777, 300, 3
    X, Y, _ = O.synth_cohort(DS, n, p, h2=0.5, n_causal=20)
    rng = np.random.default_rng(5)
    fixed = rng.normal(size=(n, 2))
    for xs in (L.X_F32, L.X_2BIT):
        s = brr.Session(L.MODEL_GROUPS, n, p, K=4, groups=G, F=2, x_storage=xs)
        s.upload_x(X).set_y(Y).set_fixed(fixed)
        s.set_bayesr(**HYP, cva=np.tile(CVA, (G, 1)), gAssign=(np.arange(p) % G).astype(np.int32))
        s.init(1)
        beta = np.where(rng.random(p) < 0.4, rng.normal(size=p), 0.0)
        alpha = rng.normal(size=2)
        s.set_vector(L.BETA, beta)
        s.set_vector(L.ALPHA, alpha)
        ref = X.astype(np.float64) @ beta + fixed @ alpha
        got = s.linear_predictor()
        assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-12
        s.close()


def _invariant(s, L, Y):
    eps, mu = s.vector(L.EPS), s.scalar(L.MU)
    ref = Y - mu - s.linear_predictor()
    return float(np.max(np.abs(eps - ref)) / np.max(np.abs(ref)))


def test_c3_residual_invariant(brr, require_gpu):
    """C3 (BayesRSamplerV2Groups, 22 groups, gAssign = floor(22 j / P), one all-zero fixed column,
    vignettes/BayesRR.Rmd:166) at full size: after 10 sweeps eps = Y - mu - X beta - F alpha
    (BayesRv2Groups.cpp:203,212-214,220-224,243,295) within 1e-9; sigmaGG finite and positive, every
    group's pi a probability vector, v counts add up to P."""
    from bayesrrcpp_amd import _lib as L
    G = 22
    with brr.Session(L.MODEL_GROUPS, N, P, K=4, groups=G, F=1) as s:
        s.synthesize(DS, 0.5, -1)
        s.set_bayesr(**HYP, cva=np.tile(CVA, (G, 1)), gAssign=(np.arange(P) * G // P).astype(np.int32))
        s.set_fixed(np.zeros((N, 1)))
        s.init(1)
        Y = s.vector(L.EPS).copy()  # eps after init = Y - mu with mu = 0 (BayesRv2Groups.cpp:203)
        s.sweep(10)
        err = _invariant(s, L, Y)
        sgg, pi, vc = s.vector(L.SIGMAGG), s.vector(L.PI).reshape(G, 4), s.vector(L.VCOUNT)
        nz = int(np.count_nonzero(s.vector(L.BETA)))
    assert err < 1e-9, err
    assert np.all(np.isfinite(sgg)) and np.all(sgg > 0)
    assert np.all(pi >= 0) and np.allclose(pi.sum(1), 1.0, rtol=1e-12)
    assert vc.sum() == P and 0 < nz <= P


def test_c4_residual_invariant(brr, require_gpu):
    """C4 (HorseshoeR, A = (1/sqrt N) 1500 / (P - 1500), HorseshoeR.cpp:315-323) at full size: after
    10 sweeps eps = Y - mu - X beta (HorseshoeR.cpp:186,210-212,224,238) within 1e-9; every marker moved
    (Horseshoe resamples all); lambda, tau, c2, eta finite and positive (HorseshoeR.cpp:242-253)."""
    from bayesrrcpp_amd import _lib as L
    with brr.Session(L.MODEL_HORSESHOE, N, P, K=1) as s:
        s.synthesize(DS, 0.5, -1)
        s.set_horseshoe(A=(1 / N ** 0.5) * 1500 / (P - 1500), v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0, c2=1.0,
                        vC=10.0, sC=10.0)
        s.init(1)
        Y = s.vector(L.EPS).copy()  # eps after init = Y - mu - X 0 (HorseshoeR.cpp:186)
        s.sweep(10)
        err = _invariant(s, L, Y)
        lam, beta = s.vector(L.LAMBDA), s.vector(L.BETA)
        sc = [s.scalar(w) for w in (L.TAU, L.C2, L.ETA, L.SIGMAE)]
    assert err < 1e-9, err
    assert np.count_nonzero(beta) == P
    assert np.all(np.isfinite(lam)) and np.all(lam > 0)
    assert all(np.isfinite(v) and v > 0 for v in sc), sc
