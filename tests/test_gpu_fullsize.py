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
    s = _c2_session(brr, L, L.X_F32)
    Y = s.vector(L.EPS).copy()  # eps after init = Y - 0 - X 0
    s.sweep(10)
    beta, eps, mu = s.vector(L.BETA), s.vector(L.EPS), s.scalar(L.MU)
    s.close()  # frees the 200 GB of X before the next session
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
    s = _c2_session(brr, L, L.X_F32)
    for _ in range(4):
        s.sweep(1)
        traj.append((s.vector(L.BETA), s.vector(L.COMP), s.vector(L.EPS), s.scalar(L.SIGMAE), s.scalar(L.MU)))
    s.close()  # frees the 200 GB of X before the next session
    s = _c2_session(brr, L, L.X_2BIT)
    for it, (b, c, e, se, mu) in enumerate(traj):
        s.sweep(1)
        assert np.array_equal(s.vector(L.BETA), b), f"beta differs at sweep {it}"
        assert np.array_equal(s.vector(L.COMP), c), f"comp differs at sweep {it}"
        assert np.array_equal(s.vector(L.EPS), e), f"eps differs at sweep {it}"
        assert s.scalar(L.SIGMAE) == se and s.scalar(L.MU) == mu, f"scalars differ at sweep {it}"
