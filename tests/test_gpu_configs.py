"""GPU tests at the two BASELINE.json configurations the other GPU suites do not run at their
stated shape:

* C1 (configs[0]): the drop-in one-shot brr_BayesRSamplerV2 at exactly N = 2,000 x P = 10,000
  with the vignette's 3-component mixture (vignettes/BayesRR.Rmd:93-100), through the C ABI, against
  the oracle's reference-faithful one-shot CSV (src/BayesRv2.cpp:171-272).  Block size is left to
  the library, so this also covers the automatic B = 128 path below N = 32,768.
* C5 (configs[4]): one rank's real workload of the 8-way column-sharded cohort -- N = 500,000 rows x
  P_local = 125,000 of M_total = 1,000,000 markers (shard 0 of 8), f32, 250 GB of X on the device --
  through the split protocol (sweep_local -> exchange -> sweep_finish) with the other seven ranks'
  residual deltas zero.  The oracle cannot run this size; the checks are size-independent:
  the exchange buffer equals eps_local_end - eps_start bit for bit after every local sweep, and
  after 10 sweeps eps = Y - mu - X_local beta_local (src/BayesRv2.cpp:168,191,243) within 1e-9.
"""
import numpy as np
import pytest

from conftest import CVA, HYP

pytestmark = pytest.mark.gpu


def test_c1_oneshot_at_stated_shape(brr, oracle_mod, require_gpu, tmp_path):
    O = oracle_mod
    N, P = 2_000, 10_000
    X, Y, _ = O.synth_cohort(20261015, N, P, h2=0.5)  # min(1000, P/10) causal effects
    p_gpu, p_orc = str(tmp_path / "gpu.csv"), str(tmp_path / "orc.csv")
    MAXIT, BURN, THIN = 40, 10, 10
    brr.BayesRSamplerV2(p_gpu, 1, MAXIT, BURN, THIN, X, Y, HYP["sigma0"], HYP["v0E"], HYP["s02E"],
                        HYP["v0G"], HYP["s02G"], CVA, log=lambda m: None)  # raises on a device error
    O.run_csv(p_orc, O.V2, X, Y, MAXIT, BURN, THIN, cva=CVA, seed=1, order_mode=0, **HYP)
    g = open(p_gpu).read().splitlines()
    o = open(p_orc).read().splitlines()
    assert g[0] == o[0]  # header (src/BayesRv2.cpp:16-37)
    kept = [i for i in range(BURN, MAXIT) if i % THIN == 0]
    assert len(g) == len(o) == 1 + len(kept)
    for lg, lo in zip(g[1:], o[1:]):
        a = np.array([float(v) for v in lg.split(", ")])
        b = np.array([float(v) for v in lo.split(", ")])
        assert a.shape == b.shape == (2 * P + N + 4,)
        comp = slice(2 + P + 2, 2 + 2 * P + 2)
        assert np.array_equal(a[comp], b[comp])  # component assignments identical
        assert np.allclose(a, b, rtol=2e-5, atol=1e-9)  # 6 significant digits on both sides


def test_c5_rank_workload(brr, require_gpu):
    from bayesrrcpp_amd import _lib as L
    N, P_loc, M_tot, R = 500_000, 125_000, 1_000_000, 8
    # the 250 GB of X go at the with-block's end, also when an assertion inside fails (a retained
    # session made the next 200 GB create fail, gpurun_out/r04rn_tests.log)
    with brr.Session(L.MODEL_V2, N, P_loc, K=4, M_total=M_tot, col_offset=0, shard_rank=0, shard_count=R) as s:
        assert s.block_size == 512
        s.synthesize(20261015, 0.5, -1)
        # Y from this shard's genetic values (the other shards' parts zero), standardised
        s.synth_y(s.synth_partial_y(), 20261015, 0.5)
        s.set_bayesr(**HYP, cva=CVA)
        s.init(1)
        Y = s.vector(L.EPS).copy()  # eps after init = Y - 0 - X 0
        s.exchange_buffers()
        E = s.exchanges_per_sweep
        assert E == 8  # automatic
        for it in range(10):
            for e in range(E):
                eps0, mu0 = s.vector(L.EPS), s.scalar(L.MU)
                s.sweep_local()
                mu1 = s.scalar(L.MU)
                # the sweep start's shift (src/BayesRv2.cpp:177-179); later segments start from eps as is
                eps_start = (eps0 + mu0) - mu1 if e == 0 else eps0
                dE, stats = s.exchange_get()
                eps_loc = s.vector(L.EPS)
                assert np.array_equal(dE, eps_loc - eps_start), f"exchange buffer != eps_local - eps_start at {it}.{e}"
                if e < E - 1:
                    assert not np.any(stats), "statistics follow the last segment only"
                # the seven other ranks contribute zero deltas and zero statistics: the sum is this rank's
                s.exchange_set(dE, stats)
                s.sweep_finish()
            assert s.iteration == it + 1
        beta, eps, mu = s.vector(L.BETA), s.vector(L.EPS), s.scalar(L.MU)
        xb = s.linear_predictor()
        sigmaE = s.scalar(L.SIGMAE)
    nz = int(np.count_nonzero(beta))
    assert 0 < nz < P_loc
    ref = Y - mu - xb
    err = float(np.max(np.abs(eps - ref)) / np.max(np.abs(ref)))
    assert err < 1e-9, err
    assert np.isfinite(sigmaE) and sigmaE > 0
