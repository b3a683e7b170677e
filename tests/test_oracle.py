"""CPU tests of the parity oracle: known-answer tests for its pinned pieces, distribution
moments, reference invariants and statistical recovery (the reference itself has no tests,
SURVEY.md section 4; oracle parity vs reference outputs is unpinned, see oracle/brr_oracle.h)."""
import ctypes
import ctypes.util
import os
import subprocess

import numpy as np
import pytest

from conftest import CVA, HYP


# ---------------------------------------------------------------- Philox4x32-10 KATs
# Random123 kat_vectors (philox4x32 10): counter, key -> output
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_kat(oracle_mod, ctr, key, out):
    assert oracle_mod.philox(ctr, key) == out


def test_philox_matches_rocrand_engine(oracle_mod, tmp_path):
    """The device side draws through rocRAND's Philox4x32-10 engine; compile its (host-capable)
    block function and compare with the oracle's independent implementation."""
    src = tmp_path / "r.cpp"
    src.write_text(r'''
#include <cstdio>
#include "bayesrrcpp_amd/csrc/brr_rng.hpp"
int main() {
  for (unsigned i = 0; i < 8; ++i) {
    uint4 w = brr::philox(0x123456789ULL + i, i * 7u, 3u + i, 1000u * i, 17u);
    printf("%u %u %u %u\n", w.x, w.y, w.z, w.w);
  }
}''')
    exe = tmp_path / "r"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", f"-I{repo}",
           str(src), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"hipcc host build unavailable: {r.stderr[-200:]}")
    lines = subprocess.run([str(exe)], capture_output=True, text=True).stdout.split("\n")
    for i in range(8):
        seed = 0x123456789 + i
        ref = oracle_mod.philox([i * 7, 3 + i, 1000 * i, 17], [seed & 0xFFFFFFFF, seed >> 32])
        assert [int(v) for v in lines[i].split()] == ref


# ---------------------------------------------------------------- glibc rand / shuffle
def test_glibc_rand_matches_libc(oracle_mod):
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    for seed in (1, 2, 12345):
        libc.srand(seed)
        want = [libc.rand() for _ in range(2000)]
        got = oracle_mod.glibc_rand(seed, 2000).tolist()
        assert got == want


def test_random_shuffle_known_answer(oracle_mod):
    """std::random_shuffle of 0..9 from a fresh process (verified against libstdc++ 11 here):
    4 3 7 8 0 5 2 1 6 9, then 0 5 7 8 4 3 9 2 1 6 (the array persists across sweeps)."""
    r = oracle_mod.glibc_rand(1, 18)
    a = list(range(10))
    for sweep_expect in ([4, 3, 7, 8, 0, 5, 2, 1, 6, 9], [0, 5, 7, 8, 4, 3, 9, 2, 1, 6]):
        for i in range(1, 10):
            j = r[0] % (i + 1)
            r = r[1:]
            a[i], a[j] = a[j], a[i]
        assert a == sweep_expect


def test_reference_order_in_sampler(oracle_mod):
    O = oracle_mod
    X = np.asfortranarray(np.random.default_rng(0).normal(size=(20, 10)))
    Y = np.random.default_rng(1).normal(size=20)
    o = O.Oracle(O.V2, X, Y, cva=CVA, order_mode=O.ORDER_REFERENCE, **HYP)
    o.sweep(1)
    assert o.vector(O.V_ORDER).astype(int).tolist() == [4, 3, 7, 8, 0, 5, 2, 1, 6, 9]
    o.sweep(1)
    assert o.vector(O.V_ORDER).astype(int).tolist() == [0, 5, 7, 8, 4, 3, 9, 2, 1, 6]


def test_blocked_order_is_block_restricted_permutation(oracle_mod):
    P, B = 1000, 128
    for it in range(3):
        o = oracle_mod.blocked_order(7, it, P, B)
        assert sorted(o.tolist()) == list(range(P))
        # every run of visits stays inside one fixed block
        pos = 0
        while pos < P:
            blk = o[pos] // B
            size = min(B, P - blk * B)
            assert set((o[pos:pos + size] // B).tolist()) == {blk}
            pos += size
    # block sequence: a rotation of the block cycle, forwards or backwards (consecutive blocks
    # are cycle neighbours, so their cross-Gram blocks can be precomputed)
    nb = (P + B - 1) // B
    dirs = set()
    for it in range(16):
        o = oracle_mod.blocked_order(7, it, P, B)
        starts = np.concatenate([[0], np.cumsum([min(B, P - b * B) for b in range(nb)])])
        seq, pos = [], 0
        while pos < P:
            blk = int(o[pos] // B)
            seq.append(blk)
            pos += min(B, P - blk * B)
        d = (seq[1] - seq[0]) % nb
        assert d in (1, nb - 1)
        dirs.add(d)
        assert all((seq[i + 1] - seq[i]) % nb == d for i in range(nb - 1))
    assert dirs == {1, nb - 1}
    assert not np.array_equal(oracle_mod.blocked_order(7, 0, P, B), oracle_mod.blocked_order(7, 1, P, B))


# ---------------------------------------------------------------- distributions
def test_uniform_and_normal_moments(oracle_mod):
    L = oracle_mod.lib()
    u = np.array([L.orc_uniform(5, 1, i, 0, 0) for i in range(20000)])
    z = np.array([L.orc_normal(5, 1, i, 0, 1) for i in range(20000)])
    assert 0 < u.min() and u.max() < 1
    assert abs(u.mean() - 0.5) < 0.01 and abs(u.var() - 1 / 12) < 0.003
    assert abs(z.mean()) < 0.03 and abs(z.var() - 1) < 0.04


@pytest.mark.parametrize("shape", [0.3, 1.0, 2.5, 50.0, 5e4])
def test_gamma_moments(oracle_mod, shape):
    L = oracle_mod.lib()
    g = np.array([L.orc_gamma(9, shape, 3, i, 0) for i in range(8000)])
    assert np.all(g > 0)
    assert abs(g.mean() / shape - 1) < 4 * np.sqrt(1 / shape / 8000) + 1e-3
    assert abs(g.var() / shape - 1) < 0.12


def test_synthetic_x_standardised(oracle_mod):
    X = oracle_mod.synth_x(20261015, 500, 40)
    assert np.allclose(X.mean(0), 0, atol=1e-6)
    assert np.allclose((X ** 2).sum(0), 499, rtol=1e-5)
    # values are f32-representable (the device stores X as f32)
    assert np.array_equal(X.astype(np.float32).astype(np.float64), X)


# ---------------------------------------------------------------- sampler invariants
@pytest.mark.parametrize("order", [0, 1, 2])
def test_v2_residual_invariant_and_recovery(oracle_mod, order):
    O = oracle_mod
    X, Y, b = O.synth_cohort(3, 600, 300, h2=0.5, n_causal=15)
    o = O.Oracle(O.V2, X, Y, cva=CVA, seed=2, order_mode=order, block_size=64, **HYP)
    bs = []
    for i in range(120):
        o.sweep(1)
        if i >= 40:
            bs.append(o.vector(O.V_BETA))
    eps, beta, mu = o.vector(O.V_EPS), o.vector(O.V_BETA), o.scalar(O.S_MU)
    # epsilon = Y - mu - X beta holds throughout (BayesRv2.cpp:177-179, :243)
    assert np.max(np.abs(eps - (Y - mu - X @ beta))) < 1e-10
    assert np.corrcoef(np.mean(bs, 0), b)[0, 1] > 0.8
    comp = o.vector(O.V_COMP)
    assert np.all((comp == 0) == (beta == 0))
    pi = o.vector(O.V_PI)
    assert abs(pi.sum() - 1) < 1e-12


def test_groups_and_fixed_effects_recovery(oracle_mod):
    O = oracle_mod
    N, P, G = 500, 200, 4
    X, Y, b = O.synth_cohort(4, N, P, h2=0.5, n_causal=10)
    rng = np.random.default_rng(0)
    fixed = rng.normal(size=(N, 2))
    alpha_true = np.array([0.5, -0.3])
    Y2 = Y + fixed @ alpha_true
    gA = (np.arange(P) * G // P).astype(np.int32)
    o = O.Oracle(O.GROUPS, X, Y2, cva=np.tile(CVA, (G, 1)), G=G, gAssign=gA, fixed=fixed, seed=5, **HYP)
    al = []
    for i in range(150):
        o.sweep(1)
        if i >= 50:
            al.append(o.vector(O.V_ALPHA))
    assert np.allclose(np.mean(al, 0), alpha_true, atol=0.08)
    # BayesRv2Groups.cpp:283 counts per group sum to the selected markers
    v = o.vector(O.V_VCOUNT).reshape(G, -1)
    assert v.sum() <= P and v.sum() >= P - 5
    eps, beta, mu = o.vector(O.V_EPS), o.vector(O.V_BETA), o.scalar(O.S_MU)
    assert np.max(np.abs(eps - (Y2 - mu - X @ beta - fixed @ o.vector(O.V_ALPHA)))) < 1e-10


def test_restart_continues_chain(oracle_mod):
    O = oracle_mod
    N, P, G = 300, 150, 2
    X, Y, _ = O.synth_cohort(6, N, P, n_causal=10)
    gA = (np.arange(P) % G).astype(np.int32)
    a = O.Oracle(O.GROUPS, X, Y, cva=np.tile(CVA, (G, 1)), G=G, gAssign=gA, seed=1, **HYP)
    a.sweep(20)
    r = O.Oracle(O.RESTART, X, None, cva=np.tile(CVA, (G, 1)), G=G, gAssign=gA, seed=2, N=N,
                 mu0=a.scalar(O.S_MU), beta0=a.vector(O.V_BETA), sigmaE0=a.scalar(O.S_SIGMAE),
                 sigmaGG0=a.vector(O.V_SIGMAGG), eps0=a.vector(O.V_EPS), comp0=a.vector(O.V_COMP), **HYP)
    # pi re-drawn from the components (BRv2Grstart.cpp:157-165) is a probability vector per group
    pi = r.vector(O.V_PI).reshape(G, -1)
    assert np.allclose(pi.sum(1), 1)
    r.sweep(5)
    eps, beta, mu = r.vector(O.V_EPS), r.vector(O.V_BETA), r.scalar(O.S_MU)
    assert np.max(np.abs(eps - (Y - mu - X @ beta))) < 1e-10


def test_horseshoe_invariants(oracle_mod):
    O = oracle_mod
    N, P = 400, 300
    X, Y, b = O.synth_cohort(8, N, P, n_causal=10)
    A = (1 / np.sqrt(N)) * 150 / (P - 150)
    o = O.Oracle(O.HORSESHOE, X, Y, A=A, v0E=1e-3, s02E=1e-3, vL=1, vT=1, c2=1, vC=10, sC=10, seed=3)
    bs = []
    for i in range(150):
        o.sweep(1)
        if i >= 50:
            bs.append(o.vector(O.V_BETA))
    assert o.scalar(O.S_TAU) > 0 and o.scalar(O.S_C2) > 0 and o.scalar(O.S_ETA) > 0
    assert np.all(o.vector(O.V_LAMBDA) > 0)
    assert np.corrcoef(np.mean(bs, 0), b)[0, 1] > 0.7
    eps, beta, mu = o.vector(O.V_EPS), o.vector(O.V_BETA), o.scalar(O.S_MU)
    assert np.max(np.abs(eps - (Y - mu - X @ beta))) < 1e-10


def test_sharded_emulation_single_shard_identical(oracle_mod):
    O = oracle_mod
    X, Y, _ = O.synth_cohort(2, 200, 256, n_causal=10)
    a = O.Oracle(O.V2, X, Y, cva=CVA, seed=4, block_size=64, n_shards=1, **HYP)
    b = O.Oracle(O.V2, X, Y, cva=CVA, seed=4, block_size=64, n_shards=2, **HYP)
    a.sweep(3)
    b.sweep(3)
    # shards see stale residuals: not the same chain, but same visit set and valid state
    assert sorted(b.vector(O.V_ORDER).tolist()) == list(range(256))
    eps, beta, mu = b.vector(O.V_EPS), b.vector(O.V_BETA), b.scalar(O.S_MU)
    assert np.max(np.abs(eps - (Y - mu - X @ beta))) < 1e-10


def test_guard_fallthrough_keeps_beta(oracle_mod):
    """700-guard (BayesRv2.cpp:216-242): a huge signal zeroes the dominant component's
    probability; when nothing is selected the marker keeps its beta and is not counted."""
    O = oracle_mod
    N = 400
    rng = np.random.default_rng(0)
    x = rng.normal(size=N)
    x = (x - x.mean()) / x.std(ddof=1)
    X = np.asfortranarray(np.c_[x, rng.normal(size=N)])
    Y = 40.0 * x + rng.normal(size=N) * 0.01
    o = O.Oracle(O.V2, X, Y, cva=[1e-4, 1e-3, 1e-2], seed=1, order_mode=O.ORDER_IDENTITY, **HYP)
    o.sweep(3)
    v = o.vector(O.V_VCOUNT)
    assert v.sum() <= 2


def test_csv_format(oracle_mod, tmp_path):
    O = oracle_mod
    X, Y, _ = O.synth_cohort(1, 30, 12, n_causal=3)
    p = str(tmp_path / "o.csv")
    assert O.run_csv(p, O.V2, X, Y, 12, 4, 3, cva=CVA, **HYP) == 0
    lines = open(p).read().splitlines()
    hdr = lines[0].split(",")
    assert hdr[:3] == ["iteration", "mu", "beta[1]"] and hdr[-1] == "epsilon[30]"
    assert len(hdr) == 2 * 12 + 30 + 4
    kept = [i for i in range(4, 12) if i % 3 == 0]
    assert [int(float(l.split(", ")[0])) for l in lines[1:]] == kept
    # validation: burn_in > max_iterations -> header only, status 1 (BayesRv2.cpp:69-80)
    assert O.run_csv(p, O.V2, X, Y, 5, 10, 1, cva=CVA, **HYP) == 1
    assert len(open(p).read().splitlines()) == 1


# r_compat stream against values R itself prints (R's documented defaults:
# Mersenne-Twister, Inversion): set.seed(42); runif(3) / set.seed(1); runif(3) /
# set.seed(1); rnorm(5) / set.seed(123); rnorm(5) / set.seed(42); rnorm(3) / set.seed(1); rexp(3)
R_KAT = [
    (42, "unif", [0.9148060, 0.9370754, 0.2861395]),
    (1, "unif", [0.2655087, 0.3721239, 0.5728534]),
    (1, "norm", [-0.6264538, 0.1836433, -0.8356286, 1.5952808, 0.3295078]),
    (123, "norm", [-0.56047565, -0.23017749, 1.55870831, 0.07050839, 0.12928774]),
    (42, "norm", [1.3709584, -0.5646982, 0.3631284]),
    (1, "exp", [0.7551818, 1.1816428, 0.1457067]),
]


@pytest.mark.parametrize("seed,kind,vals", R_KAT)
def test_r_compat_stream_known_answers(oracle_mod, seed, kind, vals):
    got = oracle_mod.r_stream(seed, kind, len(vals))
    np.testing.assert_allclose(got, vals, rtol=0, atol=6e-8 if kind != "norm" or seed != 123 else 6e-9)


@pytest.mark.parametrize("shape", [0.3, 1.0, 2.5, 7.0, 50.0])
def test_r_compat_gamma_and_beta_moments(oracle_mod, shape):
    """rgamma / rbeta(1,1) of the r_compat stream: parity unpinned (no R here), moments only"""
    g = oracle_mod.r_stream(7, "gamma", 100_000, shape)
    assert abs(g.mean() - shape) < 5 * np.sqrt(shape / g.size)
    assert abs(g.var() / shape - 1) < 0.05
    b = oracle_mod.r_stream(8, "beta11", 100_000)
    assert abs(b.mean() - 0.5) < 0.005 and abs(b.var() - 1 / 12) < 0.002 and b.min() > 0 and b.max() < 1


def test_r_compat_chain_is_deterministic_and_differs_from_philox(oracle_mod):
    O = oracle_mod
    X, Y, _ = O.synth_cohort(5, 200, 60, h2=0.5, n_causal=4)
    run = lambda **kw: O.Oracle(O.V2, X, Y, cva=CVA, order_mode=O.ORDER_REFERENCE, **HYP, **kw).sweep(5)  # noqa: E731
    a, b, c = run(r_seed=3), run(r_seed=3), run(seed=3)
    assert np.array_equal(a.vector(O.V_BETA), b.vector(O.V_BETA))
    assert not np.array_equal(a.vector(O.V_BETA), c.vector(O.V_BETA))


@pytest.mark.parametrize("kind,shape", [("gamma", 0.5), ("gamma", 1.0), ("gamma", 3.3), ("gamma", 20.0),
                                        ("exp", 1.0), ("beta11", 1.0), ("norm", 1.0)])
def test_r_compat_distributions_ks(oracle_mod, kind, shape):
    """The r_compat stream's draws follow their distributions (Kolmogorov-Smirnov against scipy's
    CDFs, 20,000 draws, fixed seeds): rgamma's GD / GS branches, exp_rand, rbeta(1,1), Inversion."""
    from scipy import stats
    x = oracle_mod.r_stream(11, kind, 20_000, shape)
    cdf = {"gamma": stats.gamma(shape).cdf, "exp": stats.expon().cdf, "beta11": stats.uniform().cdf,
           "norm": stats.norm().cdf}[kind]
    assert stats.kstest(x, cdf).pvalue > 1e-3


@pytest.mark.parametrize("shape", [0.3, 1.0, 4.5, 60.0])
def test_philox_gamma_ks(oracle_mod, shape):
    """The device's gamma (Marsaglia-Tsang on Philox, boost for a < 1; the GPU's rocRAND engine
    gives the same words) follows Gamma(shape): Kolmogorov-Smirnov against scipy, 20,000 draws."""
    from scipy import stats
    L = oracle_mod.lib()
    g = np.array([L.orc_gamma(9, shape, 3, i, 0) for i in range(20_000)])
    assert stats.kstest(g, stats.gamma(shape).cdf).pvalue > 1e-3


def test_philox_normal_uniform_ks(oracle_mod):
    from scipy import stats
    L = oracle_mod.lib()
    z = np.array([L.orc_normal(5, 1, i, 0, 1) for i in range(20_000)])
    u = np.array([L.orc_uniform(5, 1, i, 0, 0) for i in range(20_000)])
    assert stats.kstest(z, stats.norm().cdf).pvalue > 1e-3
    assert stats.kstest(u, stats.uniform().cdf).pvalue > 1e-3
