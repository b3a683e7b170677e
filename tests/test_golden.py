"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py from the CPU oracle).

CPU: the files match MANIFEST.json's SHA-256, and the oracle re-run on the same seeded inputs
reproduces every stored value bit for bit (an oracle regression fails here before it can move
the GPU parity tests).  GPU: the device chain, fed the same inputs, matches the stored
trajectories -- identical component assignments, everything else within relative 1e-9 (the
tolerance of tests/test_gpu_parity.py) -- with no oracle in the loop at run time.
The fixtures are oracle outputs: parity against the reference itself is unpinned.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import make_golden as MG  # noqa: E402

MANIFEST = json.load(open(os.path.join(GOLD, "MANIFEST.json")))
NAMES = sorted(MANIFEST["cases"])


def _load(name):
    return dict(np.load(os.path.join(GOLD, f"{name}.npz"), allow_pickle=False))


def test_manifest_hashes():
    assert sorted(MANIFEST["sha256"]) == [f"{n}.npz" for n in NAMES]
    for f, h in MANIFEST["sha256"].items():
        with open(os.path.join(GOLD, f), "rb") as fh:
            assert hashlib.sha256(fh.read()).hexdigest() == h, f


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(oracle_mod, name):
    gold = _load(name)
    res = MG.run_case(oracle_mod, MANIFEST["cases"][name])
    for k, v in gold.items():
        assert np.array_equal(res[k], v), f"{name}: {k} differs from the golden fixture"


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    scale = np.maximum(np.abs(b), np.max(np.abs(b)) * 1e-3 + 1e-300)
    return float(np.max(np.abs(a - b) / scale)) if a.size else 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_golden(brr, oracle_mod, require_gpu, name):
    from bayesrrcpp_amd import _lib as L
    c = MANIFEST["cases"][name]
    gold = _load(name)
    X, Y, kw = MG.inputs(oracle_mod, c)  # the oracle only regenerates the seeded inputs here
    h = hashlib.sha256(np.ascontiguousarray(X).tobytes() + np.ascontiguousarray(Y).tobytes()).digest()
    assert bytes(gold["input_sha256"]) == h
    model, N, P = c["model"], c["N"], c["P"]
    G, F = c.get("G", 1), c.get("F", 0)
    K = 1 if model == 3 else len(MG.CVA) + 1
    s = brr.Session(model, N, P, K=K, groups=G, F=F, block_size=c["B"], order_mode=c["order"])
    s.upload_x(X)
    if model != 2:
        s.set_y(Y)
    if model == 3:
        s.set_horseshoe(**{k: kw[k] for k in ("A", "v0E", "s02E", "vL", "vT", "c2", "vC", "sC")})
    else:
        s.set_bayesr(kw["sigma0"], kw["v0E"], kw["s02E"], kw["v0G"], kw["s02G"], kw["cva"], kw.get("gAssign"))
    if F:
        s.set_fixed(kw["fixed"])
    if model == 2:
        s.set_restart(kw["mu0"], kw["beta0"], kw["sigmaE0"], kw["sigmaGG0"], kw["eps0"], kw["comp0"])
    s.init(MG.CHAIN_SEED)
    for it in range(c["sweeps"]):
        s.sweep(1)
        tag = f"{name} sweep {it}"
        assert _rel(s.vector(L.BETA), gold["beta"][it]) < 1e-9, tag
        assert _rel(s.vector(L.EPS), gold["eps"][it]) < 1e-9, tag
        assert abs(s.scalar(L.MU) - gold["mu"][it]) <= 1e-9 * (1 + abs(gold["mu"][it])), tag
        assert _rel([s.scalar(L.SIGMAE)], [gold["sigmaE"][it]]) < 1e-9, tag
        if model == 3:
            assert _rel([s.scalar(L.TAU)], [gold["tau"][it]]) < 1e-9, tag
            assert _rel([s.scalar(L.C2)], [gold["c2"][it]]) < 1e-9, tag
            assert _rel(s.vector(L.LAMBDA), gold["lam"][it]) < 1e-9, tag
        else:
            assert np.array_equal(s.vector(L.COMP), gold["comp"][it]), tag
            assert _rel(s.vector(L.SIGMAGG), gold["sigmaG"][it]) < 1e-9, tag
            assert _rel(s.vector(L.PI), gold["pi"][it]) < 1e-9, tag
    assert np.array_equal(s.vector(L.ORDER).astype(np.int32), gold["order"]), name
