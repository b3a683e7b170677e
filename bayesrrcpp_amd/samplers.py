"""The reference's R-level interface, mirrored in Python over the C ABI.

Same names, argument order and meaning as the R closures (R/RcppExports.R:25-76) and the
C++ functions behind them (src/BayesRv2.cpp:60, src/BayesRv2Groups.cpp:75,
src/BRv2Grstart.cpp:77, src/HorseshoeR.cpp:109).  Each call runs the whole chain on the GPU
and writes the reference's CSV file; like the R functions it returns None (invisible NULL).
Validation follows the reference: an invalid iteration setting prints the reference's error
message and returns without sampling (status 1 from the C ABI); hyper-parameter problems only
warn.  Extra keyword-only options (device, block_size, order_mode, verbose, log) select the
device path's knobs; they do not change the meaning of the reference arguments.
"""
from __future__ import annotations

import sys

import numpy as np

from . import _lib as L


def _f(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def _logger(log):
    return log if log is not None else (lambda m: sys.stderr.write(m))


def _run(fn, *args):
    rc = fn(*args)
    if rc < 0:
        raise L.BrrError(f"{fn.__name__} failed (rc={rc}): {L.last_error()}")
    return rc


def BayesRSamplerV2(outputFile, seed, max_iterations, burn_in, thinning, X, Y, sigma0, v0E, s02E,
                    v0G, s02G, cva, *, device=0, block_size=0, order_mode=L.ORDER_BLOCKED,
                    verbose=0, log=None):
    X = _f(X)
    Y = np.ascontiguousarray(Y, dtype=np.float64).ravel()
    cva = np.ascontiguousarray(cva, dtype=np.float64).ravel()
    N, M = X.shape
    opt = L.options(device, block_size, order_mode, 0, 1, verbose, _logger(log))
    _run(L.lib().brr_BayesRSamplerV2, outputFile.encode(), seed, max_iterations, burn_in, thinning,
         X.ctypes.data_as(L.D), N, M, Y.ctypes.data_as(L.D), sigma0, v0E, s02E, v0G, s02G,
         cva.ctypes.data_as(L.D), len(cva), opt)
    return None


def BayesRSamplerV2Groups(outputFile, seed, max_iterations, burn_in, thinning, X, Y, sigma0, v0E,
                          s02E, v0G, s02G, cva, groups, gAssign, fixed, *, device=0, block_size=0,
                          order_mode=L.ORDER_BLOCKED, verbose=0, log=None):
    X = _f(X)
    N, M = X.shape
    Y = np.ascontiguousarray(Y, dtype=np.float64).ravel()
    cva = _f(np.atleast_2d(cva).reshape(groups, -1))
    ga = np.ascontiguousarray(gAssign, dtype=np.int32).ravel()
    fixed = _f(np.asarray(fixed, dtype=np.float64).reshape(N, -1))
    F = fixed.shape[1]
    opt = L.options(device, block_size, order_mode, 0, 1, verbose, _logger(log))
    _run(L.lib().brr_BayesRSamplerV2Groups, outputFile.encode(), seed, max_iterations, burn_in,
         thinning, X.ctypes.data_as(L.D), N, M, Y.ctypes.data_as(L.D), sigma0, v0E, s02E, v0G, s02G,
         cva.ctypes.data_as(L.D), cva.shape[1], groups, ga.ctypes.data_as(L.I32),
         fixed.ctypes.data_as(L.D), F, opt)
    return None


def BRV2Grstart(outputFile, seed, max_iterations, burn_in, thinning, mu, beta, sigmaE, sigmaGG, X,
                epsilon, components, sigma0, v0E, s02E, v0G, s02G, cva, groups, gAssign, *,
                device=0, block_size=0, order_mode=L.ORDER_BLOCKED, verbose=0, log=None):
    X = _f(X)
    N, M = X.shape
    beta = np.ascontiguousarray(beta, dtype=np.float64).ravel()
    sgg = np.ascontiguousarray(sigmaGG, dtype=np.float64).ravel()
    eps = np.ascontiguousarray(epsilon, dtype=np.float64).ravel()
    comp = np.ascontiguousarray(components, dtype=np.float64).ravel()
    cva = _f(np.atleast_2d(cva).reshape(groups, -1))
    ga = np.ascontiguousarray(gAssign, dtype=np.int32).ravel()
    if len(eps) != N:  # N is taken from epsilon.size() in the reference (BRv2Grstart.cpp:81)
        raise ValueError("epsilon must have one entry per row of X")
    opt = L.options(device, block_size, order_mode, 0, 1, verbose, _logger(log))
    _run(L.lib().brr_BRV2Grstart, outputFile.encode(), seed, max_iterations, burn_in, thinning, mu,
         beta.ctypes.data_as(L.D), sigmaE, sgg.ctypes.data_as(L.D), X.ctypes.data_as(L.D), N, M,
         eps.ctypes.data_as(L.D), comp.ctypes.data_as(L.D), sigma0, v0E, s02E, v0G, s02G,
         cva.ctypes.data_as(L.D), cva.shape[1], groups, ga.ctypes.data_as(L.I32), opt)
    return None


def HorseshoeR(outputFile, seed, max_iterations, burn_in, thinning, X, Y, A, v0E, s02E, vL, vT, c2,
               vC, sC, *, device=0, block_size=0, order_mode=L.ORDER_BLOCKED, verbose=0, log=None):
    X = _f(X)
    N, M = X.shape
    Y = np.ascontiguousarray(Y, dtype=np.float64).ravel()
    opt = L.options(device, block_size, order_mode, 0, 1, verbose, _logger(log))
    _run(L.lib().brr_HorseshoeR, outputFile.encode(), seed, max_iterations, burn_in, thinning,
         X.ctypes.data_as(L.D), N, M, Y.ctypes.data_as(L.D), A, v0E, s02E, vL, vT, c2, vC, sC, opt)
    return None
