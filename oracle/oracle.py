"""ctypes wrapper around oracle/_build/liboracle.so -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker (never as the measured or shipped path).  It wraps
the C restatement in brr_oracle.c (see its header for what it restates and the
parity status: unpinned against reference-produced outputs, none exist).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

V2, GROUPS, RESTART, HORSESHOE = 0, 1, 2, 3
ORDER_BLOCKED, ORDER_REFERENCE, ORDER_IDENTITY = 0, 1, 2

(S_MU, S_SIGMAE, S_SIGMAG, S_SIGMAF, S_TAU, S_ETA, S_C2, S_SUMSQ_BETA) = range(8)
(V_BETA, V_COMP, V_EPS, V_SIGMAGG, V_PI, V_ALPHA, V_LAMBDA, V_XSQ, V_ORDER, V_VCOUNT,
 V_BETAACUM, V_HSV) = range(12)

T_MARKER, T_MU, T_SIGMAE, T_SIGMAG, T_PI = 1, 2, 3, 4, 5
T_INIT = 13
INIT_IT = 0xFFFFFFFF


class OrcConfig(C.Structure):
    _fields_ = [
        ("model", C.c_int32), ("N", C.c_int64), ("P", C.c_int64), ("K", C.c_int32),
        ("G", C.c_int32), ("F", C.c_int32),
        ("X", C.POINTER(C.c_double)), ("Y", C.POINTER(C.c_double)),
        ("fixed", C.POINTER(C.c_double)), ("cva", C.POINTER(C.c_double)),
        ("gAssign", C.POINTER(C.c_int32)),
        ("sigma0", C.c_double), ("v0E", C.c_double), ("s02E", C.c_double),
        ("v0G", C.c_double), ("s02G", C.c_double),
        ("A", C.c_double), ("vL", C.c_double), ("vT", C.c_double), ("c2", C.c_double),
        ("vC", C.c_double), ("sC", C.c_double),
        ("mu0", C.c_double), ("sigmaE0", C.c_double),
        ("beta0", C.POINTER(C.c_double)), ("sigmaGG0", C.POINTER(C.c_double)),
        ("eps0", C.POINTER(C.c_double)), ("comp0", C.POINTER(C.c_double)),
        ("seed", C.c_int32), ("order_mode", C.c_int32), ("block_size", C.c_int32),
        ("n_shards", C.c_int32), ("pi0", C.POINTER(C.c_double)),
        ("shard_only", C.c_int32), ("n_exchanges", C.c_int32),
    ]


def build() -> str:
    """Compile the oracle with its Makefile (idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(OrcConfig)]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_init.argtypes = [C.c_void_p]
        L.orc_sweep.argtypes = [C.c_void_p, C.c_int]
        L.orc_iteration.argtypes = [C.c_void_p]
        L.orc_get_scalar.restype = C.c_double
        L.orc_get_scalar.argtypes = [C.c_void_p, C.c_int]
        L.orc_set_scalar.argtypes = [C.c_void_p, C.c_int, C.c_double]
        L.orc_get_vector.restype = C.c_int64
        L.orc_get_vector.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        L.orc_set_vector.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        L.orc_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]
        L.orc_u53.restype = C.c_double
        L.orc_u53.argtypes = [C.c_uint32, C.c_uint32]
        for fn in ("orc_uniform", "orc_normal"):
            getattr(L, fn).restype = C.c_double
            getattr(L, fn).argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                       C.c_uint32]
        L.orc_gamma.restype = C.c_double
        L.orc_gamma.argtypes = [C.c_uint64, C.c_double, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_glibc_rand.argtypes = [C.c_uint32, C.c_int, C.POINTER(C.c_int32)]
        L.orc_blocked_order.argtypes = [C.c_uint64, C.c_uint32, C.c_int64, C.c_int32,
                                        C.c_int32, C.c_int64, C.POINTER(C.c_int32)]
        L.orc_synth_x.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int64,
                                  C.POINTER(C.c_double)]
        L.orc_synth_beta.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                     C.POINTER(C.c_double)]
        L.orc_sweep_local.argtypes = [C.c_void_p]
        L.orc_sweep_finish.argtypes = [C.c_void_p]
        L.orc_stats_size.restype = C.c_int64
        L.orc_stats_size.argtypes = [C.c_void_p]
        L.orc_exchange_get.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_exchange_set.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_set_rng_r.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
        L.orc_rstream_create.restype = C.c_void_p
        L.orc_rstream_create.argtypes = [C.c_uint32]
        L.orc_rstream_destroy.argtypes = [C.c_void_p]
        for fn in ("orc_r_unif", "orc_r_norm", "orc_r_exp", "orc_r_beta11"):
            getattr(L, fn).restype = C.c_double
            getattr(L, fn).argtypes = [C.c_void_p]
        L.orc_r_gamma.restype = C.c_double
        L.orc_r_gamma.argtypes = [C.c_void_p, C.c_double]
        L.orc_run_csv.argtypes = [C.POINTER(OrcConfig), C.c_char_p, C.c_int, C.c_int, C.c_int]
        _lib = L
    return _lib


def _dptr(a):
    if a is None:
        return C.POINTER(C.c_double)()
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _iptr(a):
    if a is None:
        return C.POINTER(C.c_int32)()
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def r_stream(r_seed: int, kind: str, n: int, shape: float = 1.0) -> np.ndarray:
    """n draws of R's set.seed(r_seed); kind in unif / norm / exp / gamma / beta11."""
    L = lib()
    h = L.orc_rstream_create(C.c_uint32(int(r_seed) & 0xFFFFFFFF))
    try:
        if kind == "gamma":
            return np.array([L.orc_r_gamma(h, shape) for _ in range(n)])
        fn = {"unif": L.orc_r_unif, "norm": L.orc_r_norm, "exp": L.orc_r_exp, "beta11": L.orc_r_beta11}[kind]
        return np.array([fn(h) for _ in range(n)])
    finally:
        L.orc_rstream_destroy(h)


def glibc_rand(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.int32)
    lib().orc_glibc_rand(seed, n, _iptr(out))
    return out


def blocked_order(seed, it, P, B, shard=0, col_offset=0) -> np.ndarray:
    out = np.zeros(P, dtype=np.int32)
    lib().orc_blocked_order(seed & 0xFFFFFFFFFFFFFFFF, it, P, B, shard, col_offset, _iptr(out))
    return out


def synth_x(data_seed: int, N: int, P: int, col0: int = 0) -> np.ndarray:
    X = np.zeros((P, N), dtype=np.float64)  # column-major storage: row p = column p
    lib().orc_synth_x(data_seed, N, P, col0, _dptr(X))
    return X.T  # N x P view (Fortran-ordered)


def synth_beta(data_seed: int, P_total: int, n_causal: int, col0: int, P: int) -> np.ndarray:
    b = np.zeros(P, dtype=np.float64)
    lib().orc_synth_beta(data_seed, P_total, n_causal, col0, P, _dptr(b))
    return b


def synth_cohort(data_seed: int, N: int, P: int, h2: float = 0.5, n_causal: int | None = None):
    """Host synthetic cohort: X standardised f32-valued, Y standardised."""
    if n_causal is None:
        n_causal = max(1, min(1000, P // 10))
    X = synth_x(data_seed, N, P)
    b = synth_beta(data_seed, P, n_causal, 0, P) * np.sqrt(h2 / n_causal)
    rng = np.random.default_rng(data_seed)
    y = X @ b + rng.normal(0.0, np.sqrt(1.0 - h2), N)
    Y = (y - y.mean()) / y.std(ddof=1)
    return np.asfortranarray(X), Y, b


class Oracle:
    """One oracle chain. Arrays are kept alive on the instance (C holds raw pointers)."""

    def __init__(self, model, X=None, Y=None, *, cva=None, gAssign=None, fixed=None, G=1,
                 seed=1, order_mode=ORDER_BLOCKED, block_size=0, n_shards=1,
                 sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3,
                 A=1.0, vL=1.0, vT=1.0, c2=1.0, vC=10.0, sC=10.0,
                 mu0=0.0, sigmaE0=1.0, beta0=None, sigmaGG0=None, eps0=None, comp0=None,
                 pi0=None, N=None, shard_only=-1, r_seed=None, n_exchanges=1):
        # r_seed: draw from the r_compat stream (R's set.seed(r_seed) Mersenne-Twister /
        # Inversion / rgamma / rbeta, in the reference's call order) instead of Philox
        self._keep = []
        X = np.asfortranarray(np.asarray(X, dtype=np.float64))
        if N is None:
            N = X.shape[0] if Y is None else len(Y)
        P = X.shape[1]
        cfg = OrcConfig()
        cfg.model = model
        cfg.N, cfg.P = N, P
        if cva is not None:
            cva = np.asfortranarray(np.atleast_2d(np.asarray(cva, dtype=np.float64)))
            if cva.shape[0] != G and cva.shape[1] == G:
                cva = np.asfortranarray(cva.T)
            cfg.K = cva.shape[1] + 1
        else:
            cfg.K = 1
        cfg.G = G
        cfg.F = 0 if fixed is None else np.atleast_2d(fixed).reshape(N, -1).shape[1]
        keep = lambda a: (self._keep.append(a), a)[1]  # noqa: E731
        cfg.X = _dptr(keep(X))
        if Y is not None:
            cfg.Y = _dptr(keep(np.ascontiguousarray(Y, dtype=np.float64)))
        if fixed is not None:
            cfg.fixed = _dptr(keep(np.asfortranarray(np.asarray(fixed, np.float64).reshape(N, -1))))
        if cva is not None:
            cfg.cva = _dptr(keep(cva))
        if gAssign is not None:
            cfg.gAssign = _iptr(keep(np.ascontiguousarray(gAssign, dtype=np.int32)))
        cfg.sigma0, cfg.v0E, cfg.s02E, cfg.v0G, cfg.s02G = sigma0, v0E, s02E, v0G, s02G
        cfg.A, cfg.vL, cfg.vT, cfg.c2, cfg.vC, cfg.sC = A, vL, vT, c2, vC, sC
        cfg.mu0, cfg.sigmaE0 = mu0, sigmaE0
        for name, arr in (("beta0", beta0), ("sigmaGG0", sigmaGG0), ("eps0", eps0),
                          ("comp0", comp0), ("pi0", pi0)):
            if arr is not None:
                setattr(cfg, name, _dptr(keep(np.ascontiguousarray(arr, dtype=np.float64).ravel())))
        cfg.seed = seed
        cfg.order_mode = order_mode
        # 0 = the library's automatic block size (brr_session.cpp brr_session_create)
        cfg.block_size = block_size or (128 if model in (HORSESHOE, GROUPS) or N < 32768 or order_mode == ORDER_REFERENCE else 512)
        cfg.n_shards = n_shards
        cfg.shard_only = shard_only
        cfg.n_exchanges = n_exchanges
        self.cfg = cfg
        self.N, self.P, self.K, self.G = N, P, cfg.K, G
        self.h = lib().orc_create(C.byref(cfg))
        if not self.h:
            raise ValueError("orc_create rejected the configuration")
        if r_seed is not None:
            lib().orc_set_rng_r(self.h, 1, C.c_uint32(int(r_seed) & 0xFFFFFFFF))
        lib().orc_init(self.h)

    def sweep(self, n=1):
        lib().orc_sweep(self.h, n)
        return self

    @property
    def exchanges_per_sweep(self):
        """per-shard protocol: local / exchange / finish rounds per sweep (n_exchanges)"""
        return self.cfg.n_exchanges if self.cfg.n_shards > 1 and self.cfg.shard_only >= 0 else 1

    # per-shard protocol (shard_only >= 0): local sweep -> exchange -> finish
    def sweep_local(self):
        assert lib().orc_sweep_local(self.h) == 0

    def exchange_get(self):
        ns = lib().orc_stats_size(self.h)
        e, s = np.zeros(self.N), np.zeros(ns)
        lib().orc_exchange_get(self.h, _dptr(e), _dptr(s))
        return e, s

    def exchange_set(self, eps_sum, stats_sum):
        e = np.ascontiguousarray(eps_sum, dtype=np.float64)
        s = np.ascontiguousarray(stats_sum, dtype=np.float64)
        lib().orc_exchange_set(self.h, _dptr(e), _dptr(s))

    def sweep_finish(self):
        lib().orc_sweep_finish(self.h)

    def scalar(self, which):
        return lib().orc_get_scalar(self.h, which)

    def vector(self, which):
        n = lib().orc_get_vector(self.h, which, None)
        out = np.zeros(max(n, 0), dtype=np.float64)
        lib().orc_get_vector(self.h, which, _dptr(out))
        return out

    def set_vector(self, which, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        self._keep.append(arr)
        assert lib().orc_set_vector(self.h, which, _dptr(arr)) == 0

    def set_scalar(self, which, v):
        assert lib().orc_set_scalar(self.h, which, v) == 0

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().orc_destroy(self.h)
                self.h = None
        except Exception:
            pass


def run_csv(path, model, X, Y, max_iterations, burn_in, thinning, **kw):
    """Reference-faithful one-shot run writing the reference CSV (orc_run_csv)."""
    tmp = Oracle(model, X, Y, **kw)  # marshals the config; orc_run_csv builds its own chain
    return lib().orc_run_csv(C.byref(tmp.cfg), path.encode(), max_iterations, burn_in, thinning)
