"""Python view of one device-resident chain (brr_session_* in include/brr.h)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _d(a):
    return a.ctypes.data_as(L.D)


def comm_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0 creates it, the caller broadcasts it)."""
    buf = C.create_string_buffer(128)
    L.check(L.lib().brr_comm_unique_id(buf), "comm_unique_id")
    return buf.raw


class Session:
    """One Gibbs chain on one GPU (one column shard).

    model: L.MODEL_V2 / MODEL_GROUPS / MODEL_RESTART / MODEL_HORSESHOE.
    K = mixture components including the zero one (len(cva) + 1).
    """

    def __init__(self, model, N, M, *, K=1, groups=1, F=0, M_total=None, col_offset=0,
                 device=0, block_size=0, order_mode=L.ORDER_BLOCKED, shard_rank=0,
                 shard_count=1, verbose=0, log=None, x_storage=L.X_F32, row_shard_rank=0,
                 row_shard_count=1, row_offset=0, N_total=0, exchanges_per_sweep=0):
        self._keep = []
        self.model, self.N, self.M, self.K, self.G, self.F = model, N, M, K, groups, F
        self.M_total = M if M_total is None else M_total
        self.col_offset = col_offset
        self.row_offset, self.N_total = row_offset, (N_total or N)
        self.opt = L.options(device, block_size, order_mode, shard_rank, shard_count, verbose, log,
                             x_storage, row_shard_rank, row_shard_count, row_offset, N_total,
                             exchanges_per_sweep)
        self.h = L.lib().brr_session_create(model, N, M, self.M_total, col_offset, K, groups, F,
                                            C.byref(self.opt))
        if not self.h:
            raise L.BrrError(f"brr_session_create failed: {L.last_error()}")

    # -- data -------------------------------------------------------------------------
    def upload_x(self, X):
        X = np.asarray(X)
        if X.shape != (self.N, self.M):
            raise ValueError(f"X must be {self.N} x {self.M}")
        if X.dtype == np.float32:
            Xf = np.asfortranarray(X)
            L.check(L.lib().brr_session_upload_x_f32(self.h, Xf.ctypes.data_as(C.POINTER(C.c_float)),
                                                     self.N), "upload_x_f32")
        else:
            Xd = np.asfortranarray(X, dtype=np.float64)
            L.check(L.lib().brr_session_upload_x_f64(self.h, _d(Xd), self.N), "upload_x_f64")
        return self

    def upload_bed(self, bed, bytes_per_col=None):
        """PLINK .bed body (after the 3 magic bytes) of this shard's markers: uint8 array of
        M * bytes_per_col bytes (SNP-major), or an (M, bytes_per_col) array."""
        b = np.ascontiguousarray(bed, dtype=np.uint8)
        if bytes_per_col is None:
            bytes_per_col = b.shape[1] if b.ndim == 2 else (self.N + 3) // 4
        if b.size < self.M * bytes_per_col:
            raise ValueError("bed holds fewer than M * bytes_per_col bytes")
        L.check(L.lib().brr_session_upload_bed(self.h, b.ctypes.data_as(C.POINTER(C.c_uint8)), bytes_per_col),
                "upload_bed")
        return self

    def synthesize(self, data_seed=20261015, h2=0.5, n_causal=-1):
        L.check(L.lib().brr_session_synthesize(self.h, data_seed, h2, n_causal), "synthesize")
        return self

    def synth_partial_y(self):
        out = np.zeros(self.N)
        L.check(L.lib().brr_session_synth_partial_y(self.h, _d(out)), "synth_partial_y")
        return out

    def synth_y(self, genetic_sum, data_seed=20261015, h2=0.5):
        g = np.ascontiguousarray(genetic_sum, dtype=np.float64)
        L.check(L.lib().brr_session_synth_y(self.h, _d(g), data_seed, h2), "synth_y")
        return self

    def set_y(self, Y):
        Y = np.ascontiguousarray(Y, dtype=np.float64)
        L.check(L.lib().brr_session_set_y(self.h, _d(Y)), "set_y")
        return self

    def set_fixed(self, fixed):
        f = np.asfortranarray(np.asarray(fixed, dtype=np.float64).reshape(self.N, -1))
        L.check(L.lib().brr_session_set_fixed(self.h, _d(f)), "set_fixed")
        return self

    def set_bayesr(self, sigma0, v0E, s02E, v0G, s02G, cva, gAssign=None):
        cva = np.asfortranarray(np.atleast_2d(np.asarray(cva, dtype=np.float64)).reshape(self.G, -1))
        ga = None
        if gAssign is not None:
            ga = np.ascontiguousarray(gAssign, dtype=np.int32)
            self._keep.append(ga)
        L.check(L.lib().brr_session_set_bayesr(self.h, sigma0, v0E, s02E, v0G, s02G, _d(cva),
                                               ga.ctypes.data_as(L.I32) if ga is not None else None),
                "set_bayesr")
        return self

    def set_horseshoe(self, A, v0E, s02E, vL, vT, c2, vC, sC):
        L.check(L.lib().brr_session_set_horseshoe(self.h, A, v0E, s02E, vL, vT, c2, vC, sC),
                "set_horseshoe")
        return self

    def set_restart(self, mu, beta, sigmaE, sigmaGG, eps, comp):
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (beta, sigmaGG, eps, comp)]
        L.check(L.lib().brr_session_set_restart(self.h, mu, _d(arrs[0]), sigmaE, _d(arrs[1]),
                                                _d(arrs[2]), _d(arrs[3])), "set_restart")
        return self

    def set_pi(self, pi):
        pi = np.ascontiguousarray(pi, dtype=np.float64).ravel()
        L.check(L.lib().brr_session_set_pi(self.h, _d(pi)), "set_pi")
        return self

    # -- chain ------------------------------------------------------------------------
    def init(self, seed=1):
        L.check(L.lib().brr_session_init(self.h, seed), "init")
        return self

    def sweep(self, n=1):
        L.check(L.lib().brr_session_sweep(self.h, n), "sweep")
        return self

    def init_local(self, seed=1):
        """Column-sharded init without a communicator: sum exchange_get()[1] across shards,
        exchange_set(None, total), then init_finish() (restart model; a full init otherwise)."""
        L.check(L.lib().brr_session_init_local(self.h, seed), "init_local")
        return self

    def init_finish(self):
        L.check(L.lib().brr_session_init_finish(self.h), "init_finish")
        return self

    def exchange_sizes(self):
        a, b = C.c_int64(), C.c_int64()
        L.check(L.lib().brr_session_exchange_sizes(self.h, C.byref(a), C.byref(b)), "exchange_sizes")
        return a.value, b.value

    def set_exchange(self, eps_ptr: int, stats_ptr: int):
        L.check(L.lib().brr_session_set_exchange(self.h, C.c_void_p(eps_ptr), C.c_void_p(stats_ptr)),
                "set_exchange")

    def exchange_buffers(self):
        e, st = C.c_void_p(), C.c_void_p()
        L.check(L.lib().brr_session_exchange_buffers(self.h, C.byref(e), C.byref(st)), "exchange_buffers")
        return e.value, st.value

    def exchange_get(self):
        ne, ns = self.exchange_sizes()
        e, st = np.zeros(ne), np.zeros(ns)
        L.check(L.lib().brr_session_exchange_copy(self.h, 0, _d(e), _d(st)), "exchange_copy")
        return e, st

    def exchange_set(self, eps, stats):
        e = None if eps is None else np.ascontiguousarray(eps, dtype=np.float64)
        st = None if stats is None else np.ascontiguousarray(stats, dtype=np.float64)
        L.check(L.lib().brr_session_exchange_copy(self.h, 1, None if e is None else _d(e),
                                                  None if st is None else _d(st)), "exchange_copy")

    def comm_init(self, unique_id: bytes, nranks: int, rank: int):
        L.check(L.lib().brr_session_comm_init(self.h, unique_id, nranks, rank), "comm_init")

    def sweep_local(self):
        L.check(L.lib().brr_session_sweep_local(self.h), "sweep_local")

    def sweep_finish(self):
        L.check(L.lib().brr_session_sweep_finish(self.h), "sweep_finish")

    @property
    def exchanges_per_sweep(self):
        """local / exchange / finish rounds per sweep (column shards, brr_options.exchanges_per_sweep)"""
        return L.lib().brr_session_exchanges_per_sweep(self.h)

    def synchronize(self):
        L.check(L.lib().brr_session_synchronize(self.h), "synchronize")

    @property
    def iteration(self):
        return L.lib().brr_session_iteration(self.h)

    # -- state ------------------------------------------------------------------------
    def scalar(self, which):
        out = C.c_double()
        L.check(L.lib().brr_session_get_scalar(self.h, which, C.byref(out)), "get_scalar")
        return out.value

    def vector(self, which):
        n = L.lib().brr_session_get_vector(self.h, which, None)
        if n < 0:
            raise L.BrrError(f"get_vector({which}): {L.last_error()}")
        out = np.zeros(n, dtype=np.float64)
        if n:
            r = L.lib().brr_session_get_vector(self.h, which, _d(out))
            if r < 0:
                raise L.BrrError(f"get_vector({which}): {L.last_error()}")
        return out

    def linear_predictor(self):
        """X beta + F alpha of this shard (N doubles; plain validation kernel, not the sweep path)."""
        out = np.zeros(self.N)
        L.check(L.lib().brr_session_linear_predictor(self.h, _d(out)), "linear_predictor")
        return out

    def set_vector(self, which, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        L.check(L.lib().brr_session_set_vector(self.h, which, _d(arr)), "set_vector")

    def set_scalar(self, which, v):
        L.check(L.lib().brr_session_set_scalar(self.h, which, v), "set_scalar")

    def state(self):
        s = {"mu": self.scalar(L.MU), "sigmaE": self.scalar(L.SIGMAE),
             "beta": self.vector(L.BETA), "eps": self.vector(L.EPS)}
        if self.model == L.MODEL_HORSESHOE:
            s.update(tau=self.scalar(L.TAU), eta=self.scalar(L.ETA), c2=self.scalar(L.C2),
                     lambda_=self.vector(L.LAMBDA))
        else:
            s.update(comp=self.vector(L.COMP), pi=self.vector(L.PI), sigmaGG=self.vector(L.SIGMAGG))
            if self.model == L.MODEL_GROUPS:
                s.update(sigmaF=self.scalar(L.SIGMAF), alpha=self.vector(L.ALPHA))
        return s

    # -- sample output ----------------------------------------------------------
    def output_open(self, path, header=True, ring_depth=4):
        """Reference CSV of kept sweeps (asynchronous: device snapshot -> pinned ring -> writer)."""
        L.check(L.lib().brr_session_output_open(self.h, str(path).encode(), self.model, self.N, self.M,
                                                self.G, self.F, 1 if header else 0, ring_depth), "output_open")

    def output_sample(self, iteration):
        L.check(L.lib().brr_session_output_sample(self.h, iteration), "output_sample")

    def output_close(self):
        """Drains the writer; returns the most rows ever in flight (bounded by ring_depth)."""
        m = C.c_int32()
        L.check(L.lib().brr_session_output_close(self.h, C.byref(m)), "output_close")
        return m.value

    # -- instrumentation ----------------------------------------------------------------
    def set_timing(self, on: bool):
        L.check(L.lib().brr_session_set_timing(self.h, 1 if on else 0), "set_timing")

    def timing(self):
        a, b = C.c_double(), C.c_double()
        na, nb = C.c_int64(), C.c_int64()
        L.check(L.lib().brr_session_timing(self.h, C.byref(a), C.byref(na), C.byref(b), C.byref(nb)),
                "timing")
        return {"stream_ms": a.value, "stream_launches": na.value,
                "solve_ms": b.value, "solve_launches": nb.value}

    @property
    def block_size(self):
        return L.lib().brr_session_block_size(self.h)

    def close(self):
        if getattr(self, "h", None):
            L.lib().brr_session_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()  # device memory goes now, not when a failed test's traceback lets go of the object
        return False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Group:
    """Exact row shards driven in lock step from one process (brr_group_*).

    members: Sessions created with row_shard_rank 0..n-1 / row_shard_count n (rows
    [row_offset, row_offset + N) of an N_total-row cohort, every marker).  Data setters stay per
    session; init and sweeps run through the group (the cross-shard sums happen on the device).
    """

    def __init__(self, members):
        self.members = list(members)
        arr = (C.c_void_p * len(self.members))(*[m.h for m in self.members])
        self.h = L.lib().brr_group_create(arr, len(self.members))
        if not self.h:
            raise L.BrrError(f"brr_group_create failed: {L.last_error()}")

    def init(self, seed=1):
        L.check(L.lib().brr_group_init(self.h, seed), "group_init")
        return self

    def sweep(self, n=1):
        L.check(L.lib().brr_group_sweep(self.h, n), "group_sweep")
        return self

    def close(self):
        if getattr(self, "h", None):
            L.lib().brr_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
