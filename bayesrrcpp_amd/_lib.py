"""ctypes binding of libbrr.so (include/brr.h).

Loading fails loudly: there is no CPU fallback for the sampler.  `lib()` raises if the
shared library is missing or cannot be loaded; every session call raises BrrError with the
library's message when the device path fails.
"""
from __future__ import annotations

import ctypes as C
import os

from .build import LIB_PATH

MODEL_V2, MODEL_GROUPS, MODEL_RESTART, MODEL_HORSESHOE = 0, 1, 2, 3
ORDER_BLOCKED, ORDER_REFERENCE, ORDER_IDENTITY = 0, 1, 2
X_F32, X_2BIT = 0, 1  # brr_x_storage
(MU, SIGMAE, SIGMAG, SIGMAF, TAU, ETA, C2, SUMSQ_BETA) = range(8)
(BETA, COMP, EPS, SIGMAGG, PI, ALPHA, LAMBDA, XSQ, ORDER, VCOUNT, BETAACUM, HSV) = range(12)
ABI_VERSION = 4

LOG_FN = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)


class BrrError(RuntimeError):
    pass


class Options(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("device", C.c_int32), ("block_size", C.c_int32),
        ("order_mode", C.c_int32), ("shard_rank", C.c_int32), ("shard_count", C.c_int32),
        ("verbose", C.c_int32), ("x_storage", C.c_int32),
        ("log", LOG_FN), ("log_userdata", C.c_void_p),
        ("row_shard_rank", C.c_int32), ("row_shard_count", C.c_int32),
        ("row_offset", C.c_int64), ("N_total", C.c_int64),
        ("exchanges_per_sweep", C.c_int32),
    ]


# every symbol include/brr.h declares (checked by tests/test_capi.py)
EXPORTED = [
    "brr_options_default", "brr_options_effective", "brr_last_error", "brr_device_count", "brr_device_memory",
    "brr_BayesRSamplerV2", "brr_BayesRSamplerV2Groups", "brr_BRV2Grstart", "brr_HorseshoeR",
    "brr_session_create", "brr_session_destroy", "brr_session_upload_x_f64",
    "brr_session_upload_x_f32", "brr_session_upload_bed", "brr_session_synthesize", "brr_session_synth_partial_y",
    "brr_session_synth_y", "brr_session_set_y",
    "brr_session_set_fixed", "brr_session_set_bayesr", "brr_session_set_horseshoe",
    "brr_session_set_restart", "brr_session_set_pi", "brr_session_init", "brr_session_sweep",
    "brr_session_exchange_sizes", "brr_session_set_exchange", "brr_session_exchange_buffers",
    "brr_session_exchange_copy", "brr_comm_unique_id", "brr_session_comm_init",
    "brr_session_sweep_local", "brr_session_init_local", "brr_session_init_finish",
    "brr_session_sweep_finish", "brr_session_exchanges_per_sweep", "brr_session_get_scalar", "brr_session_get_vector",
    "brr_session_set_vector", "brr_session_set_scalar", "brr_session_iteration",
    "brr_session_set_timing", "brr_session_timing", "brr_session_block_size",
    "brr_session_synchronize", "brr_session_linear_predictor",
    "brr_group_create", "brr_group_init", "brr_group_sweep", "brr_group_destroy",
    "brr_session_output_open", "brr_session_output_sample", "brr_session_output_close",
]

_lib = None

D = C.POINTER(C.c_double)
I32 = C.POINTER(C.c_int32)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("BRR_LIB", LIB_PATH)  # alternative in-tree build (kernel variants)
    if not os.path.exists(path):
        raise BrrError(f"{path} is missing: build it with bayesrrcpp_amd.build.build_library() "
                       "(the MI355X sampler has no CPU fallback)")
    L = C.CDLL(path)
    vp = C.c_void_p
    L.brr_options_default.argtypes = [C.POINTER(Options)]
    L.brr_options_effective.argtypes = [C.POINTER(Options), C.POINTER(Options)]
    L.brr_last_error.restype = C.c_char_p
    L.brr_device_count.restype = C.c_int
    L.brr_device_memory.argtypes = [C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.brr_BayesRSamplerV2.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, D, C.c_int64,
                                      C.c_int64, D, C.c_double, C.c_double, C.c_double, C.c_double,
                                      C.c_double, D, C.c_int32, C.POINTER(Options)]
    L.brr_BayesRSamplerV2Groups.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, D,
                                            C.c_int64, C.c_int64, D, C.c_double, C.c_double,
                                            C.c_double, C.c_double, C.c_double, D, C.c_int32,
                                            C.c_int, I32, D, C.c_int64, C.POINTER(Options)]
    L.brr_BRV2Grstart.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, D,
                                  C.c_double, D, D, C.c_int64, C.c_int64, D, D, C.c_double,
                                  C.c_double, C.c_double, C.c_double, C.c_double, D, C.c_int32,
                                  C.c_int, I32, C.POINTER(Options)]
    L.brr_HorseshoeR.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, D, C.c_int64,
                                 C.c_int64, D, C.c_double, C.c_double, C.c_double, C.c_double,
                                 C.c_double, C.c_double, C.c_double, C.c_double, C.POINTER(Options)]
    L.brr_session_create.restype = vp
    L.brr_session_create.argtypes = [C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                     C.c_int32, C.c_int32, C.c_int64, C.POINTER(Options)]
    L.brr_session_destroy.argtypes = [vp]
    L.brr_session_upload_x_f64.argtypes = [vp, D, C.c_int64]
    L.brr_session_upload_x_f32.argtypes = [vp, C.POINTER(C.c_float), C.c_int64]
    L.brr_session_upload_bed.argtypes = [vp, C.POINTER(C.c_uint8), C.c_int64]
    L.brr_session_synthesize.argtypes = [vp, C.c_uint64, C.c_double, C.c_int64]
    L.brr_session_synth_partial_y.argtypes = [vp, D]
    L.brr_session_synth_y.argtypes = [vp, D, C.c_uint64, C.c_double]
    L.brr_session_set_y.argtypes = [vp, D]
    L.brr_session_set_fixed.argtypes = [vp, D]
    L.brr_session_set_bayesr.argtypes = [vp, C.c_double, C.c_double, C.c_double, C.c_double,
                                         C.c_double, D, I32]
    L.brr_session_set_horseshoe.argtypes = [vp] + [C.c_double] * 8
    L.brr_session_set_restart.argtypes = [vp, C.c_double, D, C.c_double, D, D, D]
    L.brr_session_set_pi.argtypes = [vp, D]
    L.brr_session_init.argtypes = [vp, C.c_int32]
    L.brr_session_sweep.argtypes = [vp, C.c_int32]
    L.brr_session_exchange_sizes.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.brr_session_set_exchange.argtypes = [vp, vp, vp]
    L.brr_session_exchange_buffers.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
    L.brr_session_exchange_copy.argtypes = [vp, C.c_int32, D, D]
    L.brr_comm_unique_id.argtypes = [C.c_char_p]
    L.brr_session_comm_init.argtypes = [vp, C.c_char_p, C.c_int32, C.c_int32]
    L.brr_session_sweep_local.argtypes = [vp]
    L.brr_session_init_local.argtypes = [vp, C.c_int32]
    L.brr_session_init_finish.argtypes = [vp]
    L.brr_session_sweep_finish.argtypes = [vp]
    L.brr_session_exchanges_per_sweep.restype = C.c_int32
    L.brr_session_exchanges_per_sweep.argtypes = [vp]
    L.brr_session_get_scalar.argtypes = [vp, C.c_int32, D]
    L.brr_session_get_vector.restype = C.c_int64
    L.brr_session_get_vector.argtypes = [vp, C.c_int32, D]
    L.brr_session_set_vector.argtypes = [vp, C.c_int32, D]
    L.brr_session_set_scalar.argtypes = [vp, C.c_int32, C.c_double]
    L.brr_session_iteration.restype = C.c_int32
    L.brr_session_iteration.argtypes = [vp]
    L.brr_session_set_timing.argtypes = [vp, C.c_int32]
    L.brr_session_timing.argtypes = [vp, D, C.POINTER(C.c_int64), D, C.POINTER(C.c_int64)]
    L.brr_session_block_size.restype = C.c_int64
    L.brr_session_block_size.argtypes = [vp]
    L.brr_session_synchronize.argtypes = [vp]
    L.brr_session_linear_predictor.argtypes = [vp, D]
    L.brr_group_create.restype = vp
    L.brr_group_create.argtypes = [C.POINTER(vp), C.c_int32]
    L.brr_group_init.argtypes = [vp, C.c_int32]
    L.brr_group_sweep.argtypes = [vp, C.c_int32]
    L.brr_group_destroy.argtypes = [vp]
    L.brr_session_output_open.argtypes = [vp, C.c_char_p, C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int64,
                                          C.c_int32, C.c_int32]
    L.brr_session_output_sample.argtypes = [vp, C.c_int32]
    L.brr_session_output_close.argtypes = [vp, C.POINTER(C.c_int32)]
    _lib = L
    return L


def device_memory(device=0):
    """(free, total) bytes of a HIP device."""
    f, t = C.c_int64(), C.c_int64()
    check(lib().brr_device_memory(device, C.byref(f), C.byref(t)), "device_memory")
    return f.value, t.value


def last_error() -> str:
    msg = lib().brr_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> int:
    if rc != 0:
        raise BrrError(f"{what} failed (rc={rc}): {last_error()}")
    return rc


def options(device=0, block_size=0, order_mode=ORDER_BLOCKED, shard_rank=0, shard_count=1,
            verbose=0, log=None, x_storage=X_F32, row_shard_rank=0, row_shard_count=1, row_offset=0,
            N_total=0, exchanges_per_sweep=0) -> Options:
    o = Options()
    lib().brr_options_default(C.byref(o))
    o.device, o.block_size, o.order_mode = device, block_size, order_mode
    o.shard_rank, o.shard_count, o.verbose = shard_rank, shard_count, verbose
    o.x_storage = x_storage
    o.row_shard_rank, o.row_shard_count = row_shard_rank, row_shard_count
    o.row_offset, o.N_total = row_offset, N_total
    o.exchanges_per_sweep = exchanges_per_sweep
    if log is not None:
        cb = LOG_FN(lambda msg, _u: log(msg.decode()))
        o.log = cb
        o._cb = cb  # keep the callback alive with the struct
    return o
