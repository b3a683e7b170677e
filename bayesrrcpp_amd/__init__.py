"""bayesrrcpp_amd -- MI355X-native BayesR / BayesRR / Horseshoe Gibbs sampler.

Drop-in for the per-marker Gibbs sweep of medical-genomics-group/BayesRRcpp
(BayesRSamplerV2, BayesRSamplerV2Groups, BRV2Grstart, HorseshoeR).  The compute path is
libbrr.so (HIP kernels for gfx950 + a C ABI, include/brr.h); this package is a thin ctypes
mirror of the reference's interface on top of it.  Importing it does not touch the GPU; the
first call loads libbrr.so and fails loudly if the library or a HIP device is missing.
"""
from ._lib import (ABI_VERSION, BrrError, MODEL_GROUPS, MODEL_HORSESHOE, MODEL_RESTART,
                   MODEL_V2, ORDER_BLOCKED, ORDER_IDENTITY, ORDER_REFERENCE, lib)
from .build import LIB_PATH, build_library
from .samplers import BRV2Grstart, BayesRSamplerV2, BayesRSamplerV2Groups, HorseshoeR
from .session import Group, Session

__all__ = [
    "ABI_VERSION", "BrrError", "MODEL_V2", "MODEL_GROUPS", "MODEL_RESTART", "MODEL_HORSESHOE",
    "ORDER_BLOCKED", "ORDER_REFERENCE", "ORDER_IDENTITY", "lib", "LIB_PATH", "build_library",
    "BayesRSamplerV2", "BayesRSamplerV2Groups", "BRV2Grstart", "HorseshoeR", "Session", "Group",
]
