"""CPU tests of the C ABI boundary: libbrr.so builds for gfx950, loads, exports every symbol
include/brr.h declares, and fails loudly (no CPU fallback) when no HIP device is present."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "brr.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(brr_[A-Za-z0-9_]+)\s*\(", txt)) - {"brr_log_fn"})


def test_library_exports_every_header_symbol(brr):
    out = subprocess.run(["nm", "-D", "--defined-only", brr.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (brr_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, f"declared in brr.h but not exported: {missing}"
    from bayesrrcpp_amd import _lib
    assert sorted(_lib.EXPORTED) == sorted(header_symbols())


def test_library_contains_gfx950_code(brr):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={brr.LIB_PATH}"], capture_output=True, text=True)
    blob = open(brr.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_device_fails_loudly(brr):
    L = brr.lib()
    if L.brr_device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(brr.BrrError, match="no HIP device"):
        brr.Session(brr.MODEL_V2, 10, 10, K=4)


def test_oneshot_without_device_returns_error(brr, tmp_path):
    L = brr.lib()
    if L.brr_device_count() > 0:
        pytest.skip("a HIP device is visible")
    msgs = []
    X = np.ones((5, 3))
    with pytest.raises(brr.BrrError):
        brr.BayesRSamplerV2(str(tmp_path / "o.csv"), 1, 10, 5, 1, X, np.ones(5), 0.01, 1e-4, 1e-3,
                            1e-4, 1e-3, [1e-4, 1e-3, 1e-2], log=msgs.append)


def test_validation_precedes_device(brr, tmp_path):
    """Reference semantics: an invalid iteration setting is reported and returns status 1 before
    any sampling (BayesRv2.cpp:76-80) -- even without a device; V2 writes the header first."""
    msgs = []
    p = str(tmp_path / "bad.csv")
    rc = brr.lib().brr_BayesRSamplerV2(p.encode(), 1, 5, 10, 1,
                                        np.ones(6).ctypes.data_as(C.POINTER(C.c_double)), 3, 2,
                                        np.ones(3).ctypes.data_as(C.POINTER(C.c_double)),
                                        0.01, 1e-4, 1e-3, 1e-4, 1e-3,
                                        np.array([1e-3, 1e-2]).ctypes.data_as(C.POINTER(C.c_double)), 2,
                                        C.byref(__import__("bayesrrcpp_amd")._lib.options(log=msgs.append)))
    assert rc == 1
    assert any("burn_in has to be a positive integer" in m for m in msgs)
    assert open(p).read().startswith("iteration,mu,beta[1],beta[2],sigmaE,sigmaG,comp[1],comp[2],")
    # HorseshoeR validates before opening the file (HorseshoeR.cpp:119-123)
    p2 = str(tmp_path / "hs.csv")
    rc = brr.lib().brr_HorseshoeR(p2.encode(), 1, 5, 0, 1,
                                   np.ones(6).ctypes.data_as(C.POINTER(C.c_double)), 3, 2,
                                   np.ones(3).ctypes.data_as(C.POINTER(C.c_double)),
                                   1.0, 1e-3, 1e-3, 1.0, 1.0, 1.0, 10.0, 10.0,
                                   C.byref(__import__("bayesrrcpp_amd")._lib.options(log=msgs.append)))
    assert rc == 1 and not os.path.exists(p2)


def test_header_compiles_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "brr.h"\nint main(void){brr_options o; brr_options_default(&o); return o.block_size == 128 ? 0 : 1;}\n')
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{REPO}/include", "-c", str(src),
                        "-o", str(tmp_path / "t.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_options_struct_layout(brr, tmp_path):
    # the ctypes mirror has the C compiler's layout of brr_options (ABI 2: row-shard fields, ABI 3:
    # exchanges_per_sweep, 0 = automatic)
    from bayesrrcpp_amd import _lib
    o = _lib.options()
    assert o.abi_version == _lib.ABI_VERSION == 4
    assert o.row_shard_count == 1 and o.row_shard_rank == 0 and o.N_total == 0
    assert o.exchanges_per_sweep == 0  # automatic (column shards: E = 8, capped at the blocks per shard)
    src = tmp_path / "lay.c"
    fields = [f[0] for f in _lib.Options._fields_]
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "brr.h"\nint main(void){'
                   'printf("%zu", sizeof(brr_options));'
                   + "".join(f'printf(" %zu", offsetof(brr_options, {f}));' for f in fields)
                   + 'return 0;}\n')
    exe = tmp_path / "lay"
    r = subprocess.run(["gcc", "-std=c99", f"-I{REPO}/include", str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert got[0] == C.sizeof(_lib.Options)
    assert got[1:] == [getattr(_lib.Options, f).offset for f in fields]


@pytest.mark.parametrize("abi,given,want", [(4, 0, 0), (4, 3, 3), (3, 0, 0), (3, 5, 5), (2, 7, 0), (1, 7, 0)])
def test_older_abi_exchanges_per_sweep(brr, abi, given, want):
    # exchanges_per_sweep = 0 is automatic (E = 8) for every ABI, as ABI 3's header documented it; a
    # caller built against ABI 1 / 2 has no such field (whatever follows its struct is not read) and
    # gets that default
    from bayesrrcpp_amd import _lib
    L = brr.lib()
    o = _lib.options(block_size=256, shard_count=2)
    o.abi_version, o.exchanges_per_sweep = abi, given
    out = _lib.Options()
    L.brr_options_effective(C.byref(o), C.byref(out))
    assert out.abi_version == _lib.ABI_VERSION
    assert out.exchanges_per_sweep == want
    assert out.shard_count == 2
    assert out.block_size == 256
    assert out.row_shard_count == 1
    L.brr_options_effective(None, C.byref(out))  # NULL: the defaults
    assert out.exchanges_per_sweep == 0 and out.shard_count == 1
