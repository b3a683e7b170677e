"""Build libbrr.so in-tree for gfx950 (hipcc), and the test oracle (gcc).

The shared library is the product: HIP kernels (brr_kernels.hip) + host session / C ABI
(brr_session.cpp, brr_oneshot.cpp).  It links only the HIP runtime (no torch), so the same
.so is what an R package or any other FFI loads.
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libbrr.so")
SOURCES = ["brr_kernels.hip", "brr_session.cpp", "brr_oneshot.cpp"]
HEADERS = ["brr_device.hpp", "brr_launch.hpp", "brr_rng.hpp", "brr_chain.hpp", "brr_sample.hpp", "brr_ovsolve.hpp"]
ARCH = os.environ.get("BRR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build the MI355X library")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(p) > t for p in deps)


def build_library(force: bool = False, verbose: bool = False, out: str | None = None,
                  defines: list[str] | None = None) -> str:
    """Build libbrr.so (or a kernel variant at `out` with extra -D `defines`)."""
    target = out or LIB_PATH
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(REPO, "include", "brr.h"))
    if not force and not _stale(target, deps):
        return target
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-o", target + ".tmp"] + [f"-D{x}" for x in (defines or [])] + [
        os.path.join(CSRC, f) for f in SOURCES] + [
        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(target + ".tmp", target)
    return target


def build_oracle() -> str | None:
    """Compile the CPU oracle (test infrastructure) with its own Makefile."""
    mk = os.path.join(REPO, "oracle", "Makefile")
    if not os.path.exists(mk):
        return None
    subprocess.run(["make", "-s", "-C", os.path.dirname(mk)], check=True)
    return os.path.join(REPO, "oracle", "_build", "liboracle.so")


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
    print(build_oracle())
