"""The CPU oracle built with AddressSanitizer + UndefinedBehaviorSanitizer
and driven through every path: the three visit orders, Groups with fixed effects, restart,
Horseshoe, the 2-shard emulation and exchange protocol, forced state and the four CSV writers
(oracle/sanitize_driver.c).  Any invalid access, leak or undefined operation aborts the driver."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(HERE, "..", "oracle")
CASES = ["v2 order 0", "v2 order 1", "v2 order 2", "groups G=3 F=2", "restart", "horseshoe",
         "horseshoe ref order", "v2 2-shard emulation", "v2 shard protocol", "v2 forced state"]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True)
    # (verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(ORACLE, "_build", "sanitize_driver"), str(tmp_path)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.splitlines()
    for c in CASES:
        assert any(l.startswith(c + " ") and "e+" in l or l.startswith(c + " ") and "e-" in l for l in lines), c
    for m in ("v2", "groups", "restart", "horseshoe"):
        assert (tmp_path / f"sanitize_{m}.csv").stat().st_size > 0
