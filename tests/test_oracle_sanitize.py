"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer: every entry
point of prepsubband_oracle.c and sp_oracle.c run by oracle/oracle_selftest.c on small
synthetic cases (8/4/16-bit, both band orders, masks, clipping, downsampling, padding, the
single-pulse hits); any report aborts the run."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


def test_oracle_clean_under_asan_ubsan():
    if shutil.which("make") is None or shutil.which(os.environ.get("CC", "cc")) is None:
        pytest.skip("no C toolchain")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(["make", "-s", "-C", ORACLE, "selftest"], capture_output=True, text=True, timeout=300, env=env)
    if r.returncode and "cannot find -lasan" in (r.stderr + r.stdout):
        pytest.skip("sanitizer runtime not installed")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "oracle selftest ok" in r.stdout
