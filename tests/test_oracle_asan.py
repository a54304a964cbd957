"""The C restatement (oracle/sgm_ref.c) under AddressSanitizer + UBSan: builds
oracle/asan_check (make -C oracle asan) and runs its sweep of small shapes (narrow
images, one-row images, negative minDisparity, blockSize up to 23, BGR, census,
5/8 paths, speckles, the f32 volume entry).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_under_asan_ubsan():
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in (b.stderr or ""):
        pytest.skip("toolchain lacks the sanitizer runtimes: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(ROOT, "oracle", "asan_check")], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "asan_check ok" in r.stdout
