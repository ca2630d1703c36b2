"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer:
oracle/selftest.c drives every oracle entry point (random-map episodes with deadlocks and
boxed-in agents, dense warehouses, fixed resets, A*, BFS, GAE, the eviction-order sets);
any sanitizer report or broken invariant fails it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_and_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "selftest_asan")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "selftest: OK" in r.stdout
