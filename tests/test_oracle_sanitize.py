"""The oracle built with AddressSanitizer + UndefinedBehaviorSanitizer (host only), driven over
every window kind, API, aggregation phase and value type with NULLs, NaN / +-0.0, late records,
flushes and snapshot/restore cuts (oracle/san_driver.cpp).  Any sanitizer report aborts the
driver, so a clean exit is the assertion."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "san"], check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([os.path.join(ORACLE, "san_driver")], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = dict(l.split() for l in p.stdout.strip().splitlines())
    for name in ("sql_tumble", "sql_hop", "sql_cumulate", "sql_two_phase_hop", "ds_tumble", "ds_sliding"):
        assert int(lines[name]) > 0, name
