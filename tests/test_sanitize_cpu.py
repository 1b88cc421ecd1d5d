"""ASan / UBSan runs of the host code (VERDICT r1 hygiene): the CPU restatement
(oracle/rc2dgi_oracle.c: whole frames in every mode plus row-restricted passes) and the row-strip
planner (csrc/rc2dgi_shard.cpp: plan_frame and the JumpFlood exchange over many sizes and shard
counts, with its invariants checked), built by tests/sanitize/Makefile with
-fsanitize=address,undefined (UB fatal).  GPU sanitizers are not available on this pool."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def built():
    if not shutil.which("gcc") or not shutil.which("g++"):
        pytest.skip("no host compiler")
    subprocess.run(["make", "-s", "-C", HERE], check=True)


@pytest.mark.parametrize("exe", ["oracle_asan", "plan_asan"])
def test_sanitized_run_is_clean(built, exe):
    r = subprocess.run([os.path.join(HERE, exe)], capture_output=True, text=True, env=ENV, timeout=600)
    report = r.stdout[-2000:] + r.stderr[-4000:]
    assert r.returncode == 0, report
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, report
