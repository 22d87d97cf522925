"""SURVEY.md §5 'Race detection / sanitizers': the host C of libhsfft.so (planner, plan
registry, pass scheduler, chunking, real and convolution drivers, per-device locks) built
with -fsanitize=address,undefined and with -fsanitize=thread against a null device
(tests/sanitize/null_device.c: computes nothing, touches the first and last element of every
row each launch would read or write), and run through tests/sanitize/sanitize_driver.c:
planner bytes vs the oracle for N <= 3000, every schedule family, edited plans, 8 host
threads sharing plans and cycling the convolution plan cache, and hsfft_exec_multi over 4
null devices (one host thread per device).  CPU only."""
import os
import subprocess

import pytest

import hsfft_testlib as T

SAN = os.path.join(T.REPO, "tests", "sanitize")


@pytest.mark.parametrize("target", ["sanitize_asan", "sanitize_tsan"])
def test_host_code_under_sanitizer(target):
    subprocess.check_call(["make", "-s", "-C", SAN, target])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1", HSFFT_NULL_NDEV="4")
    r = subprocess.run([os.path.join(SAN, target)], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "sanitize: ok" in r.stdout
    assert "runtime error" not in r.stderr        # UBSan
    assert "WARNING: ThreadSanitizer" not in r.stderr
