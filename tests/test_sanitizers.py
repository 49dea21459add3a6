"""Sanitizer builds of the host-side native code (SURVEY.md §5 "Race detection / sanitizers"),
on the CPU: tests/sanitize/Makefile builds
  * host_asan / host_tsan: csrc/rsac_host.hip -- the scan and its device-record replay, the OpenCV
    MWC subset sampler on the 16-thread parallel_for pool, the LM / EPnP / homography refits,
    Rodrigues -- under AddressSanitizer + UndefinedBehaviorSanitizer, and ThreadSanitizer;
  * oracle_asan: oracle/rsac_oracle.c, every loop of the CPU restatement incl. its OpenMP
    hypothesis loop, under AddressSanitizer + UndefinedBehaviorSanitizer (leak checks on).
Each harness also checks results (the parallel pool against sequential runs, the record replay
against the sequential scan); any sanitizer report fails the run."""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    out = tmp_path_factory.mktemp("sanitize")
    subprocess.run(["make", "-s", "-j3", "-C", HERE, f"OUT={out}"], check=True, timeout=600)
    return out


@pytest.mark.parametrize("exe,env", [("host_asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"}),
                                     ("host_tsan", {"TSAN_OPTIONS": "halt_on_error=1"}),
                                     ("oracle_asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})])
def test_sanitized_harness(built, exe, env):
    r = subprocess.run([str(built / exe)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="4", **env))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    for bad in ("ERROR: AddressSanitizer", "WARNING: ThreadSanitizer", "runtime error:", "ERROR: LeakSanitizer"):
        assert bad not in out, out[-3000:]
    assert "ok (0 failed checks)" in out
