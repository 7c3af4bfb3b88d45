"""Host sanitizers (SURVEY.md §5 "Race detection / sanitizers"): libvolkit's host code rebuilt
with AddressSanitizer + UBSan and with ThreadSanitizer, driven by tests/sanitize/host_driver.cpp
under the CPU execution policy (handles, accessors, codec, memory, streams, CPU-policy error
paths, concurrent per-thread policies / resource registry).  CPU only: GPU sanitizers are not
available on the GPU pool and the driver needs no device."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "sanitize")


@pytest.fixture(scope="module")
def drivers():
    jobs = str(min(8, os.cpu_count() or 1))
    # device kernels of the normal build, then the instrumented host objects + drivers
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "volkit_amd", "csrc")], check=True)
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tests", "sanitize")], check=True)
    return {k: os.path.join(OUT, f"host_driver_{k}") for k in ("asan", "tsan")}


def run(exe, tmp_path, env):
    e = dict(os.environ, **env)
    p = subprocess.run([exe, str(tmp_path)], env=e, capture_output=True, text=True, timeout=600)
    report = p.stdout + p.stderr
    return p.returncode, report


def test_address_and_undefined_behaviour(drivers, tmp_path):
    rc, report = run(drivers["asan"], tmp_path, {
        # the image may preload a helper library ahead of the ASan runtime
        "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
        "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
    })
    assert "ERROR: AddressSanitizer" not in report and "runtime error:" not in report, report[-4000:]
    assert "ERROR: LeakSanitizer" not in report, report[-4000:]
    assert rc == 0 and "0 failed checks" in report, report[-4000:]


def test_thread_sanitizer(drivers, tmp_path):
    rc, report = run(drivers["tsan"], tmp_path, {"TSAN_OPTIONS": "halt_on_error=0:exitcode=66"})
    assert "WARNING: ThreadSanitizer" not in report, report[-4000:]
    assert rc == 0 and "0 failed checks" in report, report[-4000:]
