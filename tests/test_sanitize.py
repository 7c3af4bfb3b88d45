"""Host sanitizers (SURVEY.md §5 "Race detection / sanitizers"): libvolkit's host code rebuilt
with AddressSanitizer + UBSan and with ThreadSanitizer, driven by tests/sanitize/host_driver.cpp
under the CPU execution policy (handles, accessors, codec, memory, streams, CPU-policy error
paths, concurrent per-thread policies / resource registry).  CPU only: GPU sanitizers are not
available on the GPU pool and the driver needs no device."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "sanitize")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _toolchain_missing():
    """Reason to skip, or None: the sanitizer builds need hipcc, make, the clang sanitizer
    runtimes and roctx (libvolkit links it)."""
    if not (os.access(HIPCC, os.X_OK) or shutil.which("hipcc")):
        return f"hipcc not found ({HIPCC})"
    if not shutil.which("make"):
        return "make not found"
    for rt in ("asan", "tsan"):
        if not glob.glob(f"/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.{rt}-x86_64.a"):
            return f"clang {rt} runtime not installed"
    if not glob.glob("/opt/rocm/lib/libroctx64.so*") and not glob.glob("/opt/rocm/lib/librocprofiler-sdk-roctx.so*"):
        return "roctx library not installed"
    return None


@pytest.fixture(scope="module")
def drivers():
    reason = _toolchain_missing()
    if reason:
        pytest.skip(reason)
    jobs = str(min(8, os.cpu_count() or 1))
    # device kernels of the normal build, then the instrumented host objects + drivers; a build
    # failure is reported as such (not as a sanitizer finding)
    for d in (os.path.join(ROOT, "volkit_amd", "csrc"), os.path.join(ROOT, "tests", "sanitize")):
        p = subprocess.run(["make", "-s", "-j", jobs, "-C", d], capture_output=True, text=True)
        if p.returncode != 0:
            pytest.fail(f"sanitizer build failed in {d} (not a sanitizer report):\n{p.stderr[-4000:]}",
                        pytrace=False)
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
