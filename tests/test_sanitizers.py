"""Race detection / memory safety of the native host runtime (SURVEY.md §5:
the reference runs `go test -race`, .github/workflows/go.yml:27).

Builds csrc/tests/stress_native.cpp (MultiLevelQueue, DelayedQueue, ShmRing
under concurrent producers/consumers) with ThreadSanitizer and with
AddressSanitizer+UBSan, host code only, and requires a clean run.

Compiler: ROCm's clang++.  GCC 11's libtsan does not intercept
``pthread_cond_clockwait`` (used by libstdc++'s steady-clock ``wait_for``),
which makes every condition-variable wait look like a race; LLVM's runtime
handles it.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "llvm", "bin", "clang++")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_native_runtime_under_sanitizer(san, tmp_path):
    cxx = CLANG if os.path.exists(CLANG) else shutil.which("clang++")
    if cxx is None:
        pytest.skip("clang++ not available")
    exe = str(tmp_path / "stress")
    src = os.path.join(ROOT, "csrc", "tests", "stress_native.cpp")
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           f"-I{os.path.join(ROOT, 'csrc')}", src, "-o", exe, "-lrt", "-lcrypto", "-pthread"]
    if "undefined" in san:
        cmd.insert(5, "-fno-sanitize-recover=undefined")
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66",
               ASAN_OPTIONS="detect_leaks=1 halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ALL OK" in out and "WARNING:" not in out and "runtime error" not in out, out[-4000:]
