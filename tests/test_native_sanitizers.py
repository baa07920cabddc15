"""Host-side sanitizer runs of the native runtime.

GPU AddressSanitizer / xnack+ is not available on the MI355X pool, so the
C++ runtime's host logic is checked here on the CPU: the token loader core
(csrc/runtime/token_loader_core.h — the same code the torch class wraps) is
compiled into a standalone driver under AddressSanitizer + UBSan and under
ThreadSanitizer (its producer thread, restore() racing it, shutdown while
blocked), and must finish with zero reports.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "test_loader_core.cpp")


def _build_and_run(tmp_path, flags, name):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", f"-I{os.path.join(ROOT, 'csrc')}",
           *flags, SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "loader core: ok" in out
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "runtime error:" not in out  # UBSan


def test_loader_core_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined"], "loader_asan")


def test_loader_core_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], "loader_tsan")
