"""Race / memory-safety checks of the native host code (the reference has none).

The token loader's threading core (csrc/token_loader.h) is compiled standalone with ThreadSanitizer
and with AddressSanitizer+UBSan and stress-tested by tests/native/test_token_loader.cpp (workers
racing for ring slots, mid-stream set_state restarts, epoch reshuffles, destruction while producers
are blocked).  Host code only: GPU sanitizers are not available on the target pool.
"""

import os
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "test_token_loader.cpp")


def _build_and_run(flags, tag):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tempfile.mkdtemp()
    exe = os.path.join(d, tag)
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-pthread", *flags, SRC, "-o", exe], check=True,
                   capture_output=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, os.path.join(d, "corpus.bin")], capture_output=True, text=True, timeout=600, env=env)
    shutil.rmtree(d, ignore_errors=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "token_loader stress OK" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_token_loader_tsan():
    _build_and_run(["-fsanitize=thread"], "tl_tsan")


def test_token_loader_asan_ubsan():
    _build_and_run(["-fsanitize=address,undefined", "-fno-omit-frame-pointer"], "tl_asan")
