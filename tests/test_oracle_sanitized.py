"""The C restatement under AddressSanitizer + UndefinedBehaviorSanitizer (a
-fsanitize=address host build of the CPU restatement).  oracle/dpt_oracle.c is the checker of
every full-size GPU test, so its own memory safety is checked here: `make -C oracle asan` builds
build/libdpt_oracle_asan.so and the reference-pinned C oracle tests run against it in a child
interpreter with the ASan runtime preloaded (a sanitizer report aborts the child: the test fails).
CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_c_oracle_clean_under_asan_ubsan():
    rt = _runtime()
    if rt is None:
        pytest.skip("no gcc ASan runtime on this host")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    lib = os.path.join(ROOT, "oracle", "build", "libdpt_oracle_asan.so")
    env = dict(os.environ, LD_PRELOAD=rt, DPT_ORACLE_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    # the child confirms it really runs the sanitized build, then the reference-pinned checks
    code = ("import sys, pytest; sys.path.insert(0, %r); from oracle import c_oracle; c_oracle.load(); "
            "maps = open('/proc/self/maps').read(); "
            "assert c_oracle._LIB == %r and 'libasan' in maps and 'libdpt_oracle_asan' in maps; "
            "sys.exit(pytest.main(['-q', '-x', '-p', 'no:cacheprovider', %r, '-k', "
            "'c_bandit_oracle or c_darkroom_oracle']))") % (ROOT, lib, os.path.join(ROOT, "tests",
                                                                                     "test_oracle_golden.py"))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "passed" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
