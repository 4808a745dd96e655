"""Sanitizer builds of the C++ runtime (SURVEY.md §5 "Race detection / sanitizers"): the KV store
and the TCP ring collectives under ASan+UBSan and under TSan, exercised by a standalone driver
(csrc/native/tests/native_selftest.cpp) with ranks as threads over localhost TCP.  Each build is
also checked to be live: a deliberate data race / out-of-bounds read must be reported."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import build_native  # noqa: E402

pytestmark = pytest.mark.timeout(600)


def _binary(kind):
    return build_native.build_selftest(kind)


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=0")
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env)


@pytest.mark.parametrize("kind,marker", [("address", "AddressSanitizer"), ("thread", "ThreadSanitizer")])
def test_runtime_clean_under_sanitizer(kind, marker):
    r = _run(_binary(kind))
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "native selftest ok" in r.stdout
    assert marker not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]


@pytest.mark.parametrize("kind,defect,marker", [("address", "oob", "heap-buffer-overflow"),
                                                ("thread", "race", "data race")])
def test_sanitizer_build_is_live(kind, defect, marker):
    r = _run(_binary(kind), defect)
    assert r.returncode != 0 and marker in r.stderr, r.stderr[-2000:]
