"""Host sanitizers over the multithreaded C++ runtime (ThreadSanitizer, AddressSanitizer + UBSan)."""
import os
import subprocess

import pytest

from oni_ml_amd import _build


@pytest.mark.parametrize("kind", ["thread", "address"])
def test_native_runtime_under_sanitizer(kind, tmp_path):
    exe = _build.build_sanitized(kind)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "native selftest: ok" in r.stdout
