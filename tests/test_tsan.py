"""The host code under ThreadSanitizer (the reference runs its tests
under tsan in CI): `make tsan-test` builds the library's host sources and capi.hip's host
side with -fsanitize=thread and runs tools/tsan_stress.cpp, which calls SubspaceCRC32 /
SubspaceCRC32C (first use included), the split-buffer allocator callbacks, the thread-local
error string and host registration from 8 threads at once. Any race report aborts."""
import os
import shutil
from pathlib import Path
import subprocess

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(not Path("/opt/rocm/llvm/bin/clang++").exists() or shutil.which("make") is None
                    or not Path("/opt/rocm/lib/libamdhip64.so").exists(),
                    reason="needs ROCm's clang and the HIP runtime library")
@pytest.mark.skipif(bool(os.environ.get("SUBSPACE_CRC_ASAN_DIR")), reason="running under asan-test")
def test_host_code_under_tsan():
    r = subprocess.run(["make", "-C", str(ROOT), "-j8", "tsan-test"], capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ThreadSanitizer" not in out, out[-4000:]
    assert "8 threads x 200 iterations, 0 failures" in out
