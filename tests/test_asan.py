"""The host code under AddressSanitizer + UBSan: `make asan-test`
builds the sanitized library with ROCm's clang -- the host CRC incl. the PCLMULQDQ body, the
split-buffer allocator and capi.hip's host side (hipcc -Xarch_host -fsanitize=...: argument
validation, workspace sizing, the host-slot pipeline, the call scope) -- plus tools/config_a,
tools/drain_demo, the C-client binding (tests/c/c_binding.c) and tests/c/batch_gates.cpp,
and runs test_host_api.py, test_capi.py, test_split_alloc.py, test_c_binding.py and
test_batch_gates.py against them with clang's ASan runtime preloaded (any finding aborts)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None or not Path("/opt/rocm/lib/libamdhip64.so").exists(),
                    reason="needs g++ and the HIP runtime library")
@pytest.mark.skipif(bool(os.environ.get("SUBSPACE_CRC_ASAN_DIR")), reason="already running under asan-test")
def test_host_code_under_asan_and_ubsan():
    r = subprocess.run(["make", "-C", str(ROOT), "-j8", "asan-test"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert " passed" in r.stdout and "failed" not in r.stdout.splitlines()[-1]
    # capi.hip's host side is instrumented, not linked in plain
    nm = subprocess.run(["nm", str(ROOT / "build" / "asan" / "capi.o")], capture_output=True, text=True)
    assert "__asan_" in nm.stdout and "__ubsan_" in nm.stdout
