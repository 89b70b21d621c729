"""The host code under AddressSanitizer + UBSan: `make asan-test`
builds the sanitized library (host CRC incl. the PCLMULQDQ body, split-buffer allocator,
C-ABI argument checks), tools/config_a, tools/drain_demo and the C-client binding
(tests/c/c_binding.c) with -fsanitize=address,undefined, and runs test_host_api.py,
test_capi.py, test_split_alloc.py and test_c_binding.py against them (any finding aborts)."""
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
