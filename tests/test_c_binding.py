"""The C client binding of INTEGRATION.md section 3 (tests/c/c_binding.c), compiled and
run: the SubspaceChecksumCallback stub (c_client/subspace.h:129-136) over
libsubspace_crc.so's SubspaceCRC32 stores exactly the oracle's CalculateCRC32Checksum value
for every message (spans of every length 0..300 and around the 16-B folding boundaries,
any alignment: each span is its own exact-size allocation), and the split-buffer callbacks
have the reference C client's signatures (c_client/subspace.h:140-158). Under `make
asan-test` the same program is the AddressSanitizer + UBSan build (build/asan/c_binding)."""
import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _binary(tmp_path):
    asan = os.environ.get("SUBSPACE_CRC_ASAN_DIR")
    if asan:
        return Path(asan) / "c_binding"
    exe = tmp_path / "c_binding"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror=incompatible-pointer-types", "-O1",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "c" / "c_binding.c"), "-o", str(exe),
                    f"-L{ROOT / 'subspace_amd'}", "-lsubspace_crc", f"-Wl,-rpath,{ROOT / 'subspace_amd'}"],
                   check=True)
    return exe


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_c_checksum_callback_matches_oracle(lib, oracle, tmp_path):
    exe = _binary(tmp_path)
    rng = np.random.default_rng(0xCB)
    msgs = []
    for n in list(range(0, 301)) + [1023, 1024, 1025, 4095, 4096, 4097, 65536 + 7]:
        msgs.append([rng.integers(0, 256, n, dtype=np.uint8).tobytes()])
    for _ in range(200):  # three spans, as GetMessageChecksumData passes them (common/channel.h:527-542)
        msgs.append([rng.integers(0, 256, int(k), dtype=np.uint8).tobytes()
                     for k in (44, rng.integers(0, 40), rng.integers(0, 9000))])
    stdin = "\n".join(" ".join(s.hex() if s else "-" for s in m) for m in msgs) + "\n"
    r = subprocess.run([str(exe)], input=stdin, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = [int(x) for x in r.stdout.split()]
    want = [int.from_bytes(oracle.checksum(m), "little") for m in msgs]
    assert got == want
