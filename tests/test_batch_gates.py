"""The reference's checksum gates carried into the batched C++ helper:
ValidateChecksum (client/subscriber.h:264-275) returns true with checksums off and compares a
custom ChecksumCallback's full checksum_size bytes with memcmp; the publisher
(client/publisher.cc:664-675) defers to the callback too. tests/c/batch_gates.cpp publishes
three channels through include/subspace/checksum_batch.h (CRC32 with metadata, the 20-byte
Checksum20Byte callback of client/client_test.cc:5210-5272, checksums off) and checks a mixed,
shuffled drain against the reference's per-message decision.

CPU: the callback and checksum-off channels (no device is touched) and a clean error for a
CRC32 slot without a device. GPU: all three channels, the CRC32 group on the device."""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _binary():
    asan = os.environ.get("SUBSPACE_CRC_ASAN_DIR")
    if asan:
        return Path(asan) / "batch_gates"
    exe = ROOT / "tools" / "batch_gates"
    if not exe.exists():
        subprocess.run(["make", "-C", str(ROOT), "tools/batch_gates"], check=True)
    return exe


def _run(mode):
    r = subprocess.run([str(_binary()), mode], capture_output=True, text=True, timeout=300)
    return r.returncode, r.stdout.strip(), r.stderr[-3000:]


def test_gates_host_channels(lib):
    rc, out, err = _run("host")
    assert rc == 0, out + err
    assert '"failures": 0' in out and '"callback_mismatches": 3' in out


@pytest.mark.gpu
def test_gates_mixed_drain_gpu(lib):
    rc, out, err = _run("full")
    assert rc == 0, out + err
    assert '"failures": 0' in out and '"mode": "full"' in out
