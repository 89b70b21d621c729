"""CRC-32C (Castagnoli): the function a -msse4.2 x86 build of the reference computes in
SubspaceCRC32 (client/checksum.cc:56-76). CPU checks: the oracle's restatement and the
host SubspaceCRC32C against the published known answers (tests/golden/crc32c_kat.json),
and against each other on random data with raw-state chaining."""
import json
from pathlib import Path

import numpy as np

from subspace_amd import checksum

KAT = json.loads((Path(__file__).parent / "golden" / "crc32c_kat.json").read_text())["kats"]
M32 = 0xFFFFFFFF


def test_oracle_crc32c_known_answers(oracle):
    for k in KAT:
        data = bytes.fromhex(k["data_hex"])
        assert (~oracle.crc32c(M32, data)) & M32 == k["checksum"], k["name"]


def test_host_crc32c_known_answers():
    for k in KAT:
        data = bytes.fromhex(k["data_hex"])
        assert (~checksum.subspace_crc32c(M32, data)) & M32 == k["checksum"], k["name"]


def test_host_crc32c_matches_oracle_and_chains(oracle):
    rng = np.random.default_rng(32)
    for n in list(range(0, 70)) + [255, 256, 4095, 4096, 4097, 65537]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        want = oracle.crc32c(seed, data)
        assert checksum.subspace_crc32c(seed, data) == want, n
        cut = n // 3
        assert checksum.subspace_crc32c(checksum.subspace_crc32c(seed, data[:cut]), data[cut:]) == want, n


def test_crc32c_differs_from_ieee(oracle):
    assert oracle.crc32c(M32, b"123456789") != oracle.crc32(M32, b"123456789")


def test_sse42_restatement_matches_table_crc32c(oracle):
    """The informational -msse4.2 restatement (client/checksum.cc:56-76) computes CRC-32C:
    equal to the table restatement, and to the published check value."""
    import pytest
    if not oracle.has_sse42():
        pytest.skip("CPU without SSE4.2")
    assert (~oracle.crc32c_sse42(M32, b"123456789")) & M32 == 0xE3069283
    rng = np.random.default_rng(42)
    for n in (0, 1, 3, 4, 5, 7, 8, 9, 15, 16, 17, 100, 4096, 4099):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        assert oracle.crc32c_sse42(seed, data) == oracle.crc32c(seed, data), n
