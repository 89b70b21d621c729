"""Pin the oracle (oracle/crc32_oracle.c) before trusting it as the checker.

Pins: the golden fixtures (zlib-derived, tests/golden/make_golden.py), the
reference's own literal tests (rust_client/tests/client_test.rs:169-218), and --
when the reference checkout is present in this container -- the 256 table
constants of the reference's default-build path (client/checksum.cc:79-122).
"""
import json
import re
import zlib
from pathlib import Path

import numpy as np
import pytest

GOLDEN = json.loads((Path(__file__).parent / "golden" / "golden.json").read_text())
REFERENCE_CHECKSUM_CC = Path("/root/reference/client/checksum.cc")
M32 = 0xFFFFFFFF


def test_table_is_reflected_ieee(oracle):
    t = oracle.table()
    assert t[1] == 0x77073096 and t[128] == 0xEDB88320 and t[255] == 0x2D02EF8D


@pytest.mark.skipif(not REFERENCE_CHECKSUM_CC.exists(), reason="reference checkout not present")
def test_table_matches_reference_source(oracle):
    """Compare with the constants in client/checksum.cc:79-122 (read as text, not copied)."""
    src = REFERENCE_CHECKSUM_CC.read_text()
    body = src[src.index("crc32_table[256]"):]
    body = body[:body.index("};")]
    ref = [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]{8})", body)]
    assert len(ref) == 256
    assert ref == oracle.table()


def test_kats(oracle):
    for k in GOLDEN["kat"]:
        d = bytes.fromhex(k["data_hex"])
        assert oracle.crc32(M32, d) == k["raw"]
        assert (~oracle.crc32(M32, d)) & M32 == k["final"]


def test_reference_literal_tests(oracle):
    # rust_client/tests/client_test.rs:169-173, 175-180
    assert oracle.crc32(M32, b"") == 0xFFFFFFFF
    assert (~oracle.crc32(M32, b"hello")) & M32 == 0x3610A686
    # :183-191 incremental == one-shot
    assert oracle.crc32(oracle.crc32(M32, b"hello "), b"world") == oracle.crc32(M32, b"hello world")
    # :213-218 single span == multi span
    assert oracle.checksum([b"foobar"]) == oracle.checksum([b"foo", b"bar"])
    # :194-203 calculate / verify / flipped
    c = int.from_bytes(oracle.checksum([b"subspace", b"ipc"]), "little")
    assert c != 0


def test_prefix_lengths(oracle):
    g = GOLDEN["prefix_lengths"]
    buf = bytes.fromhex(g["buffer_hex"])
    assert oracle.synth_bytes(g["seed"], g["msg"], len(buf)) == buf
    for n, raw in enumerate(g["raw"]):
        assert oracle.crc32(M32, buf[:n]) == raw, n


def test_long_lengths(oracle):
    for g in GOLDEN["long_lengths"]:
        assert oracle.synth_crc(g["seed"], g["msg"], g["length"]) == g["raw"]


def test_raw_states(oracle):
    for g in GOLDEN["raw_states"]:
        assert oracle.crc32(g["state"], bytes.fromhex(g["data_hex"])) == g["raw"]


def test_three_span(oracle):
    for g in GOLDEN["three_span"]:
        prefix = bytes.fromhex(g["prefix_hex"])
        cs, ms = g["checksum_size"], g["metadata_size"]
        spans = [prefix[4:48], prefix[48 + cs:48 + cs + ms], bytes.fromhex(g["payload_hex"])]
        assert oracle.checksum(spans).hex() == g["checksum_le_hex"]


def test_checksum20(oracle):
    g = GOLDEN["checksum20"]
    prefix = bytes.fromhex(g["prefix_hex"])
    spans = [prefix[4:48], b"", bytes.fromhex(g["payload_hex"])]
    for k, want in enumerate(g["values"]):
        crc = M32 ^ ((k * 0x11111111) & M32)
        for s in spans:
            crc = oracle.crc32(crc, s)
        assert (~crc) & M32 == want


def test_oracle_equals_zlib_random(oracle):
    rng = np.random.default_rng(7)
    for _ in range(300):
        n = int(rng.integers(0, 3000))
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert oracle.crc32(s, d) == (~zlib.crc32(d, (~s) & M32)) & M32


def test_synth_generators_agree(oracle):
    from subspace_amd import synth
    for msg, start, n in [(0, 0, 100), (5, 3, 77), (1 << 20, 8, 4096), (123456, 1001, 333)]:
        assert synth.synth_bytes(0x5EED000C, msg, n, start) == oracle.synth_bytes(0x5EED000C, msg, n, start)
    assert np.array_equal(synth.ragged_lengths(0x5EED000C, 500), oracle.ragged_lengths(0x5EED000C, 500))
    lens = synth.ragged_lengths(0x5EED000C, 20000)
    assert lens.min() >= 64 and lens.max() < (1 << 20)


def test_batch_threads_consistent(oracle):
    rng = np.random.default_rng(3)
    base = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    offs = rng.integers(0, 1 << 15, 200).astype(np.uint64)
    lens = rng.integers(0, 1 << 15, 200).astype(np.uint64)
    a = oracle.crc32_batch(base, offs, lens, threads=1)
    b = oracle.crc32_batch(base, offs, lens, threads=4)
    assert np.array_equal(a, b)
    for i in range(0, 200, 37):
        o, n = int(offs[i]), int(lens[i])
        assert a[i] == oracle.crc32(M32, base[o:o + n].tobytes())
