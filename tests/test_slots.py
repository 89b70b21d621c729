"""Slot layout and the slot-checksum oracle (CPU).

The oracle's publisher/subscriber restatement (oracle/crc32_oracle.c oracle_publish_slot /
oracle_verify_slot) is pinned here against
  * zlib (independent CRC) over the spans of common/channel.h:527-542, and
  * the reference's own checksum-coverage tests, client/client_test.cc:5646-5880
    (ChecksumWithMetadata*, ChecksumIgnoresPrefixPadding*), restated as byte edits.
"""
import zlib

import numpy as np
import pytest

from subspace_amd import checksum, slots

M32 = 0xFFFFFFFF


def test_prefix_layout_matches_reference():
    # common/channel.h:88-112 field offsets
    f = slots.PREFIX_DTYPE.fields
    want = {"padding": 0, "slot_id": 4, "message_size": 8, "ordinal": 16, "timestamp": 24, "flags": 32,
            "vchan_id": 40, "checksum_size": 44, "metadata_size": 46, "checksum": 48, "padding3": 52}
    assert {k: f[k][1] for k in want} == want
    assert slots.PREFIX_DTYPE.itemsize == 64


@pytest.mark.parametrize("cs,ms,want", [(4, 0, 64), (4, 16, 128), (20, 32, 128), (32, 0, 128), (20, 50, 128),
                                        (4, 12, 64), (4, 13, 128)])
def test_prefix_size(cs, ms, want):
    # client_test.cc:5654 (4,16)->128, :5836 (20,32)->128, :5288 (32,0)->128, bridge_test.cc:877 (20,50)->128
    assert slots.compute_prefix_size(cs, ms) == want


def test_slot_stride():
    # client_channel.h:130-132: PrefixSize + Aligned<64>(SlotSize); 4 KiB payloads -> 4160
    assert slots.slot_stride(4096) == 4160
    assert slots.slot_stride(256, 4, 16) == 128 + 256
    assert slots.slot_stride(100, 20, 32) == 128 + 128


def _slot(payload: bytes, meta: bytes, cs: int, slot_size: int = 256, seed: int = 1):
    ms = len(meta)
    ps = slots.compute_prefix_size(cs, ms)
    buf = np.zeros(ps + slot_size, dtype=np.uint8)
    buf[:ps] = slots.make_prefixes(1, [len(payload)], checksum_size=cs, metadata_size=ms, seed=seed)[0]
    buf[48 + cs:48 + cs + ms] = np.frombuffer(meta, dtype=np.uint8)
    buf[ps:ps + len(payload)] = np.frombuffer(payload, dtype=np.uint8)
    return buf, ps


def _zlib_checksum(buf, ps, n, cs, ms) -> int:
    data = bytes(buf[4:48]) + bytes(buf[48 + cs:48 + cs + ms]) + bytes(buf[ps:ps + n])
    return zlib.crc32(data) & M32  # = ~chain(0xFFFFFFFF, spans)


def _publish(oracle, buf, ps, n, cs, ms):
    oracle.publish_slots(buf, [0], [ps], [n], cs, ms)


def _verify(oracle, buf, ps, n, cs, ms) -> int:
    return int(oracle.verify_slots(buf, [0], [ps], [n], cs, ms)[0])


def test_publish_matches_zlib_and_host_mirror(oracle):
    for cs, meta, payload in [(4, b"", b"hello"), (4, b"META_CHECKSUM!!\0", b"hello"),
                              (20, bytes(range(32)), b"bigpad"), (4, b"x" * 7, bytes(range(256)) * 0)]:
        ms = len(meta)
        buf, ps = _slot(payload, meta, cs)
        _publish(oracle, buf, ps, len(payload), cs, ms)
        flags = int(buf[32:40].view(np.int64)[0])
        assert flags & 4, "SetHasChecksum before the CRC"
        stored = int(buf[48:52].view(np.uint32)[0])
        assert stored == _zlib_checksum(buf, ps, len(payload), cs, ms)
        # host mirror of client/checksum.h over GetMessageChecksumData (native SubspaceCRC32)
        spans = checksum.get_message_checksum_data(buf[:ps], buf[ps:], len(payload), cs, ms)
        assert checksum.calculate_crc32_checksum(spans) == bytes(buf[48:52])
        assert checksum.verify_crc32_checksum(spans, bytes(buf[48:52]))
        assert _verify(oracle, buf, ps, len(payload), cs, ms) == 0


def test_reference_coverage_cases(oracle):
    """client_test.cc:5684-5880 as byte edits on a published slot (status 0 ok, 1 error)."""
    cases = {
        "corrupt_payload": (lambda b, ps, cs, ms: b.__setitem__(ps, ord("X")), 1),      # :5708
        "corrupt_metadata_first": (lambda b, ps, cs, ms: b.__setitem__(48 + cs, 0xFF), 1),   # :5740
        "corrupt_metadata_last": (lambda b, ps, cs, ms: b.__setitem__(48 + cs + ms - 1, b[48 + cs + ms - 1] ^ 1), 1),
        "scribble_prefix_padding": (lambda b, ps, cs, ms: b.__setitem__(slice(48 + cs + ms, ps), 0xAA), 0),  # :5815
        "scribble_padding_word": (lambda b, ps, cs, ms: b.__setitem__(slice(0, 4), 0x55), 0),  # channel.h:76-87
        "corrupt_span0_timestamp": (lambda b, ps, cs, ms: b.__setitem__(24, b[24] ^ 0x80), 1),
        "corrupt_checksum_word": (lambda b, ps, cs, ms: b.__setitem__(49, b[49] ^ 1), 1),
        "clear_flag": (lambda b, ps, cs, ms: b.__setitem__(32, b[32] & 0xFB), 2),            # client.cc:1347
    }
    for cs, ms in [(4, 16), (20, 32)]:
        meta = bytes((i * 7 + 3) & 0xFF for i in range(ms))
        for name, (edit, want) in cases.items():
            buf, ps = _slot(b"intact", meta, cs)
            _publish(oracle, buf, ps, 6, cs, ms)
            edit(buf, ps, cs, ms)
            assert _verify(oracle, buf, ps, 6, cs, ms) == want, (cs, ms, name)
    # checksum bytes beyond the first 4 are neither covered nor compared (checksum.h:46)
    buf, ps = _slot(b"bigpad", bytes(range(32)), 20)
    _publish(oracle, buf, ps, 6, 20, 32)
    buf[52:68] ^= 0xFF
    assert _verify(oracle, buf, ps, 6, 20, 32) == 0


def test_make_prefixes_fields():
    sizes = np.array([0, 5, 4096], dtype=np.uint64)
    blk = slots.make_prefixes(3, sizes, checksum_size=4, metadata_size=16, seed=3)
    assert blk.shape == (3, 128)
    head = blk[:, :64].copy().view(slots.PREFIX_DTYPE).reshape(3)
    assert list(head["message_size"]) == [0, 5, 4096]
    assert list(head["slot_id"]) == [0, 1, 2]
    assert all(int(f) & 4 == 0 for f in head["flags"])
    assert all(int(c) == 0 for c in head["checksum"])
    assert list(head["checksum_size"]) == [4, 4, 4] and list(head["metadata_size"]) == [16, 16, 16]
