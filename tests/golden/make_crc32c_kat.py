#!/usr/bin/env python3
"""Writes tests/golden/crc32c_kat.json: CRC-32C known answers (checksum = ~crc(~0, data)).

Expected values are published ones, not computed here; the script only cross-checks them
against a bitwise restatement of the reflected Castagnoli polynomial before writing.
Sources:
  * "123456789" -> 0xE3069283: the CRC-32C check value (CRC catalogue "CRC-32/ISCSI");
    also what the reference's -msse4.2 build of client/checksum.cc returned in this
    container;
  * "hello" -> 0x9A71BB4C: the reference's -msse4.2 build;
  * RFC 3720 appendix B.4: 32 bytes of 0x00 / 0xFF / 00..1F / 1F..00.
"""
import json
from pathlib import Path

KATS = [
    ("check", b"123456789", 0xE3069283, "CRC-32/ISCSI check value; reference -msse4.2 build (SURVEY 8c)"),
    ("hello", b"hello", 0x9A71BB4C, "reference -msse4.2 build (SURVEY 8c)"),
    ("zeros32", bytes(32), 0x8A9136AA, "RFC 3720 B.4"),
    ("ones32", b"\xff" * 32, 0x62A8AB43, "RFC 3720 B.4"),
    ("incrementing32", bytes(range(32)), 0x46DD794E, "RFC 3720 B.4"),
    ("decrementing32", bytes(range(31, -1, -1)), 0x113FDB5C, "RFC 3720 B.4"),
]


def crc32c_bitwise(data, crc=0xFFFFFFFF):
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def main():
    out = []
    for name, data, want, src in KATS:
        assert crc32c_bitwise(data) == want, name
        out.append({"name": name, "data_hex": data.hex(), "checksum": want, "source": src})
    path = Path(__file__).with_name("crc32c_kat.json")
    path.write_text(json.dumps({"algorithm": "CRC-32C (reflected 0x82F63B78), checksum = ~crc(0xFFFFFFFF, data)",
                                "kats": out}, indent=1) + "\n")


if __name__ == "__main__":
    main()
