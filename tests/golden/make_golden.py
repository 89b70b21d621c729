#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/.

  python tests/golden/make_golden.py            # small vectors  -> golden.json
  python tests/golden/make_golden.py --configs  # + full-size synthetic config hashes -> configs.json
  python tests/golden/make_golden.py --small    # only the small config prefixes (B_small, C_small,
                                                # C_2k), merged into the existing configs.json

Expected values come from Python's zlib.crc32 (zlib 1.2.11), an implementation of
the same published IEEE CRC-32 algorithm that is independent of this repository.
The relation to the reference's raw-state function (client/checksum.cc:125-130) is
  SubspaceCRC32(s, d) == ~zlib.crc32(d, ~s) & 0xFFFFFFFF,
verified in the survey container against the compiled reference on 2,000 random
vectors. Every value is also checked against the oracle
(oracle/crc32_oracle.c) while generating; a disagreement aborts.

The full-size config hashes (configs.json) are computed with the multi-threaded
oracle, and a random sample of each config is re-checked with zlib here.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import random
import struct
import sys
import time
import zlib
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import _oracle  # noqa: E402
from subspace_amd import synth  # noqa: E402

M32 = 0xFFFFFFFF


def ref_raw(state: int, data: bytes) -> int:
    """SubspaceCRC32(state, data) via zlib."""
    return (~zlib.crc32(data, (~state) & M32)) & M32


def make_prefix(slot_id, message_size, ordinal, timestamp, flags, vchan_id, checksum_size, metadata_size) -> bytes:
    """MessagePrefix (common/channel.h:88-112), little-endian x86-64 layout, checksum area zero."""
    p = struct.pack("<iiQQQqiHHI", 0, slot_id, message_size, ordinal, timestamp, flags, vchan_id,
                    checksum_size, metadata_size, 0)
    return p + b"\0" * (64 - len(p))


def small_vectors(oracle) -> dict:
    out: dict = {"generator": "tests/golden/make_golden.py", "zlib_version": zlib.ZLIB_VERSION}

    def check(state, data, expected):
        got = oracle.crc32(state, data)
        assert got == expected, (state, data[:16], hex(got), hex(expected))

    # 1. known answers (init 0xFFFFFFFF, raw and final)
    kats = []
    for s in [b"", b"a", b"abc", b"hello", b"123456789", b"foobar", b"hello world",
              b"The quick brown fox jumps over the lazy dog", bytes(range(256))]:
        raw = ref_raw(M32, s)
        check(M32, s, raw)
        kats.append({"data_hex": s.hex(), "raw": raw, "final": (~raw) & M32})
    out["kat"] = kats

    # 2. the reference's own literal tests (rust_client/tests/client_test.rs; C++ pins to it)
    out["reference_tests"] = {
        "crc32_empty_data (client_test.rs:169-173)": {"state": M32, "data_hex": "", "raw": M32},
        "crc32_known_value (client_test.rs:175-180)": {"state": M32, "data_hex": b"hello".hex(), "final": 0x3610A686},
        "incremental (client_test.rs:183-191)": {"whole": b"hello world".hex(), "parts": [b"hello ".hex(), b"world".hex()]},
        "single_vs_multi_span (client_test.rs:213-218)": {"whole": [b"foobar".hex()], "split": [b"foo".hex(), b"bar".hex()]},
        "calculate_and_verify (client_test.rs:194-203)": {"spans": [b"subspace".hex(), b"ipc".hex()]},
    }
    assert ((~ref_raw(M32, b"hello")) & M32) == 0x3610A686

    # 3. every prefix length 0..520 of a fixed synthetic buffer
    seed, msg = 0x601DE, 0
    buf = synth.synth_bytes(seed, msg, 520)
    assert buf == oracle.synth_bytes(seed, msg, 520)
    lens = []
    for n in range(521):
        raw = ref_raw(M32, buf[:n])
        check(M32, buf[:n], raw)
        lens.append(raw)
    out["prefix_lengths"] = {"seed": seed, "msg": msg, "buffer_hex": buf.hex(), "raw": lens}

    # 4. longer lengths (generator-defined data, see subspace_amd/synth.py)
    big = []
    for n in [1023, 1024, 1025, 4095, 4096, 4097, 8191, 8192, 8193, 65537, (1 << 20) + 3]:
        d = synth.synth_bytes(seed, 1, n)
        raw = ref_raw(M32, d)
        check(M32, d, raw)
        big.append({"seed": seed, "msg": 1, "length": n, "raw": raw})
    out["long_lengths"] = big

    # 5. arbitrary raw input states (the raw-state contract, client_test.cc:5234 uses such seeds)
    rng = random.Random(0xC0FFEE)
    raws = []
    for i in range(64):
        state = rng.getrandbits(32)
        n = rng.randrange(0, 301)
        d = synth.synth_bytes(seed, 2, n, start=rng.randrange(0, 64))
        raw = ref_raw(state, d)
        check(state, d, raw)
        raws.append({"state": state, "data_hex": d.hex(), "raw": raw})
    out["raw_states"] = raws

    # 6. three-span message checksums (common/channel.h:527-542, client/publisher.cc:664-675)
    spans_cases = []
    for (cs, ms, payload_len) in [(4, 0, 0), (4, 0, 100), (20, 0, 7), (4, 13, 4096), (32, 64, 1000)]:
        prefix_size = (48 + cs + ms + 63) & ~63
        prefix = bytearray(make_prefix(3, payload_len, 17, 1234567890123, 4, -1, cs, ms))
        prefix += b"\0" * (prefix_size - 64)
        meta = synth.synth_bytes(seed, 3, ms)
        prefix[48 + cs:48 + cs + ms] = meta
        payload = synth.synth_bytes(seed, 4, payload_len)
        spans = [bytes(prefix[4:48]), bytes(prefix[48 + cs:48 + cs + ms]), payload]
        crc = M32
        for s in spans:
            crc = ref_raw(crc, s)
        final = (~crc) & M32
        assert oracle.checksum(spans) == final.to_bytes(4, "little")
        spans_cases.append({"checksum_size": cs, "metadata_size": ms, "prefix_hex": bytes(prefix).hex(),
                            "payload_hex": payload.hex(), "checksum_le_hex": final.to_bytes(4, "little").hex()})
    out["three_span"] = spans_cases

    # 7. Checksum20Byte (client/client_test.cc:5226-5238): 5 CRCs with seeds 0xFFFFFFFF ^ k*0x11111111
    prefix = make_prefix(0, 7, 1, 42, 4, -1, 20, 0) + b"\0" * 64
    spans = [prefix[4:48], b"", b"hello20"]
    outs = []
    for k in range(5):
        crc = M32 ^ ((k * 0x11111111) & M32)
        for s in spans:
            crc = ref_raw(crc, s)
        outs.append((~crc) & M32)
    out["checksum20"] = {"prefix_hex": prefix.hex(), "payload_hex": b"hello20".hex(), "values": outs}
    return out


def list_hash(crcs: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(crcs, dtype="<u4").tobytes()).hexdigest()


def config_hashes(oracle, threads: int, small_only: bool = False) -> dict:
    res = {"generator": "tests/golden/make_golden.py --configs", "init": M32, "crc": "raw"}
    t0 = time.time()

    def add(name, seed, lengths, note):
        t = time.time()
        crcs = oracle.synth_crc_batch(seed, lengths, threads=threads)
        rng = random.Random(seed)
        for i in rng.sample(range(len(lengths)), min(24, len(lengths))):
            d = synth.synth_bytes(seed, i, int(lengths[i]))
            assert ref_raw(M32, d) == int(crcs[i]), (name, i)
        res[name] = {"seed": seed, "count": int(len(lengths)), "total_bytes": int(np.sum(lengths, dtype=np.uint64)),
                     "sha256_le_u32": list_hash(crcs), "first": [int(x) for x in crcs[:16]], "note": note}
        print(f"{name}: {len(lengths)} msgs, {res[name]['total_bytes'] / 2**30:.2f} GiB in {time.time() - t:.1f}s",
              flush=True)

    if not small_only:
        add("B", synth.SEED_B, np.full(65536, 4096, dtype=np.uint64), "65,536 x 4 KiB")
    add("B_small", synth.SEED_B, np.full(4096, 4096, dtype=np.uint64), "first 4,096 messages of B")
    if not small_only:
        add("C", synth.SEED_C, synth.ragged_lengths(synth.SEED_C, 1 << 20), "1 Mi ragged 64 B - 1 MiB")
    add("C_small", synth.SEED_C, synth.ragged_lengths(synth.SEED_C, 20000), "first 20,000 messages of C")
    add("C_2k", synth.SEED_C, synth.ragged_lengths(synth.SEED_C, 2048),
        "first 2,048 messages of C (bench.py --dry-run-cpu, contiguous shards)")
    if not small_only:
        add("D", synth.SEED_D, np.full(256, 64 << 20, dtype=np.uint64), "256 x 64 MiB")
        add("E", synth.SEED_E, np.full(8 << 20, 4096, dtype=np.uint64), "8 Mi x 4 KiB (global message ids)")
    res["seconds"] = round(time.time() - t0, 1)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", action="store_true")
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    oracle = _oracle.load()
    vec = small_vectors(oracle)
    (HERE / "golden.json").write_text(json.dumps(vec, indent=1) + "\n")
    print("wrote golden.json")
    if args.configs:
        cfg = config_hashes(oracle, args.threads)
        (HERE / "configs.json").write_text(json.dumps(cfg, indent=1) + "\n")
        print("wrote configs.json")
    elif args.small:
        cfg = json.loads((HERE / "configs.json").read_text())
        small = config_hashes(oracle, args.threads, small_only=True)
        for k in ("B_small", "C_small", "C_2k"):
            cfg[k] = small[k]
        (HERE / "configs.json").write_text(json.dumps(cfg, indent=1) + "\n")
        print("updated configs.json (small prefixes)")


if __name__ == "__main__":
    main()
