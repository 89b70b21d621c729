"""Deterministic synthetic batch layouts, host side (numpy).

Payload bytes are generated on device (gpu.fill_uniform / gpu.fill_ragged); this
module provides the shapes: BASELINE configs, ragged lengths and offsets.

  byte j of message i = byte (j mod 8), little-endian, of splitmix64(seed ^ (i << 32) ^ (j >> 3))
  ragged length i     : t = splitmix64(seed ^ 0x4C454E0000000000 ^ i); o = t % 14;
                        L = (64 << o) + (((64 << o) * ((t >> 16) & 0xFFFF)) >> 16)   (64 <= L < 1 MiB)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEED_A = 0x5EED000A
SEED_B = 0x5EED000B
SEED_C = 0x5EED000C
SEED_D = 0x5EED000D
SEED_E = 0x5EED000E

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_bytes(seed: int, msg: int, length: int, start: int = 0) -> bytes:
    """Host twin of the device generator (small sizes: tests and examples)."""
    if length <= 0:
        return b""
    u0, u1 = start >> 3, (start + length + 7) >> 3
    units = np.arange(u0, u1, dtype=np.uint64)
    key = np.uint64((seed ^ (msg << 32)) & 0xFFFFFFFFFFFFFFFF)
    words = splitmix64(key ^ units).astype("<u8").tobytes()
    off = start - (u0 << 3)
    return words[off:off + length]


def host_uniform(seed: int, ids, length: int, chunk: int = 4096) -> np.ndarray:
    """Host twin of gpu.fill_uniform for the messages `ids`: an (n, length) uint8 array
    (bench.py --dry-run-cpu; vectorised, a few hundred MB/s)."""
    ids = np.asarray(ids, dtype=np.uint64)
    out = np.empty((len(ids), length), dtype=np.uint8)
    units = np.arange((length + 7) >> 3, dtype=np.uint64)
    for a in range(0, len(ids), chunk):
        keys = np.uint64(seed) ^ (ids[a:a + chunk] << np.uint64(32))
        words = splitmix64(keys[:, None] ^ units[None, :]).astype("<u8")
        out[a:a + chunk] = words.view(np.uint8)[:, :length]
    return out


def host_ragged(seed: int, ids, lengths, offsets, arena_bytes: int) -> np.ndarray:
    """Host twin of gpu.fill_ragged: message ids[i] (lengths[i] bytes) at offsets[i] of a
    zeroed arena of `arena_bytes` bytes."""
    arena = np.zeros(arena_bytes, dtype=np.uint8)
    for i, o, n in zip(np.asarray(ids, dtype=np.uint64), np.asarray(offsets, dtype=np.uint64),
                       np.asarray(lengths, dtype=np.uint64)):
        n = int(n)
        if n:
            key = np.uint64(seed) ^ (np.uint64(i) << np.uint64(32))
            words = splitmix64(key ^ np.arange((n + 7) >> 3, dtype=np.uint64)).astype("<u8")
            arena[int(o):int(o) + n] = words.view(np.uint8)[:n]
    return arena


def ragged_lengths(seed: int, count: int, first: int = 0) -> np.ndarray:
    i = np.arange(first, first + count, dtype=np.uint64)
    t = splitmix64(np.uint64(seed ^ 0x4C454E0000000000) ^ i)
    octave = t % np.uint64(14)
    base = np.uint64(64) << octave
    frac = (t >> np.uint64(16)) & np.uint64(0xFFFF)
    return (base + ((base * frac) >> np.uint64(16))).astype(np.uint64)


def packed_offsets(lengths: np.ndarray, align: int = 64) -> tuple[np.ndarray, int]:
    """Offsets of messages packed back to back, each start rounded up to `align` (1 = unaligned)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    if align <= 1:
        padded = lengths
    else:
        padded = (lengths + np.uint64(align - 1)) & ~np.uint64(align - 1)
    ends = np.cumsum(padded, dtype=np.uint64)
    offsets = np.concatenate([np.zeros(1, dtype=np.uint64), ends[:-1]])
    total = int(ends[-1]) if len(ends) else 0
    return offsets, total


@dataclass(frozen=True)
class Config:
    name: str
    description: str
    seed: int


CONFIGS = {
    "B": Config("B", "65,536 x 4 KiB independent payloads, one CRC32 each", SEED_B),
    "C": Config("C", "1 M messages, log-uniform 64 B - 1 MiB, 64-B aligned offsets", SEED_C),
    "D": Config("D", "256 x 64 MiB payloads", SEED_D),
    "E": Config("E", "8 M x 4 KiB payloads sharded round-robin over GPUs", SEED_E),
}
