"""ctypes wrapper of oracle/liboracle_crc.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this, and
only as the checker / the timed CPU baseline, never as the computation under test.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent.parent / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle_crc.so"

_lib = None


class Oracle:
    def __init__(self, lib: ctypes.CDLL):
        self.lib = lib
        u32, u64, vp, sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t
        lib.oracle_table.restype = ctypes.POINTER(u32)
        lib.oracle_crc32.restype = u32
        lib.oracle_crc32.argtypes = [u32, vp, sz]
        lib.oracle_calculate_checksum.argtypes = [vp, vp, sz, vp]
        lib.oracle_verify_checksum.restype = ctypes.c_int
        lib.oracle_verify_checksum.argtypes = [vp, vp, sz, vp]
        lib.oracle_crc32_batch.argtypes = [vp, vp, vp, sz, u32, vp, ctypes.c_int]
        lib.oracle_crc32_batch_pinned.restype = ctypes.c_int
        lib.oracle_crc32_batch_pinned.argtypes = [vp, vp, vp, sz, u32, vp, ctypes.c_int]
        lib.oracle_first_touch_copy.restype = ctypes.c_int
        lib.oracle_first_touch_copy.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int]
        lib.oracle_splitmix64.restype = u64
        lib.oracle_splitmix64.argtypes = [u64]
        lib.oracle_synth_fill.argtypes = [u64, u64, u64, vp, sz]
        lib.oracle_synth_crc.restype = u32
        lib.oracle_synth_crc.argtypes = [u64, u64, u64, u32]
        lib.oracle_synth_crc_batch.argtypes = [u64, vp, vp, sz, u32, vp, ctypes.c_int]
        lib.oracle_ragged_length.restype = u64
        lib.oracle_ragged_length.argtypes = [u64, u64]
        lib.oracle_publish_slots.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int32, ctypes.c_int32]
        lib.oracle_verify_slots.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int32, ctypes.c_int32, vp]
        lib.oracle_has_sse42.restype = ctypes.c_int
        lib.oracle_crc32c_sse42.restype = u32
        lib.oracle_crc32c_sse42.argtypes = [u32, vp, sz]
        lib.oracle_crc32c_sse42_batch.argtypes = [vp, vp, vp, sz, u32, vp, ctypes.c_int]
        lib.oracle_crc32c.restype = u32
        lib.oracle_crc32c.argtypes = [u32, vp, sz]
        lib.oracle_synth_crc_batch_poly.argtypes = [u64, vp, vp, sz, u32, vp, ctypes.c_int, ctypes.c_int]
        lib.oracle_publish_slots_poly.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int32, ctypes.c_int32, ctypes.c_int]
        lib.oracle_verify_slots_poly.argtypes = [vp, vp, vp, vp, sz, ctypes.c_int32, ctypes.c_int32, vp,
                                                 ctypes.c_int]

    def publish_slots(self, host: np.ndarray, prefix_off, payload_off, sizes, checksum_size: int,
                      metadata_size: int, castagnoli: bool = False) -> None:
        """Publisher checksum (flag + 3-span CRC into the prefix) for every slot, in place."""
        assert host.dtype == np.uint8 and host.flags.c_contiguous
        po, yo, sz = (np.ascontiguousarray(a, dtype=np.uint64) for a in (prefix_off, payload_off, sizes))
        self.lib.oracle_publish_slots_poly(host.ctypes.data, po.ctypes.data, yo.ctypes.data, sz.ctypes.data,
                                           len(po), checksum_size, metadata_size, int(castagnoli))

    def verify_slots(self, host: np.ndarray, prefix_off, payload_off, sizes, checksum_size: int,
                     metadata_size: int, castagnoli: bool = False) -> np.ndarray:
        po, yo, sz = (np.ascontiguousarray(a, dtype=np.uint64) for a in (prefix_off, payload_off, sizes))
        st = np.zeros(len(po), dtype=np.uint32)
        self.lib.oracle_verify_slots_poly(host.ctypes.data, po.ctypes.data, yo.ctypes.data, sz.ctypes.data,
                                          len(po), checksum_size, metadata_size, st.ctypes.data, int(castagnoli))
        return st

    def table(self) -> list[int]:
        t = self.lib.oracle_table()
        return [t[i] for i in range(256)]

    def crc32(self, crc: int, data: bytes) -> int:
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        return int(self.lib.oracle_crc32(crc & 0xFFFFFFFF, buf, len(data)))

    def crc32c(self, crc: int, data: bytes) -> int:
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        return int(self.lib.oracle_crc32c(crc & 0xFFFFFFFF, buf, len(data)))

    def has_sse42(self) -> bool:
        return bool(self.lib.oracle_has_sse42())

    def crc32c_sse42(self, crc: int, data: bytes) -> int:
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        return int(self.lib.oracle_crc32c_sse42(crc & 0xFFFFFFFF, buf, len(data)))

    def crc32c_sse42_batch(self, base: np.ndarray, offsets, lengths, init: int = 0xFFFFFFFF,
                           threads: int = 1) -> np.ndarray:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        out = np.zeros(len(offsets), dtype=np.uint32)
        self.lib.oracle_crc32c_sse42_batch(base.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, len(offsets),
                                           init & 0xFFFFFFFF, out.ctypes.data, threads)
        return out

    def checksum(self, spans) -> bytes:
        crc = 0xFFFFFFFF
        for s in spans:
            crc = self.crc32(crc, bytes(s))
        return ((~crc) & 0xFFFFFFFF).to_bytes(4, "little")

    def synth_bytes(self, seed: int, msg: int, length: int, start: int = 0) -> bytes:
        buf = ctypes.create_string_buffer(max(length, 1))
        self.lib.oracle_synth_fill(seed, msg, start, buf, length)
        return buf.raw[:length]

    def synth_crc(self, seed: int, msg: int, length: int, init: int = 0xFFFFFFFF) -> int:
        return int(self.lib.oracle_synth_crc(seed, msg, length, init & 0xFFFFFFFF))

    def synth_crc_batch(self, seed: int, lengths, msg_ids=None, init: int = 0xFFFFFFFF, threads: int = 8,
                        castagnoli: bool = False) -> np.ndarray:
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        n = len(lengths)
        out = np.zeros(n, dtype=np.uint32)
        ids_p = None
        if msg_ids is not None:
            msg_ids = np.ascontiguousarray(msg_ids, dtype=np.uint64)
            ids_p = msg_ids.ctypes.data
        self.lib.oracle_synth_crc_batch_poly(seed, ids_p, lengths.ctypes.data, n, init & 0xFFFFFFFF,
                                             out.ctypes.data, threads, int(castagnoli))
        return out

    def crc32_batch(self, base: np.ndarray, offsets, lengths, init: int = 0xFFFFFFFF, threads: int = 1) -> np.ndarray:
        base = np.ascontiguousarray(base, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        out = np.zeros(len(offsets), dtype=np.uint32)
        self.lib.oracle_crc32_batch(base.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, len(offsets),
                                    init & 0xFFFFFFFF, out.ctypes.data, threads)
        return out

    def crc32_batch_pinned(self, base: np.ndarray, offsets, lengths, init: int = 0xFFFFFFFF,
                           threads: int = 1) -> tuple[np.ndarray, int]:
        """crc32_batch with one worker per core, pinned (BASELINE.md CPU-baseline plan).
        Returns (crcs, number of workers that were pinned)."""
        assert base.dtype == np.uint8 and base.flags.c_contiguous
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        out = np.zeros(len(offsets), dtype=np.uint32)
        pinned = self.lib.oracle_crc32_batch_pinned(base.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                                                    len(offsets), init & 0xFFFFFFFF, out.ctypes.data, threads)
        return out, int(pinned)

    def first_touch_copy(self, src: np.ndarray, offsets, lengths, threads: int) -> np.ndarray:
        """A copy of `src` whose message bytes are first touched by the pinned worker that
        owns them under crc32_batch_pinned's round-robin partition."""
        assert src.dtype == np.uint8 and src.flags.c_contiguous
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        dst = np.empty_like(src)  # untouched pages
        self.lib.oracle_first_touch_copy(dst.ctypes.data, src.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                                         len(offsets), threads)
        return dst

    def ragged_lengths(self, seed: int, count: int) -> np.ndarray:
        return np.array([self.lib.oracle_ragged_length(seed, i) for i in range(count)], dtype=np.uint64)


def load() -> Oracle:
    global _lib
    if _lib is None:
        if not ORACLE_LIB.exists():
            subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True)
        _lib = Oracle(ctypes.CDLL(str(ORACLE_LIB)))
    return _lib
