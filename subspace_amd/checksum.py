"""Host-side mirror of dallison/subspace ``client/checksum.h`` (and the span helpers
of ``common/channel.h``), backed by the native ``SubspaceCRC32`` in
``libsubspace_crc.so``.

Same names, argument meanings and semantics as the reference:

* ``subspace_crc32(crc, data)``           -- client/checksum.h:18-20 / checksum.cc:125-130:
  raw state in and out, no init/final XOR inside, chainable, ``len 0`` is a no-op.
* ``calculate_crc32_checksum(spans, out)`` -- client/checksum.h:29-37: start from
  0xFFFFFFFF, chain the spans, store ``~crc`` as a native-endian uint32 in the
  first 4 bytes of ``out``.
* ``verify_crc32_checksum(spans, stored)`` -- client/checksum.h:39-47.
* ``get_message_checksum_data(...)``      -- common/channel.h:527-542: the three spans
  (44 prefix bytes from offset 4, the metadata area after the checksum area, the
  payload).
* ``compute_prefix_size``                 -- common/channel.h:914-919.
"""
from __future__ import annotations

import ctypes
import struct
import sys
from typing import Sequence

from . import _lib

# MessagePrefix layout (common/channel.h:88-112)
PREFIX_SIZE = 64
OFFSET_SLOT_ID = 4
OFFSET_CHECKSUM = 48
PREFIX_SPAN_LEN = OFFSET_CHECKSUM - OFFSET_SLOT_ID  # 44
MESSAGE_HAS_CHECKSUM = 4  # kMessageHasChecksum (common/channel.h:62-70)

_NATIVE = "<" if sys.byteorder == "little" else ">"


def _buffer(data) -> tuple[ctypes.c_void_p, int, object]:
    """(pointer, length, keepalive) for any bytes-like object, zero-copy when possible."""
    mv = memoryview(data).cast("B")
    n = mv.nbytes
    if n == 0:
        return ctypes.c_void_p(0), 0, None
    if mv.readonly:
        buf = ctypes.create_string_buffer(mv.tobytes(), n)
        return ctypes.cast(buf, ctypes.c_void_p), n, buf
    arr = (ctypes.c_ubyte * n).from_buffer(mv)
    return ctypes.cast(arr, ctypes.c_void_p), n, arr


def subspace_crc32(crc: int, data) -> int:
    """``SubspaceCRC32(crc, data, len(data))`` (raw state, reference checksum.cc:125-130)."""
    ptr, n, keep = _buffer(data)
    r = _lib.load().SubspaceCRC32(crc & 0xFFFFFFFF, ptr, n)
    del keep
    return int(r)


def subspace_crc32c(crc: int, data) -> int:
    """``SubspaceCRC32C``: CRC-32C with raw state, the function a -msse4.2 build of the
    reference computes in SubspaceCRC32 (checksum.cc:56-76)."""
    ptr, n, keep = _buffer(data)
    r = _lib.load().SubspaceCRC32C(crc & 0xFFFFFFFF, ptr, n)
    del keep
    return int(r)


def _chain(spans: Sequence) -> int:
    crc = 0xFFFFFFFF
    for s in spans:
        crc = subspace_crc32(crc, s)
    return crc


def calculate_crc32_checksum(spans: Sequence, checksum: bytearray | memoryview | None = None) -> bytes:
    """CalculateCRC32Checksum<N> (checksum.h:29-37). Writes 4 bytes into ``checksum`` if given."""
    value = (~_chain(spans)) & 0xFFFFFFFF
    out = struct.pack(_NATIVE + "I", value)
    if checksum is not None:
        if len(checksum) < 4:
            raise ValueError("checksum region must be at least 4 bytes")
        checksum[:4] = out
    return out


def verify_crc32_checksum(spans: Sequence, checksum) -> bool:
    """VerifyCRC32Checksum<N> (checksum.h:39-47): compare the first 4 stored bytes."""
    stored = struct.unpack_from(_NATIVE + "I", bytes(checksum[:4]))[0]
    return stored == ((~_chain(spans)) & 0xFFFFFFFF)


def get_message_checksum_data(prefix, payload, message_size: int, checksum_size: int,
                              metadata_size: int) -> list[memoryview]:
    """GetMessageChecksumData (channel.h:527-542) over Python buffers."""
    p = memoryview(prefix).cast("B")
    return [
        p[OFFSET_SLOT_ID:OFFSET_CHECKSUM],
        p[OFFSET_CHECKSUM + checksum_size:OFFSET_CHECKSUM + checksum_size + metadata_size],
        memoryview(payload).cast("B")[:message_size],
    ]


def compute_prefix_size(checksum_size: int, metadata_size: int) -> int:
    """Channel::ComputePrefixSize (channel.h:914-919): Aligned<64>(48 + cs + ms)."""
    return (OFFSET_CHECKSUM + checksum_size + metadata_size + 63) & ~63
