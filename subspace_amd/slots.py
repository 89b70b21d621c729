"""Message-slot layout of dallison/subspace channels, for slot-checksum batches.

Mirrors the reference's data formats on either side of the checksum path:

* ``PREFIX_DTYPE``        -- ``MessagePrefix`` (common/channel.h:88-112), 64 B.
* ``compute_prefix_size`` -- ``Channel::ComputePrefixSize`` (common/channel.h:914-919).
* ``slot_stride``         -- the contiguous layout's slot pitch
  ``PrefixSize + Aligned<64>(SlotSize)`` (client/client_channel.h:130-132, :168-170).
* ``SLOT_DTYPE``          -- ``subspace_crc_slot`` (include/subspace_crc.h): the device
  records of ``subspace_crc32_slots``.
* ``make_prefixes``       -- a block of prefixes as a publisher would fill them
  (client/publisher.cc:640-660) before the checksum, for tests and bench.py.

Only layout and synthetic-input helpers live here; the checksums are computed by
``gpu.CrcContext.crc32_slots*`` (HIP) and, as the test checker, the oracle.
"""
from __future__ import annotations

import numpy as np

from .checksum import MESSAGE_HAS_CHECKSUM, compute_prefix_size  # noqa: F401  (re-exported)

PREFIX_DTYPE = np.dtype([
    ("padding", "<i4"),        # 0: written by the bridge socket, never checksummed
    ("slot_id", "<i4"),        # 4: span 0 starts here
    ("message_size", "<u8"),   # 8
    ("ordinal", "<u8"),        # 16
    ("timestamp", "<u8"),      # 24
    ("flags", "<i8"),          # 32: kMessageHasChecksum = 4
    ("vchan_id", "<i4"),       # 40
    ("checksum_size", "<u2"),  # 44
    ("metadata_size", "<u2"),  # 46: span 0 ends after this field (44 B)
    ("checksum", "<u4"),       # 48: first 4 B of the checksum area
    ("padding3", "V12"),       # 52..63
])
assert PREFIX_DTYPE.itemsize == 64

SLOT_DTYPE = np.dtype([("prefix", "<u8"), ("payload", "<u8"), ("message_size", "<u8")])
assert SLOT_DTYPE.itemsize == 24


def aligned64(n: int) -> int:
    return (n + 63) & ~63


def slot_stride(slot_size: int, checksum_size: int = 4, metadata_size: int = 0) -> int:
    """Pitch of the contiguous slot layout: PrefixSize + Aligned<64>(SlotSize)."""
    return compute_prefix_size(checksum_size, metadata_size) + aligned64(slot_size)


def make_prefixes(count: int, sizes, *, checksum_size: int = 4, metadata_size: int = 0, seed: int = 0,
                  flags_set: bool = False) -> np.ndarray:
    """(count, PrefixSize) uint8 block: MessagePrefix fields as a publisher sets them, random
    metadata, random bytes in the padding words and in the uncovered tail of the checksum area
    (those must never influence the checksum), checksum word zero."""
    rng = np.random.default_rng(seed)
    psize = compute_prefix_size(checksum_size, metadata_size)
    block = rng.integers(0, 256, (count, psize), dtype=np.uint8)
    head = np.zeros(count, dtype=PREFIX_DTYPE)
    head["padding"] = rng.integers(-2**31, 2**31, count, dtype=np.int64).astype(np.int32)
    head["slot_id"] = np.arange(count, dtype=np.int32)
    head["message_size"] = np.asarray(sizes, dtype=np.uint64)
    head["ordinal"] = np.arange(1, count + 1, dtype=np.uint64)
    head["timestamp"] = rng.integers(0, 2**62, count, dtype=np.int64).astype(np.uint64)
    head["flags"] = rng.integers(0, 4, count) & ~MESSAGE_HAS_CHECKSUM  # activation / bridged bits
    if flags_set:
        head["flags"] |= MESSAGE_HAS_CHECKSUM
    head["vchan_id"] = rng.integers(-1, 8, count).astype(np.int32)
    head["checksum_size"] = checksum_size
    head["metadata_size"] = metadata_size
    head["checksum"] = 0
    raw = head.view(np.uint8).reshape(count, 64)
    block[:, :52] = raw[:, :52]  # fields up to and including the checksum word
    return block


def slot_records(prefix_addrs, payload_addrs, sizes) -> np.ndarray:
    """subspace_crc_slot records as an (n, 3) uint64 array."""
    rec = np.empty((len(sizes), 3), dtype=np.uint64)
    rec[:, 0] = np.asarray(prefix_addrs, dtype=np.uint64)
    rec[:, 1] = np.asarray(payload_addrs, dtype=np.uint64)
    rec[:, 2] = np.asarray(sizes, dtype=np.uint64)
    return rec
