"""Split-buffer allocator (include/subspace_crc.h "Split-buffer allocator") from Python.

The reference lets a publisher keep each slot's payload in its own buffer and all
prefixes in a separate one ("split buffers", common/split_buffer.h:43-55), allocated by
user callbacks (client/options.h:242-249, :404-411; C client c_client/subspace.h:140-158).
libsubspace_crc.so provides such callbacks: memfd + shared mapping + pinning and device
mapping (subspace_crc_host_register), so the zero-copy slot-list path
(``CrcContext.crc32_host_slot_list``) reads and writes the buffers in place. This module
wraps them with ctypes mirrors of the C structs, for tests and Python tooling.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

REQUIRE_PIN = 0x1  # SUBSPACE_CRC_SPLIT_REQUIRE_PIN


class SplitInfo(ctypes.Structure):
    """subspace_crc_split_info == SubspaceSplitBufferInfo (c_client/subspace.h:109-119)."""
    _fields_ = [("channel_name", ctypes.c_char_p), ("session_id", ctypes.c_uint64),
                ("buffer_index", ctypes.c_uint32), ("slot_id", ctypes.c_uint32), ("is_prefix", ctypes.c_bool),
                ("full_size", ctypes.c_uint64), ("allocation_size", ctypes.c_uint64),
                ("handle", ctypes.c_size_t), ("registration_fd", ctypes.c_int), ("map_offset", ctypes.c_int64)]


class SplitMapping(ctypes.Structure):
    """subspace_crc_split_mapping == SubspaceSplitBufferMapping (c_client/subspace.h:120-127)."""
    _fields_ = [("handle", ctypes.c_size_t), ("address", ctypes.c_void_p), ("size", ctypes.c_size_t),
                ("private_data", ctypes.c_void_p), ("fd", ctypes.c_int), ("map_offset", ctypes.c_int64)]


class SplitAllocator(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32)]


class SplitError(RuntimeError):
    pass


def _fns():
    lib = _lib.load()
    for n in ("subspace_crc_split_allocate", "subspace_crc_split_map"):
        f = getattr(lib, n)
        f.restype = ctypes.c_bool
        f.argtypes = [ctypes.POINTER(SplitInfo), ctypes.POINTER(SplitMapping), ctypes.c_void_p]
    for n in ("subspace_crc_split_unmap", "subspace_crc_split_free"):
        f = getattr(lib, n)
        f.restype = ctypes.c_bool
        f.argtypes = [ctypes.POINTER(SplitInfo), ctypes.POINTER(SplitMapping), ctypes.c_void_p]
    lib.subspace_crc_split_is_pinned.restype = ctypes.c_int
    lib.subspace_crc_split_is_pinned.argtypes = [ctypes.c_void_p]
    return lib


@dataclass
class SplitBuffer:
    info: SplitInfo
    mapping: SplitMapping
    owner: bool  # allocated here (free) or mapped from another allocation (unmap)

    @property
    def address(self) -> int:
        return int(self.mapping.address)

    @property
    def size(self) -> int:
        return int(self.mapping.size)

    def array(self) -> np.ndarray:
        """A uint8 numpy view of the mapping (valid until unmap/free)."""
        buf = (ctypes.c_uint8 * self.size).from_address(self.address)
        return np.ctypeslib.as_array(buf)

    def pinned(self) -> bool:
        return _fns().subspace_crc_split_is_pinned(self.mapping.address) == 1


class SplitBufferCallbacks:
    """The allocate / map / unmap / free callbacks of libsubspace_crc.so."""

    def __init__(self, require_pin: bool = False):
        self._cfg = SplitAllocator(REQUIRE_PIN if require_pin else 0)
        self._lib = _fns()

    def _ud(self):
        return ctypes.cast(ctypes.pointer(self._cfg), ctypes.c_void_p)

    def allocate(self, channel: str, size: int, *, slot_id: int = 0, is_prefix: bool = False,
                 buffer_index: int = 0, session_id: int = 0) -> SplitBuffer:
        info = SplitInfo(channel.encode(), session_id, buffer_index, slot_id, is_prefix, size, size, 0, -1, 0)
        m = SplitMapping()
        if not self._lib.subspace_crc_split_allocate(ctypes.byref(info), ctypes.byref(m), self._ud()):
            raise SplitError(f"allocate: {_lib.last_error()}")
        return SplitBuffer(info, m, True)

    def map(self, other: SplitBuffer) -> SplitBuffer:
        """A second mapping of another allocation's buffer through its descriptor, as a
        subscriber maps a publisher's buffer (registration_fd from the server)."""
        o = other.info
        info = SplitInfo(o.channel_name, o.session_id, o.buffer_index, o.slot_id, o.is_prefix, o.full_size,
                         other.size, other.mapping.handle, other.mapping.fd, 0)
        m = SplitMapping()
        m.handle = other.mapping.handle
        if not self._lib.subspace_crc_split_map(ctypes.byref(info), ctypes.byref(m), self._ud()):
            raise SplitError(f"map: {_lib.last_error()}")
        return SplitBuffer(info, m, False)

    def release(self, b: SplitBuffer) -> None:
        fn = self._lib.subspace_crc_split_free if b.owner else self._lib.subspace_crc_split_unmap
        if not fn(ctypes.byref(b.info), ctypes.byref(b.mapping), self._ud()):
            raise SplitError(f"release: {_lib.last_error()}")
