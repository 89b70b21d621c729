"""Batched device CRC32 through the C ABI (include/subspace_crc.h).

``CrcContext`` owns one ``subspace_crc_ctx`` (tables uploaded once per device).
Batches are torch tensors on that device -- torch is only the device-memory and
stream plumbing here; every CRC is computed by the HIP kernels in
``libsubspace_crc.so``. There is no CPU fallback: without the library or a gfx950
device the calls raise.
"""
from __future__ import annotations

import ctypes

from . import _lib

FINALIZE = 0x1  # SUBSPACE_CRC_FINALIZE: store ~crc (the checksum CalculateCRC32Checksum writes)
POLY_IEEE = 0xEDB88320        # the reference's default builds (SubspaceCRC32)
POLY_CASTAGNOLI = 0x82F63B78  # CRC-32C: -msse4.2 reference builds (SubspaceCRC32C)

# message-slot checksums (include/subspace_crc.h)
SLOT_CALCULATE = 0  # publisher: set kMessageHasChecksum, store the 3-span checksum in the prefix
SLOT_VERIFY = 1     # subscriber: check the stored checksum of slots that carry the flag
SLOT_OK, SLOT_MISMATCH, SLOT_UNCHECKED, SLOT_OVERSIZE = 0, 1, 2, 4  # 3: the C++ helper's kSkipped
EFAULT = -5  # SUBSPACE_CRC_EFAULT: a kernel of an earlier call gave up a bounded wait


class CrcError(RuntimeError):
    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise CrcError(f"{what} failed ({rc}): {_lib.last_error()}", rc)


def _ptr(t) -> int:
    return int(t.data_ptr())


def _stream_ptr(stream) -> int | None:
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if stream.cuda_stream else None


class CrcContext:
    """Per-device context (reference analogue: the client library's per-process state)."""

    def __init__(self, device: int = 0, poly: int = POLY_IEEE):
        self._lib = _lib.load()
        self.device = device
        self.poly = poly
        h = ctypes.c_void_p()
        _check(self._lib.subspace_crc_ctx_create_poly(device, poly, ctypes.byref(h)), "subspace_crc_ctx_create_poly")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.subspace_crc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def check(self, stream=None) -> None:
        """Synchronise ``stream`` and raise CrcError (code EFAULT) if a kernel of an earlier
        call on this context gave up a bounded wait (subspace_crc_ctx_check)."""
        _check(self._lib.subspace_crc_ctx_check(self._h, _stream_ptr(stream)), "subspace_crc_ctx_check")

    def reserve(self, max_messages: int, max_tiles: int) -> None:
        _check(self._lib.subspace_crc_ctx_reserve(self._h, max_messages, max_tiles), "subspace_crc_ctx_reserve")

    def crc32_uniform(self, buf, stride: int, length: int, count: int, out, *, init: int = 0xFFFFFFFF,
                      finalize: bool = False, stream=None, base_offset: int = 0) -> None:
        """out[i] = SubspaceCRC32(init, buf[base_offset + i*stride :][:length]) for i < count."""
        _check(self._lib.subspace_crc32_batch_uniform(
            self._h, _ptr(buf) + base_offset, stride, length, count, init & 0xFFFFFFFF,
            FINALIZE if finalize else 0, _ptr(out), _stream_ptr(stream)), "subspace_crc32_batch_uniform")

    def crc32_ragged(self, buf, offsets, lengths, out, *, init: int = 0xFFFFFFFF, finalize: bool = False,
                     arena_bytes: int | None = None, stream=None) -> None:
        """out[i] = SubspaceCRC32(init, buf[offsets[i]:][:lengths[i]]) (int64 device tensors)."""
        n = int(offsets.numel())
        if int(lengths.numel()) != n or int(out.numel()) < n:
            raise ValueError("offsets, lengths and out must describe the same number of messages")
        arena = int(buf.numel() * buf.element_size()) if arena_bytes is None else arena_bytes
        _check(self._lib.subspace_crc32_batch(
            self._h, _ptr(buf), arena, _ptr(offsets), _ptr(lengths), n, init & 0xFFFFFFFF,
            FINALIZE if finalize else 0, _ptr(out), _stream_ptr(stream)), "subspace_crc32_batch")


    def crc32_slots(self, slots, *, max_message_size: int, checksum_size: int = 4, metadata_size: int = 0,
                    mode: int = SLOT_CALCULATE, status=None, error_count=None, stream=None) -> None:
        """3-span checksums of a slot list. ``slots`` is an int64 device tensor of shape (n, 3):
        (prefix address, payload address, message_size) per slot -- subspace_crc_slot records."""
        if slots.dim() != 2 or slots.shape[1] != 3 or not slots.is_contiguous():
            raise ValueError("slots must be a contiguous (n, 3) int64 tensor")
        n = int(slots.shape[0])
        if status is not None and int(status.numel()) < n:
            raise ValueError("status is shorter than the slot list")
        _check(self._lib.subspace_crc32_slots(
            self._h, _ptr(slots), n, max_message_size, checksum_size, metadata_size, mode,
            _ptr(status) if status is not None else None, _ptr(error_count) if error_count is not None else None,
            _stream_ptr(stream)), "subspace_crc32_slots")

    def crc32_slots_strided(self, buf, slot_stride: int, count: int, *, message_size: int = 0, sizes=None,
                            checksum_size: int = 4, metadata_size: int = 0, mode: int = SLOT_CALCULATE,
                            status=None, error_count=None, base_offset: int = 0, stream=None) -> None:
        """3-span checksums of ``count`` slots laid out contiguously from buf[base_offset:]
        (prefix at i*slot_stride, payload after ComputePrefixSize bytes)."""
        if status is not None and int(status.numel()) < count:
            raise ValueError("status is shorter than the slot count")
        if sizes is not None and int(sizes.numel()) < count:
            raise ValueError("sizes is shorter than the slot count")
        _check(self._lib.subspace_crc32_slots_strided(
            self._h, _ptr(buf) + base_offset, slot_stride, count, message_size,
            _ptr(sizes) if sizes is not None else None, checksum_size, metadata_size, mode,
            _ptr(status) if status is not None else None, _ptr(error_count) if error_count is not None else None,
            _stream_ptr(stream)), "subspace_crc32_slots_strided")

    def crc32_host_slots(self, host, slot_stride: int, count: int, *, message_size: int = 0, sizes=None,
                         checksum_size: int = 4, metadata_size: int = 0, mode: int = SLOT_CALCULATE,
                         status=None) -> int:
        """End-to-end slot checksums over a HOST buffer (numpy uint8 array, or a CPU torch
        tensor, ideally pinned: see host_register) holding ``count`` contiguous slots.
        CALCULATE writes the flag and checksum into the host prefixes; VERIFY fills
        ``status`` (numpy uint32, optional). Returns the mismatch count (VERIFY)."""
        import numpy as np
        ptr, nbytes = _host_ptr(host)
        if nbytes < count * slot_stride:
            raise ValueError("host buffer is shorter than count * slot_stride")
        if sizes is not None:
            sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
            if sizes.size < count:
                raise ValueError("sizes is shorter than the slot count")
        if status is not None and (status.dtype != np.uint32 or status.size < count or not status.flags.c_contiguous):
            raise ValueError("status must be a contiguous uint32 array of at least count entries")
        err = ctypes.c_uint32(0)
        _check(self._lib.subspace_crc32_host_slots(
            self._h, ptr, slot_stride, count, message_size,
            sizes.ctypes.data if sizes is not None else None, checksum_size, metadata_size, mode,
            status.ctypes.data if status is not None else None, ctypes.byref(err)), "subspace_crc32_host_slots")
        return int(err.value)


    def crc32_host_slot_list(self, records, *, max_message_size: int, checksum_size: int = 4,
                             metadata_size: int = 0, mode: int = SLOT_CALCULATE, status=None) -> int:
        """Zero-copy slot list in registered host memory (the subscriber drain hook):
        ``records`` is an (n, 3) uint64 array (slots.slot_records) of HOST addresses
        (prefix, payload, message_size). Returns the mismatch count (VERIFY); fills
        ``status`` if given."""
        import numpy as np
        records = np.ascontiguousarray(records, dtype=np.uint64)
        if records.ndim != 2 or records.shape[1] != 3:
            raise ValueError("records must be an (n, 3) array of subspace_crc_slot fields")
        n = len(records)
        if status is not None and (status.dtype != np.uint32 or status.size < n or not status.flags.c_contiguous):
            raise ValueError("status must be a contiguous uint32 array of at least len(records) entries")
        err = ctypes.c_uint32(0)
        _check(self._lib.subspace_crc32_host_slot_list(
            self._h, records.ctypes.data, n, max_message_size, checksum_size, metadata_size, mode,
            status.ctypes.data if status is not None else None, ctypes.byref(err)), "subspace_crc32_host_slot_list")
        return int(err.value)


def _host_ptr(host) -> tuple[int, int]:
    if hasattr(host, "data_ptr"):  # torch CPU tensor
        if host.is_cuda:
            raise ValueError("expected a host (CPU) buffer")
        return int(host.data_ptr()), int(host.numel() * host.element_size())
    if not host.flags.c_contiguous:
        raise ValueError("host buffer must be contiguous")
    return int(host.ctypes.data), int(host.nbytes)


def host_register(host) -> None:
    """Pin a host buffer for DMA (hipHostRegister); release with host_unregister."""
    ptr, n = _host_ptr(host)
    _check(_lib.load().subspace_crc_host_register(ptr, n), "subspace_crc_host_register")


def host_unregister(host) -> None:
    ptr, _ = _host_ptr(host)
    _check(_lib.load().subspace_crc_host_unregister(ptr), "subspace_crc_host_unregister")


# ---------------------------------------------------------------- synthetic inputs (device)
def fill_uniform(buf, stride: int, length: int, count: int, *, seed: int, first_id: int = 0, id_stride: int = 1,
                 stream=None) -> None:
    """Deterministic payloads (SURVEY.md 8d generator) for a fixed-size batch, on device."""
    _check(_lib.load_dev().subspace_crc_testutil_fill_uniform(
        _ptr(buf), stride, length, count, first_id, id_stride, seed, _stream_ptr(stream)), "fill_uniform")


def fill_ragged(buf, offsets, lengths, *, seed: int, first_id: int = 0, id_stride: int = 1, stream=None) -> None:
    _check(_lib.load_dev().subspace_crc_testutil_fill_ragged(
        _ptr(buf), _ptr(offsets), _ptr(lengths), int(offsets.numel()), first_id, id_stride, seed,
        _stream_ptr(stream)), "fill_ragged")


def slot_list_read(records, count: int, out, mode: int = 4, stride: int = 0, lds: bool = True, stream=None) -> None:
    """Slot-list read ceiling probe (testutil.hip slot_list_read_kernel): the small-message
    kernel's loads over `count` device subspace_crc_slot records -- mode 4 = its FAST loop's (the
    window's records in registers, one address and 8 immediate offsets per tile, the first
    window's prefix words) -- with an XOR fold instead of the CRC; out: int32 device tensor of at
    least the kernel's grid x 512 words (256 * 512 covers every count up to 2^22 slots)."""
    _check(_lib.load_dev().subspace_crc_testutil_slot_list_read(
        _ptr(records), int(count), int(mode), int(stride), 1 if lds else 0, _ptr(out), int(out.numel()),
        _stream_ptr(stream)), "slot_list_read")


def tile_list_read(tiles, out, stream=None) -> None:
    """Tile-list read ceiling probe (testutil.hip tile_list_read_kernel): the ragged kernel's
    loads over device records {u64 16-B-aligned start, u64 bytes <= 8192} (int64 tensor of
    shape (ntiles, 2)), an XOR fold instead of the CRC; out: int32 device tensor of 256 * 512
    words."""
    _check(_lib.load_dev().subspace_crc_testutil_tile_list_read(
        _ptr(tiles), int(tiles.shape[0]), _ptr(out), int(out.numel()), _stream_ptr(stream)), "tile_list_read")


def stream_read(buf, out, stream=None) -> None:
    """Streaming-read ceiling probe over buf (the CRC kernels' load shape, no CRC);
    out: int32 device tensor of 256 * 512 words."""
    if int(out.numel()) < 256 * 512:
        raise ValueError("out needs 131072 words")
    _check(_lib.load_dev().subspace_crc_testutil_stream_read(
        _ptr(buf), int(buf.numel() * buf.element_size()), _ptr(out), _stream_ptr(stream)), "stream_read")
