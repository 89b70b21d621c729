"""Loader for the in-tree C-ABI library ``subspace_amd/libsubspace_crc.so``.

The library is built by ``make`` (or ``__graft_entry__.build()``) with hipcc for
gfx950. There is deliberately no fallback: if the library is missing or does not
load, every entry point raises, so a GPU run can never silently compute on a CPU
path.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "libsubspace_crc.so"
if os.environ.get("SUBSPACE_CRC_PROBE_LIB"):  # investigation builds (tools/ab_lib.sh)
    LIB_PATH = Path(os.environ["SUBSPACE_CRC_PROBE_LIB"])
# Development library (tests, bench.py, tools only; devtools.hip + testutil.hip): path knobs,
# fault injection, PROBE hooks, synthetic-payload generators, read-ceiling probes. It works on
# contexts the product library creates (ctx.h); the product library never loads it.
DEV_LIB_PATH = _HERE / "libsubspace_crc_dev.so"
if os.environ.get("SUBSPACE_CRC_PROBE_DEV_LIB"):  # an A/B build's matching dev library
    DEV_LIB_PATH = Path(os.environ["SUBSPACE_CRC_PROBE_DEV_LIB"])

# Every symbol include/subspace_crc.h declares (tests check they are all exported).
EXPORTED_SYMBOLS = (
    "SubspaceCRC32",
    "SubspaceCRC32C",
    "subspace_crc_version",
    "subspace_crc_last_error",
    "subspace_crc_ctx_create",
    "subspace_crc_ctx_create_poly",
    "subspace_crc_ctx_destroy",
    "subspace_crc_ctx_check",
    "subspace_crc_ctx_reserve",
    "subspace_crc32_batch_uniform",
    "subspace_crc32_batch",
    "subspace_crc32_slots",
    "subspace_crc32_slots_strided",
    "subspace_crc32_host_slots",
    "subspace_crc32_host_slot_list",
    "subspace_crc_host_register",
    "subspace_crc_host_unregister",
    "subspace_crc_split_allocate",
    "subspace_crc_split_map",
    "subspace_crc_split_unmap",
    "subspace_crc_split_free",
    "subspace_crc_split_is_pinned",
)

_lib = None
_dev = None


class LibraryNotBuilt(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and return the library with argtypes configured."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise LibraryNotBuilt(f"{LIB_PATH} not found: run `make` (or __graft_entry__.build()) first")
    lib = ctypes.CDLL(os.fspath(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    u32, u64, vp, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int

    lib.SubspaceCRC32.restype = u32
    lib.SubspaceCRC32.argtypes = [u32, ctypes.c_void_p, ctypes.c_size_t]
    lib.SubspaceCRC32C.restype = u32
    lib.SubspaceCRC32C.argtypes = [u32, ctypes.c_void_p, ctypes.c_size_t]
    lib.subspace_crc_ctx_create_poly.restype = i32
    lib.subspace_crc_ctx_create_poly.argtypes = [i32, u32, ctypes.POINTER(vp)]
    lib.subspace_crc_version.restype = i32
    lib.subspace_crc_version.argtypes = []
    lib.subspace_crc_last_error.restype = ctypes.c_char_p
    lib.subspace_crc_last_error.argtypes = []
    lib.subspace_crc_ctx_create.restype = i32
    lib.subspace_crc_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.subspace_crc_ctx_destroy.restype = None
    lib.subspace_crc_ctx_destroy.argtypes = [vp]
    lib.subspace_crc_ctx_check.restype = i32
    lib.subspace_crc_ctx_check.argtypes = [vp, vp]
    lib.subspace_crc_ctx_reserve.restype = i32
    lib.subspace_crc_ctx_reserve.argtypes = [vp, u64, u64]
    lib.subspace_crc32_batch_uniform.restype = i32
    lib.subspace_crc32_batch_uniform.argtypes = [vp, vp, u64, u64, u64, u32, u32, vp, vp]
    lib.subspace_crc32_batch.restype = i32
    lib.subspace_crc32_batch.argtypes = [vp, vp, u64, vp, vp, u64, u32, u32, vp, vp]
    lib.subspace_crc32_slots.restype = i32
    lib.subspace_crc32_slots.argtypes = [vp, vp, u64, u64, ctypes.c_int32, ctypes.c_int32, u32, vp, vp, vp]
    lib.subspace_crc32_slots_strided.restype = i32
    lib.subspace_crc32_slots_strided.argtypes = [vp, vp, u64, u64, u64, vp, ctypes.c_int32, ctypes.c_int32, u32,
                                                 vp, vp, vp]
    lib.subspace_crc32_host_slots.restype = i32
    lib.subspace_crc32_host_slots.argtypes = [vp, vp, u64, u64, u64, vp, ctypes.c_int32, ctypes.c_int32, u32, vp, vp]
    lib.subspace_crc32_host_slot_list.restype = i32
    lib.subspace_crc32_host_slot_list.argtypes = [vp, vp, u64, u64, ctypes.c_int32, ctypes.c_int32, u32, vp, vp]
    lib.subspace_crc_host_register.restype = i32
    lib.subspace_crc_host_register.argtypes = [vp, u64]
    lib.subspace_crc_host_unregister.restype = i32
    lib.subspace_crc_host_unregister.argtypes = [vp]
    _lib = lib
    return lib


def load_dev() -> ctypes.CDLL:
    """Load (once) the development library (tests / bench / tools: never the product path)."""
    global _dev
    if _dev is not None:
        return _dev
    load()  # the product library first: the dev library acts on its contexts
    if not DEV_LIB_PATH.exists():
        raise LibraryNotBuilt(f"{DEV_LIB_PATH} not found: run `make` (or __graft_entry__.build()) first")
    lib = ctypes.CDLL(os.fspath(DEV_LIB_PATH), mode=ctypes.RTLD_LOCAL)
    u32, u64, vp, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
    lib.subspace_crc_testutil_fill_uniform.restype = i32
    lib.subspace_crc_testutil_fill_uniform.argtypes = [vp, u64, u64, u64, u64, u64, u64, vp]
    lib.subspace_crc_testutil_fill_ragged.restype = i32
    lib.subspace_crc_testutil_fill_ragged.argtypes = [vp, vp, vp, u64, u64, u64, u64, vp]
    lib.subspace_crc_testutil_tune.restype = i32
    lib.subspace_crc_testutil_tune.argtypes = [vp, i32, i32, i32]
    lib.subspace_crc_testutil_set.restype = i32
    lib.subspace_crc_testutil_set.argtypes = [vp, ctypes.c_char_p, i32]
    lib.subspace_crc_testutil_stream_read.restype = i32
    lib.subspace_crc_testutil_stream_read.argtypes = [vp, u64, vp, vp]
    lib.subspace_crc_testutil_stream_read_lds.restype = i32
    lib.subspace_crc_testutil_stream_read_lds.argtypes = [vp, u64, vp, ctypes.c_uint32, vp]
    lib.subspace_crc_testutil_uniform_alias.restype = i32
    lib.subspace_crc_testutil_uniform_alias.argtypes = [vp, vp, u64, vp, vp]
    lib.subspace_crc_testutil_probe.restype = i32
    lib.subspace_crc_testutil_probe.argtypes = [vp, vp]
    lib.subspace_crc_testutil_probe_waves.restype = u64
    lib.subspace_crc_testutil_probe_waves.argtypes = [vp, u64]
    lib.subspace_crc_testutil_slot_list_read.restype = i32
    lib.subspace_crc_testutil_slot_list_read.argtypes = [vp, u64, u32, u64, u32, vp, u64, vp]
    lib.subspace_crc_testutil_tile_list_read.restype = i32
    lib.subspace_crc_testutil_tile_list_read.argtypes = [vp, u64, vp, u64, vp]
    lib.subspace_crc_testutil_fault_words.restype = i32
    lib.subspace_crc_testutil_fault_words.argtypes = [vp, vp, vp]
    lib.subspace_crc_testutil_call_gen.restype = u32
    lib.subspace_crc_testutil_call_gen.argtypes = [vp]
    _dev = lib
    return lib


def last_error() -> str:
    msg = load().subspace_crc_last_error()
    return msg.decode() if msg else ""
