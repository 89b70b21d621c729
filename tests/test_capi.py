"""The C-ABI library loads and exports every symbol include/subspace_crc.h declares.
No compute calls that need a GPU happen here."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    hdr = (ROOT / "include" / "subspace_crc.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(SubspaceCRC32C?|subspace_crc\w+)\s*\(", hdr)))


def test_header_symbols_are_exported(lib):
    from subspace_amd import _lib
    names = declared_symbols()
    assert "SubspaceCRC32" in names and "subspace_crc32_batch" in names
    assert set(names) == set(_lib.EXPORTED_SYMBOLS)
    for n in names:
        assert hasattr(lib, n), n


def test_version_and_error_string(lib):
    assert lib.subspace_crc_version() >= 100
    assert isinstance(lib.subspace_crc_last_error(), bytes)


def test_null_args_rejected_without_gpu(lib):
    # argument validation happens before any device work
    assert lib.subspace_crc32_batch_uniform(None, None, 4096, 4096, 1, 0xFFFFFFFF, 0, None, None) == -1
    assert lib.subspace_crc32_batch(None, None, 0, None, None, 1, 0xFFFFFFFF, 0, None, None) == -1
    assert lib.subspace_crc_ctx_create(0, None) == -1


def test_no_device_is_reported(lib):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    rc = lib.subspace_crc_ctx_create(0, ctypes.byref(h))
    assert rc == -4  # SUBSPACE_CRC_ENODEV
    assert b"device" in lib.subspace_crc_last_error()


def test_gpu_entry_points_fail_loudly_without_device():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from subspace_amd.gpu import CrcContext, CrcError
    with pytest.raises(CrcError):
        CrcContext(0)
