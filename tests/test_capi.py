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


def test_library_exports_only_the_header(lib):
    """the drop-in library exports the public header's functions and
    nothing else (kernel stubs, helpers and the development hooks stay out of it: the hooks
    live in libsubspace_crc_dev.so, which the product library does not need)."""
    import shutil
    import subprocess
    from subspace_amd import _lib
    if not shutil.which("nm"):
        pytest.skip("nm not available")
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True, check=True)
    names = {ln.split()[-1] for ln in nm.stdout.splitlines() if ln.strip()}
    assert names == set(_lib.EXPORTED_SYMBOLS)
    assert not any("testutil" in n for n in names)
    if shutil.which("readelf"):
        dyn = subprocess.run(["readelf", "-d", str(_lib.LIB_PATH)], capture_output=True, text=True, check=True).stdout
        assert "libsubspace_crc_dev" not in dyn


def test_dev_library_exports_the_hooks():
    from subspace_amd import _lib
    dev = _lib.load_dev()
    for n in ("subspace_crc_testutil_set", "subspace_crc_testutil_probe", "subspace_crc_testutil_fill_uniform",
              "subspace_crc_testutil_slot_list_read", "subspace_crc_testutil_fault_words"):
        assert hasattr(dev, n), n
    # a null / foreign context is refused before anything is touched
    assert dev.subspace_crc_testutil_set(None, b"small_path", 0) != 0
    assert dev.subspace_crc_testutil_tune(None, 512, 0, 0) != 0


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
