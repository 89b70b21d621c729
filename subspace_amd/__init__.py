"""subspace_amd: MI355X-native batched CRC32 for dallison/subspace's per-message
payload checksum path (client/checksum.{h,cc}, client/arm_crc32.S).

* ``subspace_amd.checksum`` -- host mirror of client/checksum.h (native SubspaceCRC32).
* ``subspace_amd.gpu``      -- batched device CRC32 through the C ABI (HIP kernels, gfx950).
"""
from .checksum import (calculate_crc32_checksum, compute_prefix_size, get_message_checksum_data,  # noqa: F401
                       subspace_crc32, verify_crc32_checksum)

__all__ = [
    "subspace_crc32",
    "calculate_crc32_checksum",
    "verify_crc32_checksum",
    "get_message_checksum_data",
    "compute_prefix_size",
]
