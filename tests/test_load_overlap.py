"""No tile load of a product kernel has its destination VGPRs overlapping its own address VGPRs
(hipcc assigns a tile's last load its dead address registers as destination
under register pressure, and the slot-list drain ran 8-9 us slower per 65,536-slot call for it,
profiles/r05/README.md). Compiles each kernel source for gfx950 (device code only) and reads its
disassembly with tools/load_overlap.py; skipped without hipcc."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

pytestmark = pytest.mark.skipif(not Path("/opt/rocm/bin/hipcc").exists(), reason="needs hipcc")


@pytest.mark.parametrize("src,kernels", [
    ("crc_uniform.hip", ("crc32_uniform4k_kernel",)),
    ("crc_small.hip", ("crc32_small_kernel",)),
    ("crc_long.hip", ("crc32_long_kernel",)),
    ("crc_ragged.hip", ("crc32_ragged_kernel",)),
])
def test_tile_loads_keep_their_address(src, kernels):
    from load_overlap import overlaps
    res = overlaps(ROOT / "subspace_amd" / "csrc" / src)
    checked = {k: v for k, v in res.items() if any(n in k for n in kernels) and "ELb1EEEv" not in k[-60:]}
    assert checked, f"no kernel of {kernels} found in {src}"
    bad = {k: v for k, v in checked.items() if v[0]}
    assert not bad, bad
