"""Source checks of the HIP kernels that no CPU replay catches.

Wave-wide operations (ballots, __any / __all, cross-lane reads) inside a branch taken by some
lanes only see the active lanes: round 6's first REPACK2 build counted a wave's entries with a
ballot inside `if (lane == 0)`, so only lane 0 voted, the workgroup's entry count was wrong and a
later tile read a stale LDS record (a GPU memory fault, found with the SUBSPACE_RP2_DEBUG build).
This test fails on any such call inside a block (or one-line body) guarded by a per-lane
condition on `lane` or `threadIdx.x`."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
KERNELS = sorted((ROOT / "subspace_amd" / "csrc").glob("*.hip")) + [ROOT / "subspace_amd" / "csrc" / "crc_device.h"]
WAVE_OPS = re.compile(r"__ballot\(|__any\(|__all\(|__builtin_amdgcn_readlane\(|__builtin_amdgcn_ds_bpermute\(|"
                      r"__builtin_amdgcn_ds_permute\(|__builtin_amdgcn_update_dpp\(|__builtin_amdgcn_readfirstlane\(|"
                      r"\bbperm\(|\bwave_scan\(|\bmsg_value\(")
LANE_IF = re.compile(r"\bif\s*\((?:[^()]|\([^()]*\))*\b(?:lane|threadIdx\.x)\b\s*(?:==|<|>|<=|>=|!=)")


def lane_guarded_bodies(src: str):
    """(line number, body text) of every `if (... lane <op> ...)` statement's body."""
    for m in LANE_IF.finditer(src):
        # the condition's closing parenthesis
        i, depth = src.index("(", m.start()), 0
        while True:
            c = src[i]
            depth += c == "("
            depth -= c == ")"
            i += 1
            if depth == 0:
                break
        rest = src[i:]
        stripped = rest.lstrip()
        line = src.count("\n", 0, m.start()) + 1
        if stripped.startswith("{"):
            j, depth = i + (len(rest) - len(stripped)), 0
            start = j
            while True:
                c = src[j]
                depth += c == "{"
                depth -= c == "}"
                j += 1
                if depth == 0:
                    break
            yield line, src[start:j]
        else:
            yield line, rest[:rest.index(";") + 1]


@pytest.mark.parametrize("path", KERNELS, ids=lambda p: p.name)
def test_no_wave_wide_op_under_a_lane_condition(path):
    src = re.sub(r"//[^\n]*", "", path.read_text())
    bad = [(ln, WAVE_OPS.search(body).group(0)) for ln, body in lane_guarded_bodies(src) if WAVE_OPS.search(body)]
    assert not bad, f"{path.name}: wave-wide operations under a per-lane condition at lines {bad}"


def test_the_lint_catches_the_round6_defect():
    src = """if (lane == 0) {
        lds_st(a, 1u);
        lds_st(b, (u32)__builtin_popcountll(__ballot(r2n != 0u)));
      }
      if (lane == 63) lds_st(c, incl);"""
    bad = [body for _, body in lane_guarded_bodies(src) if WAVE_OPS.search(body)]
    assert len(bad) == 1 and "__ballot" in bad[0]
