"""bench.py's multi-rank launch path on the CPU (gloo), through bench.py itself.

`python bench.py --gpus N --dry-run-cpu` runs the same code as a GPU run of N ranks -- the
parent spawns N rank processes through torch.distributed.run, each rank builds its shard
(round-robin for E, byte-balanced contiguous ranges for C), times its steps between
barriers with a max-over-ranks reduction and all_gathers its 4-byte CRCs -- with the
library's host SubspaceCRC32 in place of the kernel and gloo in place of RCCL. Rank 0
checks the gathered list against the committed fixture hash (tests/golden/configs.json).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def run_bench(*args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


def last_json(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("world,workload", [(2, "E"), (2, "C"), (3, "C"), (8, "E"), (8, "C")])
def test_dry_run_spawns_ranks_and_matches_fixture(world, workload):
    """Worlds 2, 3 and the driver's 8. Rank 0's solo leg (the N = 1
    configuration, the efficiency's denominator) settles by the headline's rule
    (bench.settle_steps) before it is timed, and is bit-exact too."""
    r = run_bench("--gpus", str(world), "--dry-run-cpu", "--workload", workload, "--steps", "2", "--warmup", "1",
                  "--settle", "2", "--settle-s", "0.3")
    assert r.returncode == 0, r.stderr[-3000:]
    line = last_json(r.stdout)
    solo = line["single_gpu"]
    assert solo["settle_launches"] >= 2 and solo["settle_s"] >= 0.3
    assert solo["bitexact_vs_golden"] is True and solo["value"] > 0
    assert line["efficiency"] == pytest.approx(line["value"] / (world * solo["value"]), rel=1e-2)
    assert line["n_gpus"] == world
    assert line["bitexact_vs_golden"] is True
    assert line["scaling"] == "strong"
    assert line["value"] > 0 and line["per_gpu_value"] == pytest.approx(line["value"] / world, rel=1e-2)
    # the line is self-checking: the process group's size, the backend and one record per rank
    assert line["rccl_world"] == world and line["backend"] == "gloo"
    assert sorted(r["rank"] for r in line["ranks"]) == list(range(world))
    assert len({r["pid"] for r in line["ranks"]}) == world  # N distinct rank processes
    assert line["rank_step_ms"]["min"] <= line["rank_step_ms"]["max"]


def test_dry_run_single_rank_default_workload():
    r = run_bench("--dry-run-cpu", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-3000:]
    line = last_json(r.stdout)
    assert line["n_gpus"] == 1 and line["bitexact_vs_golden"] is True and line["scaling"] == "weak"


def test_world_size_must_match_gpus():
    r = run_bench("--gpus", "2", "--dry-run-cpu", env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_solo_leg_settles_like_the_headline():
    """The GPU run's N > 1 solo leg calls run_timed with the headline's settle arguments
    (--settle, --settle-s), not a cold start; settle_steps honours both
    bounds and reports the launches it ran."""
    mod = _bench_module()
    src = (ROOT / "bench.py").read_text()
    solo = src[src.index("the headline's settle rule (VERDICT r04 item 4)"):]
    call = solo[solo.index("run_timed(one,"):solo.index("ok1, _ = one.check")]
    assert "args.settle," in call and "settle_s=args.settle_s" in call
    calls = []
    n, t = mod.settle_steps(lambda i: calls.append(i), lambda: None, 120, 20, 0.05, block=10)
    assert n >= 100 and n == len(calls) and n % 10 == 0 and t >= 0.05
    n, t = mod.settle_steps(lambda i: None, lambda: None, 0, 0, 0.0)
    assert n == 0


def test_settle_waits_for_a_steady_launch_rate():
    """bench.py settles until the launch rate stops improving (a background VRAM wipe after a
    large free slows every HBM-bound kernel for seconds): a window shorter than 1 s or one whose
    newer half is faster than its older half is not steady; a flat or slowing one is."""
    steady = _bench_module().launch_rate_steady
    assert not steady([(0.01, 50)] * 50)  # 0.5 s: too short
    assert steady([(0.01, 50)] * 100)
    assert not steady([(0.0104, 50)] * 60 + [(0.0100, 50)] * 60)  # still speeding up (4 %)
    assert steady([(0.01002, 50)] * 60 + [(0.0100, 50)] * 60)  # within 0.3 %
    assert steady([(0.0100, 50)] * 60 + [(0.0104, 50)] * 60)  # slowing down: nothing to wait for


def _rank_envs(stdout: str) -> dict:
    """The rank records in the launcher's stdout. Each rank writes its record as one write(2) of
    a whole line (bench.py), so lines never interleave; the records are still decoded wherever
    they start in a line, so a launcher's own output on the same line cannot hide one."""
    dec, recs = json.JSONDecoder(), []
    for ln in stdout.splitlines():
        i = ln.find('{"rank"')
        while i >= 0:
            rec, end = dec.raw_decode(ln, i)
            recs.append(rec)
            i = ln.find('{"rank"', end)
    return {r["rank"]: r["env"] for r in recs}


def test_rank_records_parse_even_when_two_share_a_line():
    a = json.dumps({"rank": 0, "env": {"X": "1"}})
    b = json.dumps({"rank": 1, "env": {"X": "1"}})
    assert _rank_envs(a + b + "\n\n") == {0: {"X": "1"}, 1: {"X": "1"}}
    assert _rank_envs("noise " + a + "\n" + b + "\n") == {0: {"X": "1"}, 1: {"X": "1"}}


def test_both_launch_forms_give_ranks_the_same_environment():
    """the driver starts `python -m torch.distributed.run --nproc-per-node N
    ... bench.py --gpus N`, a plain `python bench.py --gpus N` spawns the same itself. In both,
    every rank must see HSA_ENABLE_IPC_MODE_LEGACY=0 before torch or HIP initialise (bench.py
    apply_rank_env, first thing in main), even when the parent environment lacks it."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HSA_ENABLE_IPC_MODE_LEGACY")}
    env["PYTHONUNBUFFERED"] = "1"  # (the condition of the round-5 flake: print's two writes per record)
    spawn = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--print-rank-env"],
                           capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert spawn.returncode == 0, spawn.stderr[-3000:]
    port = _bench_module().free_port()
    driver = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                             "--master-addr=127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"),
                             "--gpus", "2", "--print-rank-env"],
                            capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert driver.returncode == 0, driver.stderr[-3000:]
    a, b = _rank_envs(spawn.stdout), _rank_envs(driver.stdout)
    assert sorted(a) == sorted(b) == [0, 1]
    assert a == b
    for r in (0, 1):
        assert a[r]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert a[r]["WORLD_SIZE"] == "2" and a[r]["MASTER_ADDR"] == "127.0.0.1"
    # a value the caller sets is kept, not overridden
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    again = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--print-rank-env"],
                           capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert _rank_envs(again.stdout) == a


def test_default_secondary_configs_cover_every_row():
    """the driver's default line carries Cu (config C at unaligned
    offsets) and S_large (the reference's 32 KiB checksum channel) beside the other rows."""
    import re
    src = (Path(__file__).resolve().parent.parent / "bench.py").read_text()
    m = re.search(r'cfg_names = args\.configs if args\.configs is not None else \("([^"]+)"', src)
    assert m, "default config list not found"
    names = m.group(1).split(",")
    for want in ("C", "Cu", "D", "Du", "S", "Usmall", "S_short", "S_mixed", "S_large"):
        assert want in names, want
