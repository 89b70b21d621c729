"""bench.py's multi-rank GPU path, rehearsed on one GPU (the 8-GPU runs are the driver's).

`python bench.py --gpus 2 --rehearse-one-gpu` spawns two ranks through
torch.distributed.run exactly as `--gpus 2` does, but both ranks use cuda:0 and gloo stands
in for RCCL: each rank builds its shard on the GPU, runs the kernels, times its steps
between barriers (max over ranks), all_gathers its 4-byte CRCs from device tensors, rank 0
checks the whole list against the fixture hash and then times the whole batch alone on its
GPU (the efficiency leg). Rates are not scaling numbers here (the ranks share one GPU)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("workload", ["E", "B"])
def test_two_ranks_on_one_gpu(workload):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--rehearse-one-gpu", "--workload",
                        workload, "--steps", "5", "--warmup", "1", "--settle", "0"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["single_gpu"]["bitexact_vs_golden"] is True
    # self-checking fields: the process group's size and backend, one record per rank
    assert d["rccl_world"] == 2 and d["backend"] == "gloo"
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1]
    assert d["distinct_gpus"] == 1  # both ranks rehearse on cuda:0 (a real N-GPU run shows N)
    assert d["rank_step_ms"]["min"] <= d["rank_step_ms"]["max"]
    if workload == "E":
        assert d["bitexact_vs_golden"] is True and d["scaling"] == "strong"
        g = d["config"]["gather"]
        # the gather is timed on the device (HIP events around the collective + on-device
        # interleave); the D2H copy and host check are reported apart
        assert g["gather_ms"] > 0 and g["d2h_check_ms"] > 0 and g["gather_bytes"] == 8 * 2**20 * 4
    assert d["efficiency"] > 0 and d["per_gpu_value"] == pytest.approx(d["value"] / 2, rel=1e-2)


def test_rccl_path_one_rank():
    """The RCCL branch of bench.py on the one-GPU box: launched by torch.distributed.run with
    one rank, bench.py creates the "nccl" (RCCL) process group with device_id, times between
    RCCL barriers with the max-over-ranks all_reduce, gathers the CRCs with an RCCL all_gather
    (into global order on the device) and gathers every rank's record -- the code an N-GPU run
    executes, with N = 1. Workload E: the whole 8 Mi x 4 KiB batch, checked against its fixture."""
    import socket
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                        "--gpus", "1", "--workload", "E", "--steps", "3", "--warmup", "1", "--settle", "0"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["backend"] == "nccl" and d["rccl_world"] == 1 and d["n_gpus"] == 1
    assert d["bitexact_vs_golden"] is True
    assert d["config"]["gather"]["gather_ms"] > 0 and d["ranks"][0]["rank"] == 0


def test_single_gpu_line_reports_read_ceiling():
    """The N = 1 config-B line carries the measured read ceiling of the same access shape
    (SURVEY.md 8d): the stream-read probe over the same rotated batches, and the CRC kernel's
    fraction of it (< 1: the CRC kernel reads the same bytes plus its compute)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "50", "--warmup", "2", "--settle", "0",
                        "--configs", "none", "--no-cpu-baseline", "--no-e2e"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(lines[-1])
    assert d["bitexact_vs_golden"] is True
    ceil = d["roofline"]["read_ceiling"]
    assert ceil["us_per_launch"] > 0 and ceil["GBps"] > 1000
    assert 0.5 < d["roofline"]["frac_of_read_ceiling"] < 1.05
