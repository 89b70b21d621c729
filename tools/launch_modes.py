#!/usr/bin/env python3
"""Launch-mode experiment for the config-B step (investigation tool).

Wall time per step of the same uniform-kernel launches under different submission modes:
eager (with / without per-step events), hipGraph replay of R steps, two streams
alternating, and a graph whose steps are captured on two streams (independent nodes,
so one batch's ramp can overlap the previous batch's tail).

  python tools/launch_modes.py [--steps 400]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from subspace_amd import gpu  # noqa: E402

MSGS, MSG = 65536, 4096


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rotate", type=int, default=4)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    bufs = [torch.empty(MSGS * MSG, dtype=torch.uint8, device=dev) for _ in range(args.rotate)]
    outs = [torch.empty(MSGS, dtype=torch.int32, device=dev) for _ in range(args.rotate)]
    for k, b in enumerate(bufs):
        gpu.fill_uniform(b, MSG, MSG, MSGS, seed=0x5EED000B, first_id=k * MSGS)
    torch.cuda.synchronize()
    K = args.steps
    res = {}

    def launch(i, stream=None):
        k = i % args.rotate
        ctx.crc32_uniform(bufs[k], MSG, MSG, MSGS, outs[k], stream=stream)

    def timed(fn, n_steps):
        fn()  # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n_steps * 1e6

    # eager, no events
    res["eager"] = timed(lambda: [launch(i) for i in range(K)], K)

    # eager with events around every launch
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]

    def ev_loop():
        s = torch.cuda.current_stream()
        for i in range(K):
            evs[i][0].record(s)
            launch(i)
            evs[i][1].record(s)
    res["eager_events"] = timed(ev_loop, K)
    res["eager_events_kernel_us"] = sum(a.elapsed_time(b) for a, b in evs) / K * 1e3

    # two streams alternating
    s2 = [torch.cuda.Stream(), torch.cuda.Stream()]

    def two_streams():
        cur = torch.cuda.current_stream()
        for s in s2:
            s.wait_stream(cur)
        for i in range(K):
            launch(i, stream=s2[i & 1])
        for s in s2:
            cur.wait_stream(s)
    res["eager_2streams"] = timed(two_streams, K)

    # graphs
    for R in (args.rotate, 8 * args.rotate):
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            with torch.cuda.graph(g, stream=cap):
                for i in range(R):
                    launch(i)
        torch.cuda.synchronize()
        reps = K // R
        res[f"graph_{R}"] = timed(lambda: [g.replay() for _ in range(reps)], reps * R)

        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap):
            with torch.cuda.graph(g2, stream=cap):
                main = torch.cuda.current_stream()
                side = torch.cuda.Stream()
                side.wait_stream(main)
                for i in range(R):
                    if i & 1:
                        with torch.cuda.stream(side):
                            launch(i)
                    else:
                        launch(i)
                main.wait_stream(side)
        torch.cuda.synchronize()
        res[f"graph_{R}_2streams"] = timed(lambda: [g2.replay() for _ in range(reps)], reps * R)

    out = {k: round(v, 2) for k, v in res.items()}
    out["GiBps"] = {k: round(MSGS * MSG / (v * 1e-6) / 2**30, 1) for k, v in res.items() if not k.endswith("_us")}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
