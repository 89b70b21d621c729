"""Config S's channel (65,536 slots, 4 KiB payloads, stride 4,160) verified three ways on one
box, interleaved: the fused uniform slot kernel (subspace_crc32_slots_strided), and the
small-message kernel through subspace_crc32_slots with the records in channel order and
shuffled (bench.py's S_list). Separates the cost of the read order from the kernel's own.
One JSON line per round: ms per call of each.

  python tools/slot_list_order.py [rounds]
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from bench import time_calls
    from subspace_amd import gpu, slots
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n, size, cs, ms = 65536, 4096, 4, 0
    ps, stride = slots.compute_prefix_size(cs, ms), slots.slot_stride(size, cs, ms)
    rng = np.random.default_rng(0x5EED0005)
    host = rng.integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.full(n, size, dtype=np.uint64), checksum_size=cs,
                                                          metadata_size=ms, seed=5)
    buf = torch.from_numpy(host).to("cuda")
    ctx = gpu.CrcContext(0)
    ctx.crc32_slots_strided(buf, stride, n, message_size=size, checksum_size=cs, metadata_size=ms,
                            mode=gpu.SLOT_CALCULATE)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    errs = torch.zeros(1, dtype=torch.int32, device="cuda")
    base0 = np.uint64(buf.data_ptr())

    def recs(order):
        r = np.stack([base0 + order * np.uint64(stride), base0 + order * np.uint64(stride) + np.uint64(ps),
                      np.full(n, size, dtype=np.uint64)], axis=1)
        return torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to("cuda")

    ordered = recs(np.arange(n, dtype=np.uint64))
    shuffled = recs(rng.permutation(n).astype(np.uint64))
    calls = {
        "strided_fused": lambda: ctx.crc32_slots_strided(buf, stride, n, message_size=size, checksum_size=cs,
                                                         metadata_size=ms, mode=gpu.SLOT_VERIFY, status=status,
                                                         error_count=errs),
        "list_ordered": lambda: ctx.crc32_slots(ordered, max_message_size=size, checksum_size=cs, metadata_size=ms,
                                                mode=gpu.SLOT_VERIFY, status=status, error_count=errs),
        "list_shuffled": lambda: ctx.crc32_slots(shuffled, max_message_size=size, checksum_size=cs,
                                                 metadata_size=ms, mode=gpu.SLOT_VERIFY, status=status,
                                                 error_count=errs),
    }
    only = os.environ.get("SLOT_LIST_CALLS")  # e.g. "strided_fused,list_ordered" (timing-only variants
    if only:                                  # that assume channel order must not see the shuffled list)
        calls = {k: v for k, v in calls.items() if k in only.split(",")}
    for r in range(rounds):
        line = {"round": r}
        for k, fn in calls.items():
            line[k] = round(time_calls(fn, 200), 5)
            torch.cuda.synchronize()
            if not os.environ.get("SLOT_LIST_NOCHECK"):  # timing-only library variants compute nothing valid
                assert int(errs.item()) == 0 and bool((status == 0).all().item()), k
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
