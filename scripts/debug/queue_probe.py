#!/usr/bin/env python3
"""Do two streams run concurrently? A 20 ms device-side wait (link_delay, 1 wave) on a side
stream and a 20 ms wait on the current stream: ~20 ms total when they sit on different
hardware queues, ~40 ms when they share one (HIP serialises the packets of a queue).
Variants: side stream from torch's pool (normal priority, first / later pool entries) and
high priority. Prints GPU_MAX_HW_QUEUES as the process saw it."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if os.environ.get("PROBE_HWQ"):  # opt-in A/B of the queue budget (1..4 on the boxes)
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(max(int(os.environ["PROBE_HWQ"]), 1), 4))

import torch  # noqa: E402

from dgraph_amd import _native  # noqa: E402


def probe(side, label):
    ops = _native.ops()
    cur = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t = time.perf_counter()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        ops.link_delay(20000.0, 0, 1)
    ops.link_delay(20000.0, 0, 1)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3
    print(f"{label:40s} {ms:6.1f} ms  ({'CONCURRENT' if ms < 30 else 'SERIALISED'})",
          flush=True)


def main():
    _native.load()
    print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"))
    _native.ops().link_delay(10.0, 0, 1)
    torch.cuda.synchronize()
    for i in range(10):
        probe(torch.cuda.Stream(), f"pool stream #{i} (normal priority)")
    for i in range(3):
        probe(torch.cuda.Stream(priority=-1), f"pool stream #{i} (high priority)")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):  # a non-default compute stream
        for i in range(3):
            probe(torch.cuda.Stream(priority=-1), f"compute on pool stream, side hi #{i}")


if __name__ == "__main__":
    main()
