#!/usr/bin/env python3
"""Resident device memory of the headline bench job after setup: every CUDA storage reachable
from the Job / executor / graph objects, largest first, with the attribute path that holds
it (the W=1 headroom item of VERDICT r4)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402


def walk(obj, path, seen, out, depth=0):
    if depth > 4 or id(obj) in seen:
        return
    seen.add(id(obj))
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            st = obj.untyped_storage()
            out.setdefault(st.data_ptr(), (st.nbytes(), path))
        return
    if isinstance(obj, (list, tuple)):
        for i, v in enumerate(obj):
            walk(v, f"{path}[{i}]", seen, out, depth + 1)
        return
    if isinstance(obj, dict):
        for k, v in list(obj.items())[:200]:
            walk(v, f"{path}[{k!r}]", seen, out, depth + 1)
        return
    d = getattr(obj, "__dict__", None)
    if d is not None and type(obj).__module__.startswith(("dgraph_amd", "__main__", "bench")):
        for k, v in d.items():
            walk(v, f"{path}.{k}", seen, out, depth + 1)
    slots = getattr(type(obj), "__slots__", ())
    for k in slots if isinstance(slots, (list, tuple)) else ():
        if hasattr(obj, k):
            walk(getattr(obj, k), f"{path}.{k}", seen, out, depth + 1)


def main():
    import bench

    args = bench.parse()
    comm = type("C", (), {"get_rank": staticmethod(lambda: 0),
                          "get_world_size": staticmethod(lambda: 1), "group": None})()
    dev = torch.device("cuda", 0)
    job = bench.Job(args, comm, dev, args.global_frac, torch.float32)
    torch.cuda.synchronize()
    out = {}
    walk(job, "job", set(), out)
    walk(job.model, "model", set(), out)
    tot = sum(n for n, _ in out.values())
    print(f"allocated {torch.cuda.memory_allocated() / 1e9:.2f} GB, reachable {tot / 1e9:.2f} GB"
          f" in {len(out)} storages", flush=True)
    for n, p in sorted(out.values(), reverse=True)[:45]:
        print(f"  {n / 1e9:9.3f} GB  {p}", flush=True)


if __name__ == "__main__":
    main()
