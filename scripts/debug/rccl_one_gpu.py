#!/usr/bin/env python3
"""Bring-up probe: can two processes that share ONE GPU form an RCCL communicator?

RCCL refuses two ranks on one device when it believes they share a host ("Duplicate GPU
detected"); with a distinct NCCL_HOSTID per rank each rank looks like its own host, so the
pair connects over the socket network transport on the loopback interface (host-staged,
slow — this is a correctness path, not a bandwidth one). If it works, the torch-PG RCCL
all-to-all-v and the native grouped send/recv executor (comm/rccl_exec.py) can be tested
across real ranks on a one-GPU box.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def body(rank: int, world: int, port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0",
                      NCCL_HOSTID=f"dgraph-rank{rank}", NCCL_SOCKET_IFNAME="lo")
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t0 = time.time()
    x = torch.full((1 << 16,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    assert float(x[0]) == world * (world + 1) / 2, float(x[0])
    print(f"[r{rank}] all_reduce ok {time.time() - t0:.2f}s", flush=True)
    send_splits = [3 + 2 * p + rank for p in range(world)]
    recv_splits = [3 + 2 * rank + p for p in range(world)]
    F = 40
    send = torch.cat([torch.full((n, F), float(100 * rank + p), device=dev)
                      for p, n in enumerate(send_splits)])
    out = torch.empty(sum(recv_splits), F, device=dev)
    dist.all_to_all_single(out, send, recv_splits, send_splits)
    exp = torch.cat([torch.full((n, F), float(100 * p + rank), device=dev)
                     for p, n in enumerate(recv_splits)])
    torch.cuda.synchronize()
    assert torch.equal(out, exp)
    print(f"[r{rank}] torch all_to_all_single ok", flush=True)
    from dgraph_amd.comm.rccl_exec import RCCLExecutor

    ex = RCCLExecutor.for_group(None)
    out2 = torch.empty_like(out)
    ex.alltoallv([send], [out2], send_splits, recv_splits)
    torch.cuda.synchronize()
    assert torch.equal(out2, exp)
    out3 = torch.zeros_like(out)
    w = ex.alltoallv([send], [out3], send_splits, recv_splits, async_op=True)
    w.wait()
    assert torch.equal(out3, exp)
    print(f"[r{rank}] native executor ok", flush=True)
    RCCLExecutor.close_all()
    dist.destroy_process_group()


if __name__ == "__main__":
    import multiprocessing as mp

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=body, args=(r, world, 29611)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(150)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    print("exit codes", codes, flush=True)
    sys.exit(0 if all(c == 0 for c in codes) else 1)
