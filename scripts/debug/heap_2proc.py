"""Debug driver: the two-process symmetric-heap test body with per-step logging and a
stack dump (faulthandler) if a step stalls. Logs: gpurun_out/dbg_heap_r{rank}.log"""
import faulthandler
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))


def body(rank, world):
    os.makedirs("gpurun_out", exist_ok=True)
    f = open(f"gpurun_out/dbg_heap_r{rank}.log", "w", buffering=1)
    faulthandler.dump_traceback_later(60, exit=True, file=f)
    import builtins

    real_print = builtins.print
    builtins.print = lambda *a, **k: real_print(*a, **{**k, "file": f, "flush": True})
    import test_comm_native_gpu as T

    import dgraph_amd.comm.symheap as S

    orig_init = S.SymmetricHeap.__init__

    def init(self, *a, **k):
        print("heap init start")
        orig_init(self, *a, **k)
        print("heap init done, device_completion =", self.device_completion)

    S.SymmetricHeap.__init__ = init
    for name in ("remote_gather", "put_rows", "scatter_add", "barrier_stream", "register"):
        fn = getattr(S.SymmetricHeap, name)

        def wrap(self, *a, _fn=fn, _n=name, **k):
            print("->", _n)
            r = _fn(self, *a, **k)
            print("<-", _n)
            return r

        setattr(S.SymmetricHeap, name, wrap)
    T._heap_body(rank, world)
    print("body done")


if __name__ == "__main__":
    from conftest import run_ranks

    run_ranks(body, 2, timeout=150)
    print("ok")
