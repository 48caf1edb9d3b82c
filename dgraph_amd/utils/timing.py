"""``TimingReport``: named region timers (DGraph/utils/TimingReport.py:5-84 API).

The reference put a barrier + full device sync on both ends of every region
(TimingReport.py:43-75), which serialises the very overlap the library is built for.
Here, by default, ``start``/``stop`` only record HIP events on the current stream; the
elapsed times are resolved lazily (``resolve()`` / ``report()`` / ``_timers`` access)
after the events completed. ``TimingReport.init(comm, sync=True)`` restores the
reference's barrier-bracketed behaviour. CPU-only runs fall back to wall clock.

Also emits roctx ranges (``torch.cuda.nvtx`` maps to roctx on ROCm) so regions show up
in rocprofv3 ``--marker-trace`` timelines.
"""
from __future__ import annotations

import json
import time
from typing import Dict, List, Optional

import torch


class _Pending:
    __slots__ = ("start", "end", "t0")

    def __init__(self, start, t0):
        self.start = start
        self.end = None
        self.t0 = t0


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class TimingReport:
    _timers: Dict[str, List] = {}
    _communicator = None
    _is_initialized = False
    _sync = False
    _markers = False

    def __init__(self, name: Optional[str] = None):
        self.name = name

    def __enter__(self):
        if self.name is None:
            raise ValueError("A name must be provided to use TimingReport as a context manager.")
        self.start(self.name)
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        if self.name is not None:
            self.stop(self.name)
        return False

    @staticmethod
    def init(communicator=None, sync: bool = False, markers: bool = False):
        if TimingReport._is_initialized:
            raise RuntimeError("TimingReport is already initialized.")
        TimingReport._communicator = communicator
        TimingReport._is_initialized = True
        TimingReport._timers = {}
        TimingReport._sync = sync
        TimingReport._markers = markers

    @staticmethod
    def reset():
        TimingReport._timers = {}
        TimingReport._is_initialized = False
        TimingReport._communicator = None

    @staticmethod
    def _check():
        if not TimingReport._is_initialized:
            raise RuntimeError("TimingReport is not initialized. Call init first.")

    @staticmethod
    def start(name: str):
        TimingReport._check()
        if _capturing():
            return  # inside a HIP-graph capture: events would belong to the graph
        if TimingReport._sync and TimingReport._communicator is not None:
            TimingReport._communicator.barrier()
        lst = TimingReport._timers.setdefault(name, [])
        if torch.cuda.is_available():
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream())
            lst.append(_Pending(ev, None))
            if TimingReport._markers:
                torch.cuda.nvtx.range_push(name)
        else:
            lst.append(_Pending(None, time.perf_counter()))

    @staticmethod
    def stop(name: str):
        TimingReport._check()
        if _capturing():
            return None
        lst = TimingReport._timers.get(name)
        if not lst or not isinstance(lst[-1], _Pending):
            raise ValueError(f"No timer started for {name}")
        p = lst[-1]
        if p.start is not None:
            if TimingReport._markers:
                torch.cuda.nvtx.range_pop()
            p.end = torch.cuda.Event(enable_timing=True)
            p.end.record(torch.cuda.current_stream())
            if TimingReport._sync:
                torch.cuda.synchronize()
                lst[-1] = p.start.elapsed_time(p.end)
                if TimingReport._communicator is not None:
                    TimingReport._communicator.barrier()
                return lst[-1]
            return None
        lst[-1] = (time.perf_counter() - p.t0) * 1000.0
        return lst[-1]

    @staticmethod
    def add_time(name: str, elapsed_time: float):
        TimingReport._check()
        TimingReport._timers.setdefault(name, []).append(float(elapsed_time))

    @staticmethod
    def resolve() -> Dict[str, List[float]]:
        """Turn completed event pairs into milliseconds (synchronises once)."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        for name, lst in TimingReport._timers.items():
            for i, v in enumerate(lst):
                if isinstance(v, _Pending) and v.end is not None:
                    lst[i] = v.start.elapsed_time(v.end)
        return TimingReport._timers

    @staticmethod
    def report(skip_first: int = 0) -> Dict[str, dict]:
        out = {}
        for name, lst in TimingReport.resolve().items():
            vals = [v for v in lst if isinstance(v, float)][skip_first:]
            if vals:
                t = torch.tensor(vals)
                out[name] = {"n": len(vals), "mean_ms": float(t.mean()),
                             "min_ms": float(t.min()), "max_ms": float(t.max())}
        return out

    @staticmethod
    def dump(path: str) -> None:
        """``{region: [ms, ...]}`` JSON — the reference's timing-report file layout
        (``{log_dir}/{dataset}_timing_report_world{W}.json``, OGB/main.py:332-336)."""
        data = {k: [v for v in lst if isinstance(v, float)]
                for k, lst in TimingReport.resolve().items()}
        with open(path, "w") as f:
            json.dump(data, f)


class region:
    """``with region("name"):`` — a TimingReport region when TimingReport is initialised,
    otherwise a no-op (so models can be instrumented unconditionally)."""

    __slots__ = ("name", "on")

    def __init__(self, name: str):
        self.name = name
        self.on = False

    def __enter__(self):
        self.on = TimingReport._is_initialized
        if self.on:
            TimingReport.start(self.name)
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        if self.on:
            TimingReport.stop(self.name)
        return False
