"""Timing and metrics.

The reference times with CUDA events on the legacy default stream and ``clock_gettime`` between
pthread barriers, and prints ``"Total GPU encoding time: %fms"`` lines; throughput is derived by
hand (``doc/design.tex:490``). Here: events on the work stream (never the default stream),
host wall clocks, and a JSON-lines metrics sink that records MB/s the way the reference's docs
define it (file KB/1024 / seconds) next to GB/s.
"""
from __future__ import annotations

import json
import sys
import time
from contextlib import contextmanager

import torch


@contextmanager
def trace_range(name: str):
    """A roctx range (rocprofv3 --marker-trace) around host code; a no-op without the roctx library.

    Uses the native module's dlopen'ed roctx (csrc/include/gfrs/trace.h), the same ranges the C++
    pipeline and the streaming codec emit, so Python and native stages share one timeline.
    """
    try:
        from .._native import cpu
        c = cpu()
    except Exception:  # native module not built: tracing is optional
        c = None
    if c is not None:
        c.trace_push(name)
    try:
        yield
    finally:
        if c is not None:
            c.trace_pop()


class CudaTimer:
    """Elapsed device time of work enqueued on ``stream`` between start() and stop()."""

    def __init__(self, stream: torch.cuda.Stream | None = None):
        self.stream = stream
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.t1 = torch.cuda.Event(enable_timing=True)

    def start(self):
        self.t0.record(self.stream or torch.cuda.current_stream())
        return self

    def stop(self):
        self.t1.record(self.stream or torch.cuda.current_stream())
        return self

    def ms(self) -> float:
        self.t1.synchronize()
        return self.t0.elapsed_time(self.t1)


@contextmanager
def wall(result: dict, key: str):
    t = time.perf_counter()
    try:
        yield
    finally:
        result[key] = (time.perf_counter() - t) * 1e3


def mbps(nbytes: int, ms: float) -> float:
    """Reference definition: MB (2^20 bytes) per second."""
    return nbytes / 1048576.0 / (ms / 1e3) if ms > 0 else float("inf")


def gbps(nbytes: int, ms: float) -> float:
    return nbytes / 1e9 / (ms / 1e3) if ms > 0 else float("inf")


class Metrics:
    """Append-only JSON-lines sink (stdout by default)."""

    def __init__(self, path: str | None = None):
        self.f = open(path, "a") if path else sys.stdout

    def log(self, **rec) -> None:
        rec.setdefault("ts", time.time())
        self.f.write(json.dumps(rec) + "\n")
        self.f.flush()
