"""Stage tracing, timing and metrics (the reference has only progress prints).

* :func:`stage` — context manager around one pipeline stage: a ROCTX range (``torch.cuda.nvtx``
  maps to roctx on ROCm builds, so the stage shows up in ``rocprofv3 --marker-trace`` /
  ``--kernel-trace`` timelines), HIP-event GPU time, host wall time, a rank-aware ``logging``
  line, and an optional JSONL metrics record (``MFA_METRICS=/path/metrics.jsonl``).
* :class:`Timer` — the per-object accumulator the models expose as ``.times.ms``.

GPU time is measured with events on the current stream, so a stage is not synchronised unless
``sync=True`` (or ``MFA_SYNC_STAGES=1``) asks for exact host-side wall times.
"""
from __future__ import annotations

import contextlib
import json
import logging
import os
import time

import torch

log = logging.getLogger("mfa")


def _sync_default() -> bool:
    return os.environ.get("MFA_SYNC_STAGES", "0") == "1"


def _rank() -> int:
    try:
        import torch.distributed as dist
        return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    except Exception:  # pragma: no cover
        return 0


def setup_logging(level: int = logging.INFO, rank: int | None = None) -> None:
    """Rank-aware logging: rank 0 at ``level``, other ranks at WARNING."""
    rank = _rank() if rank is None else rank
    fmt = f"%(asctime)s [rank {rank}] %(name)s %(levelname)s: %(message)s"
    logging.basicConfig(level=level if rank == 0 else logging.WARNING, format=fmt)


def emit(record: dict) -> None:
    """Append one JSON record to the metrics file (if ``MFA_METRICS`` is set)."""
    path = os.environ.get("MFA_METRICS")
    if not path:
        return
    rec = {"ts": time.time(), "rank": _rank(), **record}
    with open(path, "a") as fh:
        fh.write(json.dumps(rec, default=float) + "\n")


class Timer:
    """Accumulated milliseconds per stage name (host wall time; GPU time when available)."""

    def __init__(self):
        self.ms: dict[str, float] = {}
        self.gpu_ms: dict[str, float] = {}

    def add(self, name: str, wall_ms: float, gpu_ms: float | None = None) -> None:
        self.ms[name] = self.ms.get(name, 0.0) + wall_ms
        if gpu_ms is not None:
            self.gpu_ms[name] = self.gpu_ms.get(name, 0.0) + gpu_ms

    def table(self) -> str:
        rows = [f"{'stage':<16}{'wall ms':>12}{'gpu ms':>12}"]
        for k, v in self.ms.items():
            g = self.gpu_ms.get(k)
            rows.append(f"{k:<16}{v:>12.3f}{(f'{g:.3f}' if g is not None else '-'):>12}")
        return "\n".join(rows)


@contextlib.contextmanager
def stage(name: str, timer: Timer | None = None, device=None, sync: bool | None = None, **fields):
    """Trace one stage.  ``device`` (a CUDA device) enables HIP-event timing."""
    sync = _sync_default() if sync is None else sync
    cuda = device is not None and getattr(device, "type", None) == "cuda" and torch.cuda.is_available()
    ev0 = ev1 = None
    if cuda:
        torch.cuda.nvtx.range_push(name)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        gpu_ms = None
        if cuda:
            ev1.record()
            torch.cuda.nvtx.range_pop()
            if sync:
                ev1.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
        if cuda and sync:
            gpu_ms = ev0.elapsed_time(ev1)
        if timer is not None:
            timer.add(name, wall_ms, gpu_ms)
        log.debug("stage %s: %.3f ms wall%s", name, wall_ms,
                  f", {gpu_ms:.3f} ms gpu" if gpu_ms is not None else "")
        emit({"stage": name, "wall_ms": wall_ms, "gpu_ms": gpu_ms, **fields})
