"""Date-sharded data parallelism (one process per GPU, RCCL over xGMI via torch.distributed).

The reference is single-process Python.  Here every cross-sectional stage is
independent per date, so rank r owns a contiguous block of dates; time-axis stages (Newey-West,
VRA) need the full factor-return series, which is one ``all_gather`` per stage (a few hundred
KB: latency-bound on xGMI, so the rule is ONE batched collective per stage, never per date).

Collective call sites:
  C3 factor-return series      all_gather   (D_local x K fp64)
  C5 MC bias accumulators      all_reduce   (D x K fp64, sims-sharded eigen adjustment)
  C6 VRA bias series           all_gather   (D_local fp64)
  C7 outputs to rank 0         gather       (only when writing CSVs: result series, the
                                             barra frame's owned rows as one fp64 block)
  C10 t+1 return across blocks all_gather   ([2, N] first-row value / presence per stock)
  C11 global stock axis        all_reduce   ([N] keep mask, MAX) + [world] kept-date counts
  C8 benchmark fences          barrier
  C9 stock-sharded (TP) CS-WLS all_reduce   (D x msize moments, then D x 5 R^2 sums;
                                             ops/xs_sharded.py)
Backend ``nccl`` is RCCL on ROCm builds; ``gloo`` serves CPU tests.

Failure detection: every process group gets a collective timeout
(``MFA_DIST_TIMEOUT_S``, default 600 s) and RCCL async error handling is on, so a dead or hung
rank turns into an exception on the others (fail fast; single node, no elastic restart) instead
of a silent hang.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from datetime import timedelta

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None
    force: bool = False  # MFA_FORCE_PG=1: a one-rank process group still runs the collectives

    @property
    def enabled(self) -> bool:
        return (self.world > 1 or self.force) and dist.is_available() and dist.is_initialized()


_CTX: DistContext | None = None


def init_distributed(backend: str | None = None, device: str | None = None) -> DistContext:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    global _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and device != "cpu"
    # MFA_DIST_BACKEND (e.g. gloo) rehearses a multi-rank run with several ranks per GPU (local
    # rank modulo the visible devices); RCCL itself refuses two ranks on one device.
    rehearse = os.environ.get("MFA_DIST_BACKEND")
    gpu = local % max(1, torch.cuda.device_count()) if use_cuda and rehearse else local
    dev = torch.device(f"cuda:{gpu}") if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(dev)
    be = backend or rehearse or ("nccl" if use_cuda else "gloo")
    # MFA_FORCE_PG=1 (under torchrun): a process group and every collective even at world size
    # 1 -- on one GPU that runs the RCCL paths themselves (communicator init with device_id, the
    # collectives on RCCL's stream next to captured graphs), which several ranks cannot do there
    force = os.environ.get("MFA_FORCE_PG") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = {"device_id": dev} if use_cuda and be == "nccl" else {}
        dist.init_process_group(be, rank=rank, world_size=world, timeout=collective_timeout(), **kw)
    _CTX = DistContext(rank, world, local, dev, be if (world > 1 or force) else None, force)
    return _CTX


def collective_timeout() -> timedelta:
    """Per-collective timeout of the process group (``MFA_DIST_TIMEOUT_S``, default 600 s)."""
    return timedelta(seconds=float(os.environ.get("MFA_DIST_TIMEOUT_S", "600")))


def context() -> DistContext:
    if _CTX is not None:
        return _CTX
    if dist.is_available() and dist.is_initialized():
        r, w = dist.get_rank(), dist.get_world_size()
        dev = torch.device(f"cuda:{torch.cuda.current_device()}") if torch.cuda.is_available() \
            and dist.get_backend() == "nccl" else torch.device("cpu")
        return DistContext(r, w, int(os.environ.get("LOCAL_RANK", "0")), dev, dist.get_backend())
    return DistContext()


def shard_range(D: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced date block [a, b) of rank ``rank``."""
    base, rem = divmod(D, world)
    a = rank * base + min(rank, rem)
    return a, a + base + (1 if rank < rem else 0)


def shard_sizes(n_local: int, ctx: DistContext | None = None) -> list[int]:
    """Leading-dim block size of every rank (one small collective; callers cache the result
    and pass it to :func:`all_gather_rows` so the per-stage gathers need no size exchange)."""
    ctx = ctx or context()
    if not ctx.enabled:
        return [int(n_local)]
    n = torch.tensor([n_local], dtype=torch.int64, device=ctx.device)
    out = torch.empty(ctx.world, dtype=torch.int64, device=ctx.device)
    dist.all_gather_into_tensor(out, n)
    return [int(v) for v in out.cpu().tolist()]


def all_gather_rows(x: torch.Tensor, ctx: DistContext | None = None,
                    sizes: list[int] | None = None) -> torch.Tensor:
    """Concatenate every rank's leading-dim block in rank order (blocks may differ in size).

    With ``sizes`` (every rank's block length, e.g. from :func:`shard_sizes`) this is ONE
    collective with no host synchronisation; without it the sizes are exchanged first."""
    ctx = ctx or context()
    if not ctx.enabled:
        return x
    if sizes is None:
        sizes = shard_sizes(x.shape[0], ctx)
    if sizes[ctx.rank] != x.shape[0]:
        raise ValueError(f"all_gather_rows: local block has {x.shape[0]} rows, sizes say "
                         f"{sizes[ctx.rank]}")
    mx = max(sizes)
    if all(s == mx for s in sizes):
        out = torch.empty((ctx.world * mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous())
        return out
    pad = torch.zeros((mx - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    xp = torch.cat([x, pad]) if mx > x.shape[0] else x.contiguous()
    out = torch.empty((ctx.world * mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, xp)
    return torch.cat([out[r * mx:r * mx + sizes[r]] for r in range(ctx.world)])


def halo_prev_rows(x: torch.Tensor, h: int, ctx: DistContext | None = None,
                   sizes: list[int] | None = None) -> torch.Tensor:
    """The ``h`` rows of the GLOBAL series that precede this rank's block (rank order =
    calendar order), NaN before the first global row: a rolling window's halo across rank
    boundaries.  One collective: every rank contributes its last min(h, D_r) rows, so a block
    shorter than the halo is covered by the ranks before it.  Float tensors only."""
    ctx = ctx or context()
    shape = (h,) + tuple(x.shape[1:])
    nan = torch.full(shape, float("nan"), dtype=x.dtype, device=x.device)
    if h <= 0:
        return nan[:0]
    if not ctx.enabled:
        return nan
    if sizes is None:
        sizes = shard_sizes(x.shape[0], ctx)
    k = min(h, x.shape[0])
    tail = nan.clone()
    if k:
        tail[h - k:] = x[x.shape[0] - k:]
    out = torch.empty((ctx.world * h,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, tail.contiguous())
    prev = [out[r * h + h - min(h, sizes[r]):(r + 1) * h] for r in range(ctx.rank)]
    got = torch.cat([nan] + prev)[-h:]
    return got.contiguous()


def broadcast_last_row(x: torch.Tensor, ctx: DistContext | None = None,
                       sizes: list[int] | None = None) -> torch.Tensor:
    """Row ``x[-1]`` of the rank that owns the LAST global row, on every rank."""
    ctx = ctx or context()
    if not ctx.enabled:
        return x[-1]
    if sizes is None:
        sizes = shard_sizes(x.shape[0], ctx)
    owner = max(r for r in range(ctx.world) if sizes[r] > 0)
    row = x[-1].contiguous().clone() if ctx.rank == owner else \
        torch.empty(tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.broadcast(row, src=owner)
    return row


def gather_to_root(x: torch.Tensor, ctx: DistContext | None = None,
                   sizes: list[int] | None = None) -> torch.Tensor | None:
    """Rows of every rank concatenated on rank 0 (None elsewhere).

    A real gather: each rank sends its exact block to rank 0 (point-to-point, all receives
    posted at once on the root), so only the root ever holds the whole tensor -- the barra
    frame at 5000 x 2520 is ~1.4 GB, which an all-gather would put on every GPU."""
    ctx = ctx or context()
    if not ctx.enabled:
        return x
    if sizes is None:
        sizes = shard_sizes(x.shape[0], ctx)
    if sizes[ctx.rank] != x.shape[0]:
        raise ValueError(f"gather_to_root: local block has {x.shape[0]} rows, sizes say "
                         f"{sizes[ctx.rank]}")
    if ctx.rank != 0:
        if x.shape[0]:
            dist.send(x.contiguous(), dst=0)
        return None
    out = torch.empty((sum(sizes),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    out[:sizes[0]] = x
    reqs, off = [], sizes[0]
    for r in range(1, ctx.world):
        if sizes[r]:
            reqs.append(dist.irecv(out[off:off + sizes[r]], src=r))
        off += sizes[r]
    for q in reqs:
        q.wait()
    return out


def all_reduce_max(x: float, ctx: DistContext | None = None, device=None) -> float:
    ctx = ctx or context()
    if not ctx.enabled:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_max_(x: torch.Tensor, ctx: DistContext | None = None) -> torch.Tensor:
    """In-place elementwise MAX over ranks (e.g. the global stock-axis keep mask of a
    date-sharded risk panel)."""
    ctx = ctx or context()
    if ctx.enabled:
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
    return x


def all_reduce_sum(x: torch.Tensor, ctx: DistContext | None = None) -> torch.Tensor:
    """In-place SUM over ranks (one collective for the whole tensor)."""
    ctx = ctx or context()
    if ctx.enabled:
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x


def barrier(ctx: DistContext | None = None) -> None:
    ctx = ctx or context()
    if ctx.enabled:
        dist.barrier()
