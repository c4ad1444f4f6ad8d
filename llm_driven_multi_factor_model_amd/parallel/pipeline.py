"""Intra-GPU stage pipelining over date chunks with HIP streams ("PP").

The reference regresses one date at a time in a Python loop (``Barra-master/mfm/MFM.py:57-66``)
on host memory.  When the panel lives in host RAM (a CSV / Mongo load that is larger than the
working set one wants resident, or a feed that arrives in date chunks), the GPU path is bound by
the host->device copy, not by the regression kernel (0.11 ms per 1000 dates at N = 5000).  This
module streams a host-resident panel through the GPU in date chunks on three HIP streams:

    h2d stream:      copy chunk c's panel slice into device slot c % depth
    compute stream:  xs_wls (fused HIP kernel) on slot c % depth       (waits on h2d[c])
    d2h stream:      copy f / r2 / stats / status / resid back into pinned host results
                                                                      (waits on compute[c])

Slot reuse waits on the d2h event of chunk c - depth, so with depth >= 2 the copy of chunk c+1,
the regression of chunk c and the write-back of chunk c-1 overlap.  Near-singular dates (the
kernel's status bit) are re-solved with the pinv reference on the host afterwards, so the
pipeline never synchronises mid-stream.
"""
from __future__ import annotations

import torch

from ..ops.cross_section import XsResult, xs_wls, xs_wls_reference, xs_wls_workspace


def _pinned(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_pinned() else t.pin_memory()


def streamed_xs_wls(X: torch.Tensor, cap: torch.Tensor, ret: torch.Tensor, ind: torch.Tensor | None,
                    P: int, device: torch.device | str = "cuda", chunk: int = 512, depth: int = 3,
                    want_resid: bool = True, pivot_mode: int = 0, refine: bool = True) -> XsResult:
    """Regress a HOST panel (X [D,Q,N], cap/ret [D,N] in f64 or f32, ind [D,N] int16) chunk by
    chunk.

    Returns host (pinned) tensors identical to ``xs_wls`` on the whole panel.  CPU ``device``
    runs the reference path directly.
    """
    device = torch.device(device)
    D, Q, N = X.shape
    K = 1 + P + Q
    if device.type != "cuda":
        return xs_wls_reference(X, cap, ret, ind, P, pivot_mode=pivot_mode, want_resid=want_resid)
    if chunk < 1 or depth < 1:
        raise ValueError("chunk and depth must be >= 1")
    chunk = min(chunk, D)
    dt = X.dtype if X.dtype == torch.float64 else torch.float32
    X, cap, ret = (_pinned(t.to(dt).contiguous()) for t in (X, cap, ret))
    ind = _pinned(ind.contiguous()) if P > 0 else None

    pin = dict(dtype=torch.float64, pin_memory=True)
    res = XsResult(f=torch.empty(D, K, **pin),
                   resid=torch.empty(D, N, dtype=dt, pin_memory=True) if want_resid else None,
                   r2=torch.empty(D, **pin), stats=torch.empty(D, Q + 2, **pin),
                   status=torch.empty(D, dtype=torch.int32, pin_memory=True))

    nslot = min(depth, (D + chunk - 1) // chunk)
    dev_in, dev_out, ws = [], [], []
    for _ in range(nslot):
        dev_in.append((torch.empty(chunk, Q, N, dtype=dt, device=device),
                       torch.empty(chunk, N, dtype=dt, device=device),
                       torch.empty(chunk, N, dtype=dt, device=device),
                       torch.empty(chunk, N, dtype=torch.int16, device=device) if P > 0 else None))
        dev_out.append(XsResult(
            f=torch.empty(chunk, K, dtype=torch.float64, device=device),
            resid=torch.empty(chunk, N, dtype=dt, device=device) if want_resid else None,
            r2=torch.empty(chunk, dtype=torch.float64, device=device),
            stats=torch.empty(chunk, Q + 2, dtype=torch.float64, device=device),
            status=torch.empty(chunk, dtype=torch.int32, device=device)))
        # the kernel's workspace is not monotone in D (auto stock chunking picks more chunks
        # per date for fewer dates), so size the slot for every chunk length it will see
        lens = {chunk} | ({D % chunk} if D % chunk else set())
        ws.append(max((xs_wls_workspace(n, P, Q, device, N) for n in lens), key=lambda t: t.numel()))

    s_h2d, s_cmp, s_d2h = (torch.cuda.Stream(device) for _ in range(3))
    loaded = [torch.cuda.Event() for _ in range(nslot)]
    computed = [torch.cuda.Event() for _ in range(nslot)]
    freed: list[torch.cuda.Event | None] = [None] * nslot
    # every slot buffer was allocated on the caller's stream: order the side streams after it
    start = torch.cuda.Event()
    start.record(torch.cuda.current_stream(device))
    for s in (s_h2d, s_cmp, s_d2h):
        s.wait_event(start)

    for c, a in enumerate(range(0, D, chunk)):
        b = min(a + chunk, D)
        n = b - a
        k = c % nslot
        xi, ci, ri, ii = dev_in[k]
        o = dev_out[k]
        with torch.cuda.stream(s_h2d):
            if freed[k] is not None:
                s_h2d.wait_event(freed[k])
            xi[:n].copy_(X[a:b], non_blocking=True)
            ci[:n].copy_(cap[a:b], non_blocking=True)
            ri[:n].copy_(ret[a:b], non_blocking=True)
            if ii is not None:
                ii[:n].copy_(ind[a:b], non_blocking=True)
            loaded[k].record(s_h2d)
        with torch.cuda.stream(s_cmp):
            s_cmp.wait_event(loaded[k])
            view = XsResult(f=o.f[:n], resid=o.resid[:n] if want_resid else None, r2=o.r2[:n],
                            stats=o.stats[:n], status=o.status[:n])
            # device pinv of near-singular dates inside the chunk's stream (no host sync)
            xs_wls(xi[:n], ci[:n], ri[:n], ii[:n] if ii is not None else None, P,
                   pivot_mode=pivot_mode, want_resid=want_resid, refine=refine, out=view,
                   workspace=ws[k])
            computed[k].record(s_cmp)
        with torch.cuda.stream(s_d2h):
            s_d2h.wait_event(computed[k])
            res.f[a:b].copy_(o.f[:n], non_blocking=True)
            res.r2[a:b].copy_(o.r2[:n], non_blocking=True)
            res.stats[a:b].copy_(o.stats[:n], non_blocking=True)
            res.status[a:b].copy_(o.status[:n], non_blocking=True)
            if want_resid:
                res.resid[a:b].copy_(o.resid[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s_d2h)
            freed[k] = ev
    s_d2h.synchronize()
    torch.cuda.current_stream(device).wait_stream(s_d2h)

    return res


__all__ = ["streamed_xs_wls"]
