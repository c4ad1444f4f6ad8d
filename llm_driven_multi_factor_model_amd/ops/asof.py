"""Device-side point-in-time as-of join (K12, ``csrc/asof.hip``).

Reference: ``Barra_factor_cal/load_data.py:41-62`` (``robust_merge_asof``: a per-``ts_code``
``pd.merge_asof(direction='backward')`` loop).  :func:`asof_search` returns, for every left row,
the index of the last right row with the same group and key <= the left key (-1 if none);
:func:`asof_gather` pulls the matched fp32 statement columns onto the daily rows (NaN where no
statement had been announced yet).  Inputs are sorted by (group, key) on both sides, as in
``utils.pit.asof_indices`` (the host path, ``csrc_host/asof.cpp``), which this matches exactly.

CPU tensors take the numpy/host path; CUDA tensors always run the HIP kernels (no fallback).
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native

_native.register("mfa_asof_search", [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                      C.c_int64, C.c_void_p, C.c_void_p])
_native.register("mfa_asof_gather", [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int,
                                      C.c_void_p, C.c_void_p])


def _check_sorted(g: torch.Tensor, k: torch.Tensor, name: str) -> None:
    if g.numel() < 2:
        return
    dg = g[1:] - g[:-1]
    bad = (dg < 0) | ((dg == 0) & (k[1:] < k[:-1]))
    if bool(bad.any()):
        raise ValueError(f"{name}: rows must be sorted by (group, key)")


def asof_search(left_groups: torch.Tensor, left_keys: torch.Tensor, right_groups: torch.Tensor,
                right_keys: torch.Tensor, check_sorted: bool = True) -> torch.Tensor:
    """int64 [nl]: last right row of the same group with key <= left key, else -1."""
    lg = left_groups.to(torch.int32).contiguous()
    lk = left_keys.to(torch.int64).contiguous()
    rg = right_groups.to(torch.int32).contiguous().to(lg.device)
    rk = right_keys.to(torch.int64).contiguous().to(lg.device)
    if lg.shape != lk.shape or rg.shape != rk.shape or lg.dim() != 1 or rg.dim() != 1:
        raise ValueError("asof_search: groups/keys must be matching 1-D tensors")
    if check_sorted:
        _check_sorted(lg, lk, "left")
        _check_sorted(rg, rk, "right")
    if not lg.is_cuda:
        from ..utils.pit import asof_indices
        return torch.from_numpy(asof_indices(lg.numpy(), lk.numpy(), rg.numpy(), rk.numpy()))
    out = torch.empty(lg.numel(), dtype=torch.int64, device=lg.device)
    _native.call("mfa_asof_search", _native.ptr(lg), _native.ptr(lk), lg.numel(), _native.ptr(rg),
                 _native.ptr(rk), rg.numel(), _native.ptr(out), _native.stream(lg.device))
    return out


def asof_gather(right_values: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """fp32 [nl, C]: ``right_values[idx]`` with NaN rows where ``idx < 0``."""
    rv = right_values.to(torch.float32)
    if rv.dim() == 1:
        rv = rv[:, None]
    rv = rv.contiguous()
    idx = idx.to(torch.int64).contiguous().to(rv.device)
    nr, Cc = rv.shape
    if idx.numel() and int(idx.max()) >= nr:
        raise IndexError("asof_gather: index out of range")
    if not rv.is_cuda:
        out = rv[idx.clamp(min=0)].clone() if nr else torch.full((idx.numel(), Cc), float("nan"))
        out[idx < 0] = float("nan")
        return out
    out = torch.empty(idx.numel(), Cc, dtype=torch.float32, device=rv.device)
    _native.call("mfa_asof_gather", _native.ptr(rv), nr, _native.ptr(idx), idx.numel(), Cc,
                 _native.ptr(out), _native.stream(rv.device))
    return out


def asof_join(left_groups, left_keys, right_groups, right_keys, right_values):
    """Search + gather in one call; returns ``(idx, values)``."""
    idx = asof_search(left_groups, left_keys, right_groups, right_keys)
    return idx, asof_gather(right_values, idx)


__all__ = ["asof_search", "asof_gather", "asof_join"]
