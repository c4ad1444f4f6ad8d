"""ctypes bridge to the in-tree gfx950 kernel library ``_lib/libmfa_hip.so``.

The library is a plain C ABI: every entry point takes raw device pointers, scalar shapes and a
``hipStream_t`` and returns a ``hipError_t``.  Torch supplies memory, streams and collectives;
all math on the GPU path runs in these hand-written kernels.

GPU ops call :func:`lib` which raises loudly when the library is missing or fails to load —
there is no silent eager fallback for tensors that live on the GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch

from ._build import LIB_PATH

_lock = threading.Lock()
_lib: C.CDLL | None = None

_vp, _i, _d, _f = C.c_void_p, C.c_int, C.c_double, C.c_float

# name -> argtypes (all return int hipError_t)
_SIGS: dict[str, list] = {
    # xs_wls.hip
    "mfa_xs_wls": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "mfa_xs_wls_f64": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "mfa_xs_wls_workspace": [_i, _i, _i, _i],
    "mfa_xs_chunks": [_i, _i],
    "mfa_xs_set_chunks": [_i],
    "mfa_xs_set_mode": [_i],
    "mfa_xs_set_coop": [_i],
    "mfa_ab_build": [],
    "mfa_gather_host_ranges": [_vp, _vp, _vp, _i, _vp, _vp, C.c_int64, _vp],
    "mfa_xs_set_pipe": [_i, _i],
    "mfa_xs_coop_chunks": [_i, _i],
    "mfa_xs_det_supported": [_i, _i],
    "mfa_xs_wls_variant": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
}


class NativeError(RuntimeError):
    pass


def register(name: str, argtypes: list) -> None:
    """Declare a C entry point signature (used by op modules at import time)."""
    _SIGS[name] = argtypes
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.argtypes = argtypes
        fn.restype = C.c_size_t if name.endswith(("_workspace", "_bytes", "_doubles")) else C.c_int


def _load() -> C.CDLL:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = Path(os.environ.get("MFA_HIP_LIB", LIB_PATH))
        if not path.exists():
            if os.environ.get("MFA_NO_AUTOBUILD"):
                raise NativeError(f"HIP kernel library missing: {path} (run python -m "
                                  "llm_driven_multi_factor_model_amd._build)")
            from ._build import build
            build()
        lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
        for name, argt in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = argt
            fn.restype = C.c_size_t if name.endswith(("_workspace", "_bytes", "_doubles")) else C.c_int
        _lib = lib
        return lib


def lib() -> C.CDLL:
    return _lib if _lib is not None else _load()


def loaded_path() -> str | None:
    return os.environ.get("MFA_HIP_LIB", str(LIB_PATH)) if _lib is not None else None


def ab_build() -> bool:
    """True when the loaded library is the A/B build (MFA_AB=1: the losing kernel variants and
    the timing ablations are compiled in; ``_build --ab``)."""
    return bool(lib().mfa_ab_build())


def ptr(t: torch.Tensor | None) -> C.c_void_p:
    if t is None:
        return C.c_void_p(0)
    return C.c_void_p(t.data_ptr())


def stream(device: torch.device | None = None) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def query(name: str, *args) -> int:
    """Call a size-returning entry point (``*_workspace`` / ``*_bytes``)."""
    return int(getattr(lib(), name)(*args))


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise NativeError(f"{name} failed with hipError_t {rc}")


def check_device_tensor(t: torch.Tensor, dtype: torch.dtype, name: str) -> torch.Tensor:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        t = t.contiguous()
    return t
