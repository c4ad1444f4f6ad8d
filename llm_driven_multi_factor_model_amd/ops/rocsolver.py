"""Batched symmetric eigensolvers of rocSOLVER for factor sets wider than one wave (K > 64).

The register-resident one-wave kernels of ``csrc/eigen.hip`` cover K <= 64 (every BASELINE
configuration: K = 42).  Wider factor sets (e.g. SW-L2 industries, K = 140) go to rocSOLVER's
STRIDED-BATCHED drivers, which solve the whole batch in a few launches instead of one library
call per matrix: ``syevd`` (tridiagonal divide and conquer) or ``syevj`` (Jacobi).  Called
through ctypes on the caller's HIP stream with one rocBLAS handle per device; eigenvalues come
back ascending, eigenvectors in the columns of the (column-major) matrix, i.e. ROW k of the
row-major [K, K] buffer is eigenvector k.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from .. import _native

_LIBS = None
_HANDLES: dict = {}
EVECT_ORIGINAL, FILL_UPPER, ESORT_ASC = 211, 121, 252


def _libs():
    global _LIBS
    if _LIBS is None:
        root = os.environ.get("ROCM_PATH", "/opt/rocm")
        rb = C.CDLL(os.path.join(root, "lib", "librocblas.so"))
        rs = C.CDLL(os.path.join(root, "lib", "librocsolver.so"))
        rb.rocblas_create_handle.argtypes = [C.POINTER(C.c_void_p)]
        rb.rocblas_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        rs.rocsolver_dsyevd_strided_batched.argtypes = [
            C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
            C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_int]
        rs.rocsolver_dsyevj_strided_batched.argtypes = [
            C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int64,
            C.c_double, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int]
        _LIBS = (rb, rs)
    return _LIBS


def _handle(dev: torch.device):
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    h = _HANDLES.get(idx)
    if h is None:
        rb, _ = _libs()
        with torch.cuda.device(idx):
            h = C.c_void_p()
            st = rb.rocblas_create_handle(C.byref(h))
            if st != 0:
                raise RuntimeError(f"rocblas_create_handle failed ({st})")
        _HANDLES[idx] = h
    return h


def syev_batched(A: torch.Tensor, method: str = "syevd"):
    """Eigen-decompose a batch of symmetric fp64 matrices [B, K, K] on the GPU.

    Returns ``(w [B, K] ascending, V [B, K, K])`` with ``V[b, :, k]`` the k-th eigenvector, and
    ``info`` [B] (0 = converged).  ``A`` is not modified."""
    if not A.is_cuda or A.dtype != torch.float64:
        raise TypeError("syev_batched needs a float64 GPU tensor")
    B, K, _ = A.shape
    dev = A.device
    rb, rs = _libs()
    h = _handle(dev)
    rb.rocblas_set_stream(h, _native.stream(dev))
    V = A.contiguous().clone()
    w = torch.empty(B, K, dtype=torch.float64, device=dev)
    info = torch.empty(B, dtype=torch.int32, device=dev)
    if B == 0:
        return w, V, info
    if method == "syevj":
        res = torch.empty(B, dtype=torch.float64, device=dev)
        sweeps = torch.empty(B, dtype=torch.int32, device=dev)
        st = rs.rocsolver_dsyevj_strided_batched(
            h, ESORT_ASC, EVECT_ORIGINAL, FILL_UPPER, K, _native.ptr(V), K, K * K, 0.0,
            _native.ptr(res), 100, _native.ptr(sweeps), _native.ptr(w), K, _native.ptr(info), B)
    else:
        E = torch.empty(B, K, dtype=torch.float64, device=dev)
        st = rs.rocsolver_dsyevd_strided_batched(
            h, EVECT_ORIGINAL, FILL_UPPER, K, _native.ptr(V), K, K * K, _native.ptr(w), K,
            _native.ptr(E), K, _native.ptr(info), B)
    if st != 0:
        raise RuntimeError(f"rocsolver {method} failed with status {st}")
    # column-major output: row k of the row-major buffer is eigenvector k
    return w, V.transpose(-1, -2), info
