// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of the Barra risk engine.
//
// Conventions used by every kernel in csrc/:
//   * wave = 64 lanes (hard-coded, never warpSize-derived);
//   * panel tensors are fp32 in HBM, small-matrix algebra and all reductions are fp64;
//   * every exported entry point is `extern "C"`, takes raw device pointers plus a
//     hipStream_t and returns a hipError_t (0 = success) so the Python side can raise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define MFA_API extern "C" __attribute__((visibility("default")))

namespace mfa {

constexpr int kWave = 64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off, kWave));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (16 waves). `scratch` needs 16 doubles of LDS.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

__device__ __forceinline__ double qnan() { return __builtin_nan(""); }
__device__ __forceinline__ float qnanf() { return __builtin_nanf(""); }

}  // namespace mfa

#define MFA_RETURN_LAST_ERROR() return hipGetLastError()
