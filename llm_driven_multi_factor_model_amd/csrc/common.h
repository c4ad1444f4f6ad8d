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

// MFA_AB = 1 (python -m llm_driven_multi_factor_model_amd._build --ab -> _lib/ab/libmfa_hip.so)
// also instantiates the kernel variants that lost their A/B measurements and the timing-only
// ablations, for the tools/ scripts; the default library holds the production kernels only.
#ifndef MFA_AB
#define MFA_AB 0
#endif

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

// ---- DPP (VALU-only) cross-lane reductions: no LDS traffic, a few cycles per step --------
// gfx9 dpp_ctrl encodings: quad_perm 0x00-0xFF, row_mirror 0x140, row_half_mirror 0x141.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// 64-bit DPP move where lanes without a source (row_shr past the row start, rows masked off by
// ROW_MASK) take `ident` instead.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_upd(double v, double ident) {
  const long long b = __builtin_bit_cast(long long, v), o = __builtin_bit_cast(long long, ident);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, ROW_MASK, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// Inclusive scan over the 64 lanes (lane order), OP: 0 = sum, 1 = max, 2 = min, 3 = product.
// Hillis-Steele
// inside each 16-lane row (row_shr 1, 2, 4, 8), then row_bcast:15 into rows 1 / 3 and
// row_bcast:31 into rows 2 / 3: six VALU-only steps, no LDS round trip.
// 64-bit DPP move, bound_ctrl: lanes whose source is outside the row read 0 (no identity copy)
template <int CTRL>
__device__ __forceinline__ double dpp_zf(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// max / min of finite or infinite (never signalling-NaN) operands: one instruction (fmax / fmin
// first canonicalise an operand that comes out of a DPP move, a second v_max_f64 per step)
__device__ __forceinline__ double vmax64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmin64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Instruction-lean scans (round 4; same results as wave_scan_dpp): the sum's row_shr steps
// zero-fill through bound_ctrl instead of copying the identity into the DPP destination, and
// max / min (idempotent) keep the lane's own value where the source is invalid (old = v, one
// 64-bit copy) and skip the canonicalisation: 4 / 4 instructions per step instead of 5 / 6.
__device__ __forceinline__ double wave_scan_sum(double v) {
  v += dpp_zf<0x111>(v);
  v += dpp_zf<0x112>(v);
  v += dpp_zf<0x114>(v);
  v += dpp_zf<0x118>(v);
  v += dpp_upd<0x142, 0xA>(v, 0.0);
  v += dpp_upd<0x143, 0xC>(v, 0.0);
  return v;
}
template <bool MAX>
__device__ __forceinline__ double wave_scan_ext(double v) {
  auto op = [](double a, double b) { return MAX ? vmax64(a, b) : vmin64(a, b); };
  v = op(v, dpp_upd<0x111, 0xF>(v, v));
  v = op(v, dpp_upd<0x112, 0xF>(v, v));
  v = op(v, dpp_upd<0x114, 0xF>(v, v));
  v = op(v, dpp_upd<0x118, 0xF>(v, v));
  v = op(v, dpp_upd<0x142, 0xA>(v, v));
  v = op(v, dpp_upd<0x143, 0xC>(v, v));
  return v;
}

template <int OP>
__device__ __forceinline__ double wave_scan_dpp(double v) {
  constexpr double id = OP == 0 ? 0.0 : (OP == 1 ? -__builtin_huge_val()
                                                  : (OP == 2 ? __builtin_huge_val() : 1.0));
  auto op = [](double a, double b) {
    return OP == 0 ? a + b : (OP == 1 ? fmax(a, b) : (OP == 2 ? fmin(a, b) : a * b));
  };
  v = op(v, dpp_upd<0x111, 0xF>(v, id));
  v = op(v, dpp_upd<0x112, 0xF>(v, id));
  v = op(v, dpp_upd<0x114, 0xF>(v, id));
  v = op(v, dpp_upd<0x118, 0xF>(v, id));
  v = op(v, dpp_upd<0x142, 0xA>(v, id));
  v = op(v, dpp_upd<0x143, 0xC>(v, id));
  return v;
}

// Sum over each row of 16 lanes; every lane of the row gets the same bits.
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]  (lane ^ 1)
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]  (lane ^ 2)
  v += dpp_mov<0x141>(v);  // row_half_mirror      (quad 0 <-> quad 1)
  v += dpp_mov<0x140>(v);  // row_mirror           (half 0 <-> half 1)
  return v;
}

__device__ __forceinline__ double readlane(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// Wave-uniform (SGPR) total over all 64 lanes, deterministic order.
__device__ __forceinline__ double wave_total(double v) {
  v = row16_sum(v);
  return (readlane(v, 0) + readlane(v, 16)) + (readlane(v, 32) + readlane(v, 48));
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
