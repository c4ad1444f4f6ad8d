// Gram matrices of 64-row blocks on the fp64 matrix cores, shared by the wide draw covariances
// (csrc/eigen.hip, mc_cov_wide_kernel) and the wide eigh orthogonality check
// (csrc/eigen_wide.hip, eigh_wide_fix_kernel).  Rows staged in LDS as Z[64][KP + 2]; the
// KT (KT + 1) / 2 upper 16 x 16 tiles (KT = KP / 16) of Z^T Z are dealt round-robin to the 4
// waves of a 256-thread workgroup, each tile one v_mfma_f64_16x16x4f64 chain.  16x16x4 f64
// layouts (tools/probes/mfma64_probe.hip): A operand lane l = A[l & 15][l >> 4], B operand
// lane l = B[l >> 4][l & 15], register e of lane l = D[(l >> 4) + 4 e][l & 15].
#pragma once
#include <utility>

#include "common.h"

namespace mfa {

typedef double f64x4g __attribute__((ext_vector_type(4)));

template <int KP>
struct WideCov {
  static constexpr int KT = KP / 16;
  static constexpr int NT = KT * (KT + 1) / 2;
  static constexpr int NW = 4;
  static constexpr int TPW = (NT + NW - 1) / NW;              // tiles per wave
  static constexpr int PART = NT * 4 * 64 + KP;               // doubles per (sim, chunk)
  static constexpr int ti(int t) {                            // tile t -> (row, col), row <= col
    int r = 0;
    while (t >= KT - r) { t -= KT - r; ++r; }
    return r;
  }
  static constexpr int tj(int t) {
    int r = 0;
    while (t >= KT - r) { t -= KT - r; ++r; }
    return r + t;
  }
};

// wave W's tiles W, W + 4, ... of one k-step (tile coordinates compile-time: the fragments
// a[] stay in registers)
template <int KP, int W, int... U>
__device__ __forceinline__ void wide_cov_step(const double* a, f64x4g* acc,
                                              std::integer_sequence<int, U...>) {
  using G = WideCov<KP>;
  ([&] {
    constexpr int t = W + G::NW * U;
    if constexpr (t < G::NT)
      acc[U] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[G::ti(t)], a[G::tj(t)], acc[U], 0, 0, 0);
  }(), ...);
}

// Accumulate Z[0..63][:]^T Z[0..63][:] into wave wv's tiles (call between the barriers that
// bracket the staging of Z).
template <int KP>
__device__ __forceinline__ void wide_gram_block(const double (*Z)[KP + 2], int wv, int lane,
                                                f64x4g* acc) {
  using G = WideCov<KP>;
  const int r16 = lane & 15, k4 = lane >> 4;
#pragma unroll 2
  for (int k = 0; k < 64; k += 4) {
    double a[G::KT];
#pragma unroll
    for (int i = 0; i < G::KT; ++i) a[i] = Z[k + k4][16 * i + r16];
    constexpr auto us = std::make_integer_sequence<int, G::TPW>{};
    switch (wv) {  // uniform per wave
      case 0: wide_cov_step<KP, 0>(a, acc, us); break;
      case 1: wide_cov_step<KP, 1>(a, acc, us); break;
      case 2: wide_cov_step<KP, 2>(a, acc, us); break;
      default: wide_cov_step<KP, 3>(a, acc, us); break;
    }
  }
}

}  // namespace mfa
