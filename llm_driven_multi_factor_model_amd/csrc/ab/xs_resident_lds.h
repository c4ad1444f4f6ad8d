// A/B-only CS-WLS kernels (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build --ab).
// Included by xs_wls_impl.h at the position they held in it; the production library never
// compiles them.  Measured against the production fused kernel in profiles/ (r02-r05).
#pragma once
// Resident fused kernel (xs_resident_kernel): instantiated for the headline fp64 Q = 10 panel;
// mode 30 forces it, mode 31 forces the LDS-DMA fused kernel, mode 0 picks it for
// deterministic fp64 steps past kXsPlainMaxD64 dates.  Returns its dynamic LDS bytes, 0 = not used.
constexpr int kResQ = 10, kResTL = 5, kResTR = 10, kResA = 2;
template <int Q, typename T>
inline size_t xs_resident_lds(int mode, bool det, int D, int N, int P) {
  if (Q != kResQ || sizeof(T) != 8 || !det || P > 128) return 0;
  const bool ab = mode >= 32 && mode <= 38;  // A/B geometries and timing ablations
  if (!(mode == 30 || ab || (mode == 0 && MFA_XS_RESIDENT_DEFAULT && !xs_plain_moments<T>(D))))
    return 0;
  const size_t b = ResGeo<Q, T>::lds_bytes(P > 0 ? P : 1, N, mode == 34 ? 0 : kResTL);
  return b + (Q + 1 + 128) * 8 + 4 * 5 * 8 + 16 <= 160 * 1024 ? b : 0;
}

