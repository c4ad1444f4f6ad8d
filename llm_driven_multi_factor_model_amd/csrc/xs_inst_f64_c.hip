// CS-WLS per-Q instantiations (double panels, Q = 10): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls_f64.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(10, double)

// Timing-only ablation entry (fp64 panel, Q = 10): 0 = full fused kernel, 4 = no residual
// pass, 8 = no solve, 12 = moments only, 13 / 14 / 15 = moments only without the segment
// atomics / the style-Gram FMAs / both (see mfa_xs_wls_variant).
MFA_API int mfa_xs_wls_variant_f64(const double* X, const double* cap, const double* ret,
                                   const int16_t* ind, int D, int N, int P, int variant, double* f,
                                   double* e, double* r2, double* stats, int* status, void* ws,
                                   void* stream) {
  hipStream_t s = (hipStream_t)stream;
  double* w = (double*)ws;
  switch (variant) {
#define MFA_V64(vv)                                                                            \
  case vv:                                                                                     \
    return (int)launch_q<10, vv, double>(X, cap, ret, ind, D, N, P, 0, 1e-14, f, e, r2, stats, \
                                         status, w, s);
    MFA_V64(0) MFA_V64(4) MFA_V64(8) MFA_V64(12) MFA_V64(13) MFA_V64(14) MFA_V64(15)
#undef MFA_V64
    default:
      return (int)hipErrorInvalidValue;
  }
}
