// CS-WLS per-Q instantiations (float panels, Q = 10): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(10, float)

// Timing-only ablation entry (fp32, Q = 10): bit 1 = no segment atomics, bit 2 = no style-Gram
// FMAs, bit 4 = no residual pass, bit 8 = no solve (fused mode only), 16 = second residual pass.
MFA_API int mfa_xs_wls_variant(const float* X, const float* cap, const float* ret,
                               const int16_t* ind, int D, int N, int P, int variant, double* f,
                               float* e, double* r2, double* stats, int* status, void* ws,
                               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  double* w = (double*)ws;
  switch (variant) {
#define MFA_V(vv)                                                                              \
  case vv:                                                                                     \
    return (int)launch_q<10, vv, float>(X, cap, ret, ind, D, N, P, 0, 1e-14, f, e, r2, stats, \
                                        status, w, s);
    MFA_V(0) MFA_V(1) MFA_V(2) MFA_V(3) MFA_V(4) MFA_V(5) MFA_V(6) MFA_V(7) MFA_V(8)
    MFA_V(12) MFA_V(13) MFA_V(14) MFA_V(15) MFA_V(16) MFA_V(20)
#undef MFA_V
  }
  return (int)hipErrorInvalidValue;
}
