// CS-WLS factor-return regression, fp64 panel storage: exported C entry points.
//
// The reference reads float64 exposures / capital / returns (Barra-master/demo.py:21-35) and
// regresses them in float64 (mfm/CrossSection.py:57-108).  Same kernels as the fp32 path
// (xs_wls_impl.h) instantiated for double rows: 16-byte LDS-DMA moves two 512-B fp64 rows per
// wave instruction into a 2-slot per-wave ring, the residual pass reads 2 stocks per 16-byte
// load and stores fp64 specific returns.  Moments / solve are fp64 either way.
#include "xs_wls_impl.h"

MFA_XS_DECLARE_ALL(double)

// Same contract as mfa_xs_wls with fp64 X / cap / ret and fp64 specific returns e.
MFA_API int mfa_xs_wls_f64(const double* X, const double* cap, const double* ret,
                           const int16_t* ind, int D, int N, int P, int Q, int pivot_mode,
                           double tol, double* f, double* e, double* r2, double* stats,
                           int* status, void* ws, void* stream) {
  return xs_wls_dispatch<double>(X, cap, ret, ind, D, N, P, Q, pivot_mode, tol, f, e, r2, stats,
                                 status, ws, stream);
}

MFA_API int mfa_xs_moments_f64(const double* X, const double* cap, const double* ret,
                               const int16_t* ind, int D, int N, int P, int Q, double* mom,
                               void* stream) {
  return split_dispatch<double>(0, X, cap, ret, ind, D, N, P, Q, 0, 0.0, mom, nullptr, nullptr,
                                nullptr, nullptr, nullptr, nullptr, stream);
}

MFA_API int mfa_xs_resid_sums_f64(const double* X, const double* cap, const double* ret,
                                  const int16_t* ind, int D, int N, int P, int Q,
                                  const double* coef, const int* status, double* e, double* sums,
                                  void* stream) {
  return split_dispatch<double>(2, X, cap, ret, ind, D, N, P, Q, 0, 0.0, nullptr, nullptr,
                                (double*)coef, nullptr, (int*)status, e, sums, stream);
}
