// CS-WLS factor-return regression, fp32 panel storage: exported C entry points.
// Kernels and algebra: xs_wls_impl.h (reference: Barra-master/mfm/CrossSection.py:12-108).
#include "xs_wls_impl.h"

MFA_XS_DECLARE_ALL(float)

int g_mfa_xs_mode = 0;
int g_mfa_xs_chunks = 0;
int g_mfa_xs_coop = 0;
int g_mfa_xs_lag = 1;
int g_mfa_xs_pipe_wpc = 0;

// Kernel mode for the next calls (both storage types): 0 = the fused kernel (production).  The
// A/B modes (1 = three separate kernels, 7 = fused without the prefetch, 10-12 MFMA moments,
// 20-24 forced moment sources, 30-38 resident kernel) exist only in MFA_AB builds:
// hipErrorInvalidValue otherwise.
MFA_API int mfa_xs_set_mode(int mode) {
  if (!MFA_AB && mode != 0) return (int)hipErrorInvalidValue;
  g_mfa_xs_mode = mode;
  return 0;
}
unsigned long long* g_mfa_xs_prof = nullptr;
MFA_API void mfa_xs_set_prof(void* p) { g_mfa_xs_prof = (unsigned long long*)p; }

// Stock chunks per date for the next calls: 0 = automatic (default: the fused kernel,
// kXsChunkMinD = 0), > 0 = forced chunk count (A/B builds only: the chunked path measured
// slower at every shard size, profiles/r04/README.md), < 0 = always one workgroup per date.
MFA_API int mfa_xs_set_chunks(int S) {
  if (!MFA_AB && S > 0) return (int)hipErrorInvalidValue;
  g_mfa_xs_chunks = S;
  return 0;
}

// Pipelined team CS-WLS kernel for the next calls (A/B builds only): 0 = off, C > 0 = C chunks
// per date, < 0 = automatic chunk count (xs_coop_chunks).
MFA_API int mfa_xs_set_coop(int C) {
  if (!MFA_AB && C != 0) return (int)hipErrorInvalidValue;
  g_mfa_xs_coop = C;
  return 0;
}
// Pipelined team kernel: residual-pass lag in tickets (1..3) and workgroups per CU (0 = max).
MFA_API int mfa_xs_set_pipe(int lag, int wpc) {
  g_mfa_xs_lag = lag;
  g_mfa_xs_pipe_wpc = wpc;
  return 0;
}
MFA_API int mfa_xs_coop_chunks(int D, int N) { return xs_coop_chunks(D, N); }

// Chunks per date the next mfa_xs_wls / mfa_xs_wls_f64 call on (D, N) will use.
MFA_API int mfa_xs_chunks(int D, int N) { return xs_chunks(D, N); }

// 1 if the bitwise-deterministic kernel (8 wave-owned segment replicas) fits P industries x Q
// styles; larger tables run the shared-replica kernel (reproducible to rounding only).
MFA_API int mfa_xs_det_supported(int P, int Q) {
  const size_t Pseg = P > 0 ? (size_t)P : 1;
  return Pseg * ((size_t)(Q + 3) * kRepMax + kXsSegPad) * sizeof(double) <= (size_t)kSegLdsBudget;
}

// Workspace bytes needed by mfa_xs_wls / mfa_xs_wls_f64 on (D, N, P, Q).
MFA_API size_t mfa_xs_wls_workspace(int D, int N, int P, int Q) {
  return xs_workspace_bytes(D, N, P, Q);
}

// X: [D][Q][N] fp32 styles, cap/ret: [D][N] fp32, ind: [D][N] int16 industry id (<0 = absent;
// may be null when P == 0).  N must be a multiple of 8 (16-byte aligned rows; pad with absent
// stocks).  Outputs: f [D][1+P+Q] fp64 (country, industries, styles), e [D][N] fp32 specific
// returns (nullable), r2 [D] fp64, stats [D][Q+2] fp64 = (mu_q, sigma, n_valid) (nullable),
// status [D] int32 XsStatus bits.  pivot_mode: 0 = last non-empty industry, 1 = reference;
// | 0x100 = bitwise-deterministic kernel (needs the 8-replica segment table: mfa_xs_det_supported,
// P <= 57 at Q = 10).
MFA_API int mfa_xs_wls(const float* X, const float* cap, const float* ret, const int16_t* ind,
                       int D, int N, int P, int Q, int pivot_mode, double tol, double* f,
                       float* e, double* r2, double* stats, int* status, void* ws,
                       void* stream) {
  return xs_wls_dispatch<float>(X, cap, ret, ind, D, N, P, Q, pivot_mode, tol, f, e, r2, stats,
                                status, ws, stream);
}

// Raw moments [D][msize] of this rank's stocks (layout: Layout<Q>, see K1).
MFA_API int mfa_xs_moments(const float* X, const float* cap, const float* ret, const int16_t* ind,
                           int D, int N, int P, int Q, double* mom, void* stream) {
  return split_dispatch<float>(0, X, cap, ret, ind, D, N, P, Q, 0, 0.0, mom, nullptr, nullptr,
                               nullptr, nullptr, nullptr, nullptr, stream);
}

// Constrained solve from (summed) moments: f [D][1+P+Q], coef [D][Q+1+P], stats, status.
MFA_API int mfa_xs_solve(const double* mom, int D, int P, int Q, int pivot_mode, double tol,
                         double* f, double* coef, double* stats, int* status, void* stream) {
  return split_dispatch<float>(1, nullptr, nullptr, nullptr, nullptr, D, 0, P, Q, pivot_mode, tol,
                               (double*)mom, f, coef, stats, status, nullptr, nullptr, stream);
}

// Specific returns of this rank's stocks (e nullable) + per-date R^2 sums [D][5].
MFA_API int mfa_xs_resid_sums(const float* X, const float* cap, const float* ret,
                              const int16_t* ind, int D, int N, int P, int Q, const double* coef,
                              const int* status, float* e, double* sums, void* stream) {
  return split_dispatch<float>(2, X, cap, ret, ind, D, N, P, Q, 0, 0.0, nullptr, nullptr,
                               (double*)coef, nullptr, (int*)status, e, sums, stream);
}

// Device pseudo-inverse of the dates `status` flags near-singular, from their (summed) raw
// moments: rewrites f [D][1+P+Q], coef [D][Q+1+P] and status in place (stock-sharded path,
// after the moments all-reduce and mfa_xs_solve; no host synchronisation).  Any K.
MFA_API int mfa_xs_refine_coef(const double* mom, int D, int P, int Q, int pivot_mode, double* f,
                               double* coef, int* status, void* stream) {
  return split_dispatch<float>(3, nullptr, nullptr, nullptr, nullptr, D, 0, P, Q, pivot_mode, 0.0,
                               (double*)mom, f, coef, nullptr, status, nullptr, nullptr, stream);
}

// Bytes per date of the raw-moment layout (msize doubles).
MFA_API size_t mfa_xs_moments_bytes(int P, int Q) { return xs_moments_bytes(P, Q); }
