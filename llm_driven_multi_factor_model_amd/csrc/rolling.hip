// Rolling-window time-series descriptors (K4, K5) for gfx950.
//
// Reference: Barra_factor_cal/factor_calculator.py
//   BETA/HSIGMA  :79-125   per stock, rolling 252 rows, min 42 valid, dropna, WLS ret ~ 1 + mret
//                          with weights (0.5^(1/63))^(251..0)[-n:] (newest valid row weight 1)
//   RSTR         :127-153  log_ret.shift(21), rolling 483 rows (partial windows allowed),
//                          min 42 valid, positional weights (0.5^(1/126))^p, p = 0 for the OLDEST
//                          row of the window (quirk Q14), NaN-renormalised weighted mean
//   DASTD        :155-196  excess = ret - mret, rolling 252, min 42, newest-first compressed
//                          weights (0.5^(1/42))^k, weighted population std
//   CMRA         :199-234  rolling 252 of log_ret, full window only (no NaN); ln(1+max Z) -
//                          ln(1+min Z), Z = exp(cumsum) - 1.  factor.py:195-226 variant: partial
//                          windows and NaN-skipping cumsum (quirk Q15)
//   STOM/Q/A     :324-367  ln(rolling sum of turnover/100 over 21/63/252 rows, min 15/42/126)
//
// Layout: the reference's master frame sorted by (ts_code, trade_date) is kept as FLAT rows;
// `seg_lo[r]` is the first row of row r's stock, so windows count the stock's own rows (not
// calendar days) exactly as pandas groupby-rolling does.  One thread per output row; taps are
// read newest-to-oldest; neighbouring lanes read neighbouring rows, so every tap is a coalesced
// 256-byte wave load that mostly hits L1/L2.  fp64 accumulation throughout.
#include "common.h"

namespace {

using namespace mfa;

__device__ __forceinline__ bool fin(float v) { return __builtin_isfinite(v); }

__global__ __launch_bounds__(256) void beta_hsigma_kernel(const float* __restrict__ y,
                                                          const float* __restrict__ x,
                                                          const int* __restrict__ seg_lo, int R,
                                                          int W, double lam, int minp,
                                                          float* __restrict__ beta,
                                                          float* __restrict__ hsig) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int lo = max(seg_lo[r], r - W + 1);
  double w = 1.0, Sw = 0, Sx = 0, Sy = 0, Sxx = 0, Sxy = 0;
  int n = 0;
  for (int j = r; j >= lo; --j) {
    const float yv = y[j], xv = x[j];
    if (!(fin(yv) && fin(xv))) continue;
    const double xd = xv, yd = yv;
    Sw += w;
    Sx = fma(w, xd, Sx);
    Sy = fma(w, yd, Sy);
    Sxx = fma(w * xd, xd, Sxx);
    Sxy = fma(w * xd, yd, Sxy);
    w *= lam;
    ++n;
  }
  float b = qnanf(), h = qnanf();
  if (n >= minp && n > 2) {
    const double mx = Sx / Sw, my = Sy / Sw;
    const double vxx = Sxx / Sw - mx * mx;
    const double cxy = Sxy / Sw - mx * my;
    const double bb = cxy / vxx;
    const double aa = my - bb * mx;
    // residual sum of squares: second pass (exact, no cancellation)
    double ssr = 0.0, ww = 1.0;
    for (int j = r; j >= lo; --j) {
      const float yv = y[j], xv = x[j];
      if (!(fin(yv) && fin(xv))) continue;
      const double e = (double)yv - aa - bb * (double)xv;
      ssr = fma(ww * e, e, ssr);
      ww *= lam;
    }
    b = (float)bb;
    h = (float)sqrt(ssr / (double)(n - 2));
  }
  beta[r] = b;
  hsig[r] = h;
}

__global__ __launch_bounds__(256) void rstr_kernel(const float* __restrict__ lr,
                                                   const int* __restrict__ seg_lo, int R, int L,
                                                   int W, double lam, int minp,
                                                   float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int s0 = seg_lo[r];
  const int lo = max(s0, r - W + 1);
  // positional weight lam^(j - lo): oldest row of the (possibly partial) window gets 1
  double num = 0.0, den = 0.0, wj = 1.0;
  int n = 0;
  for (int j = lo; j <= r; ++j) {
    const int src = j - L;
    const float v = src >= s0 ? lr[src] : qnanf();
    if (fin(v)) {
      num = fma(wj, (double)v, num);
      den += wj;
      ++n;
    }
    wj *= lam;
  }
  out[r] = (n >= minp) ? (float)(num / den) : qnanf();
}

__global__ __launch_bounds__(256) void dastd_kernel(const float* __restrict__ ret,
                                                    const float* __restrict__ mret,
                                                    const int* __restrict__ seg_lo, int R, int W,
                                                    double lam, int minp,
                                                    float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int lo = max(seg_lo[r], r - W + 1);
  double w = 1.0, Sw = 0.0, Sx = 0.0;
  int n = 0;
  for (int j = r; j >= lo; --j) {
    const float a = ret[j], b = mret[j];
    if (!(fin(a) && fin(b))) continue;
    const double e = (double)a - (double)b;
    Sw += w;
    Sx = fma(w, e, Sx);
    w *= lam;
    ++n;
  }
  float o = qnanf();
  if (n >= minp) {
    const double m = Sx / Sw;
    double v = 0.0, ww = 1.0;
    for (int j = r; j >= lo; --j) {
      const float a = ret[j], b = mret[j];
      if (!(fin(a) && fin(b))) continue;
      const double e = (double)a - (double)b - m;
      v = fma(ww * e, e, v);
      ww *= lam;
    }
    o = (float)sqrt(v / Sw);
  }
  out[r] = o;
}

__global__ __launch_bounds__(256) void cmra_kernel(const float* __restrict__ lr,
                                                   const int* __restrict__ seg_lo, int R, int W,
                                                   int partial, float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int s0 = seg_lo[r];
  float o = qnanf();
  if (!partial) {
    if (r - W + 1 >= s0) {
      double c = 0.0, zmax = -1e300, zmin = 1e300;
      bool ok = true;
      for (int j = r - W + 1; j <= r; ++j) {
        const float v = lr[j];
        if (!fin(v)) { ok = false; break; }
        c += (double)v;
        const double z = exp(c) - 1.0;
        zmax = fmax(zmax, z);
        zmin = fmin(zmin, z);
      }
      if (ok) o = (float)(log(1.0 + zmax) - log(1.0 + zmin));
    }
  } else {  // factor.py: partial windows, pandas cumsum skips NaN, max/min skip NaN
    const int lo = max(s0, r - W + 1);
    double c = 0.0, zmax = -1e300, zmin = 1e300;
    int n = 0;
    for (int j = lo; j <= r; ++j) {
      const float v = lr[j];
      if (!fin(v)) continue;
      c += (double)v;
      const double z = exp(c) - 1.0;
      zmax = fmax(zmax, z);
      zmin = fmin(zmin, z);
      ++n;
    }
    if (n > 0) o = (float)(log(1.0 + zmax) - log(1.0 + zmin));
  }
  out[r] = o;
}

// rolling NaN-skipping sum with min valid count; mode 1 = ln(sum) with sum == 0 -> NaN
__global__ __launch_bounds__(256) void rolling_sum_kernel(const float* __restrict__ x,
                                                          const int* __restrict__ seg_lo, int R,
                                                          int W, int minp, double scale, int mode,
                                                          float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int lo = max(seg_lo[r], r - W + 1);
  double s = 0.0;
  int n = 0;
  for (int j = r; j >= lo; --j) {
    const float v = x[j];
    if (fin(v)) { s += (double)v * scale; ++n; }
  }
  float o = qnanf();
  if (n >= minp) {
    if (mode == 1) o = (s == 0.0) ? qnanf() : (float)log(s);
    else o = (float)s;
  }
  out[r] = o;
}

// per-stock returns on flat rows: ret = pct_change (pandas pads NaN closes), log_ret = diff(log)
__global__ __launch_bounds__(256) void returns_kernel(const float* __restrict__ close,
                                                      const int* __restrict__ seg_lo, int R,
                                                      float* __restrict__ ret,
                                                      float* __restrict__ logret) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int s0 = seg_lo[r];
  const float c = close[r];
  float lrv = qnanf(), rv = qnanf();
  if (r > s0) {
    const float p = close[r - 1];
    if (fin(c) && fin(p) && c > 0.f && p > 0.f) lrv = (float)(log((double)c) - log((double)p));
    // pct_change(fill_method='pad'): forward-fill both this and the previous value
    int i = r;
    while (i >= s0 && !fin(close[i])) --i;
    int k = r - 1;
    while (k >= s0 && !fin(close[k])) --k;
    if (i >= s0 && k >= s0) rv = (float)((double)close[i] / (double)close[k] - 1.0);
  }
  ret[r] = rv;
  logret[r] = lrv;
}

}  // namespace

#define MFA_GRID(R) dim3(((R) + 255) / 256), dim3(256)

MFA_API int mfa_beta_hsigma(const float* y, const float* x, const int* seg_lo, int R, int W,
                            double lam, int minp, float* beta, float* hsig, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(beta_hsigma_kernel, MFA_GRID(R), 0, (hipStream_t)s, y, x, seg_lo, R, W, lam,
                     minp, beta, hsig);
  return (int)hipGetLastError();
}
MFA_API int mfa_rstr(const float* lr, const int* seg_lo, int R, int L, int W, double lam,
                     int minp, float* out, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(rstr_kernel, MFA_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, L, W, lam, minp, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_dastd(const float* ret, const float* mret, const int* seg_lo, int R, int W,
                      double lam, int minp, float* out, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(dastd_kernel, MFA_GRID(R), 0, (hipStream_t)s, ret, mret, seg_lo, R, W, lam,
                     minp, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_cmra(const float* lr, const int* seg_lo, int R, int W, int partial, float* out,
                     void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(cmra_kernel, MFA_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, W, partial, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_rolling_sum(const float* x, const int* seg_lo, int R, int W, int minp,
                            double scale, int mode, float* out, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(rolling_sum_kernel, MFA_GRID(R), 0, (hipStream_t)s, x, seg_lo, R, W, minp,
                     scale, mode, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_returns(const float* close, const int* seg_lo, int R, float* ret, float* logret,
                        void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(returns_kernel, MFA_GRID(R), 0, (hipStream_t)s, close, seg_lo, R, ret, logret);
  return (int)hipGetLastError();
}
