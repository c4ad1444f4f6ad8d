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

// The direct per-row kernels below (the reference kernels of the tests and the rank-invariant
// path) stage the rows their 256-row block's windows read through LDS: the block loads its span
// (255 + W rows, plus the lag) once, coalesced, and every row then sums its own window from LDS
// in the same fixed order as the global-memory form -- bitwise the same outputs, W fewer L1 tap
// loads per row.  Spans over kDirSpan rows read global memory as before.
constexpr int kDirSpan = 1024;
__device__ __forceinline__ void dir_stage(const float* __restrict__ x, int R, int base, int n,
                                          float* sx) {
  for (int k = threadIdx.x; k < n; k += 256) {
    const int g = base + k;
    sx[k] = (g >= 0 && g < R) ? x[g] : __builtin_nanf("");
  }
}

__global__ __launch_bounds__(256) void beta_hsigma_kernel(const float* __restrict__ y,
                                                          const float* __restrict__ x,
                                                          const int* __restrict__ seg_lo, int R,
                                                          int W, double lam, int minp,
                                                          float* __restrict__ beta,
                                                          float* __restrict__ hsig) {
  __shared__ float sy[kDirSpan], sx[kDirSpan];
  const int r0 = blockIdx.x * 256, base = r0 - W + 1, span = 255 + W;
  const bool st = span <= kDirSpan;
  if (st) {
    dir_stage(y, R, base, span, sy);
    dir_stage(x, R, base, span, sx);
  }
  __syncthreads();
  const int r = r0 + threadIdx.x;
  if (r >= R) return;
  auto Y = [&](int j) { return st ? sy[j - base] : y[j]; };
  auto X = [&](int j) { return st ? sx[j - base] : x[j]; };
  const int lo = max(seg_lo[r], r - W + 1);
  double w = 1.0, Sw = 0, Sx = 0, Sy = 0, Sxx = 0, Sxy = 0;
  int n = 0;
  for (int j = r; j >= lo; --j) {
    const float yv = Y(j), xv = X(j);
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
      const float yv = Y(j), xv = X(j);
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

// lam^k by binary powering (k < 512): no libm pow per table entry
__device__ __forceinline__ double ipow(double lam, int k) {
  double r = 1.0, b = lam;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    if (k & (1 << i)) r *= b;
    b *= b;
  }
  return r;
}

// Direct per-row RSTR (the reference kernel of the tests and the rank-invariant path): the
// positional weights lam^k come from an LDS table (no dependent weight-update chain) and the
// window sums alternate between two accumulators (half the dependent fma chain); every row's
// window is still summed in one fixed order, independent of the launch it belongs to.
constexpr int kRsDirectTab = 512;
__global__ __launch_bounds__(256) void rstr_kernel(const float* __restrict__ lr,
                                                   const int* __restrict__ seg_lo, int R, int L,
                                                   int W, double lam, int minp,
                                                   float* __restrict__ out) {
  __shared__ double pw[kRsDirectTab];
  __shared__ float sl[kDirSpan];
  const bool tab = W <= kRsDirectTab;
  if (tab)
    for (int k = threadIdx.x; k < W; k += blockDim.x) pw[k] = ipow(lam, k);
  const int r0 = blockIdx.x * 256, base = r0 - W + 1 - L, span = 255 + W;
  const bool st = span <= kDirSpan;
  if (st) dir_stage(lr, R, base, span, sl);
  __syncthreads();
  const int r = r0 + threadIdx.x;
  if (r >= R) return;
  const int s0 = seg_lo[r];
  const int lo = max(s0, r - W + 1);
  // positional weight lam^(j - lo): oldest row of the (possibly partial) window gets 1
  double num[2] = {0.0, 0.0}, den[2] = {0.0, 0.0}, wj = 1.0;
  int n = 0;
  int j = lo;
  if (st && tab) {
    // 8 taps per step: their LDS loads issue together ahead of the (same-order) fma chain
    for (; j + 8 <= r + 1; j += 8) {
      float v[8];
      double wk[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int src = j + u - L;
        v[u] = src >= s0 ? sl[src - base] : qnanf();
        wk[u] = pw[j + u - lo];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)  // j - lo is even here: tap u feeds accumulator u & 1
        if (fin(v[u])) {
          num[u & 1] = fma(wk[u], (double)v[u], num[u & 1]);
          den[u & 1] += wk[u];
          ++n;
        }
    }
  }
  for (; j <= r; ++j) {
    const int src = j - L, k = j - lo;
    const float v = src >= s0 ? (st ? sl[src - base] : lr[src]) : qnanf();
    const double wk = tab ? pw[k] : wj;
    if (fin(v)) {
      num[k & 1] = fma(wk, (double)v, num[k & 1]);
      den[k & 1] += wk;
      ++n;
    }
    if (!tab) wj *= lam;
  }
  out[r] = (n >= minp) ? (float)((num[0] + num[1]) / (den[0] + den[1])) : qnanf();
}

__global__ __launch_bounds__(256) void dastd_kernel(const float* __restrict__ ret,
                                                    const float* __restrict__ mret,
                                                    const int* __restrict__ seg_lo, int R, int W,
                                                    double lam, int minp,
                                                    float* __restrict__ out) {
  __shared__ float sa[kDirSpan], sb[kDirSpan];
  const int r0 = blockIdx.x * 256, base = r0 - W + 1, span = 255 + W;
  const bool st = span <= kDirSpan;
  if (st) {
    dir_stage(ret, R, base, span, sa);
    dir_stage(mret, R, base, span, sb);
  }
  __syncthreads();
  const int r = r0 + threadIdx.x;
  if (r >= R) return;
  const int lo = max(seg_lo[r], r - W + 1);
  double w = 1.0, Sw = 0.0, Sx = 0.0;
  int n = 0;
  for (int j = r; j >= lo; --j) {
    const float a = st ? sa[j - base] : ret[j], b = st ? sb[j - base] : mret[j];
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
      const float a = st ? sa[j - base] : ret[j], b = st ? sb[j - base] : mret[j];
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
  __shared__ float sl[kDirSpan];
  const int r0 = blockIdx.x * 256, base = r0 - W + 1, span = 255 + W;
  const bool st = span <= kDirSpan;
  if (st) dir_stage(lr, R, base, span, sl);
  __syncthreads();
  const int r = r0 + threadIdx.x;
  if (r >= R) return;
  const int s0 = seg_lo[r];
  float o = qnanf();
  // Z = exp(c) - 1 is non-decreasing in the running sum c, so max Z = exp(max c) - 1 (and min
  // likewise): two exp / log pairs per row instead of one exp per tap
  if (!partial) {
    if (r - W + 1 >= s0) {
      double c = 0.0, cmax = -INFINITY, cmin = INFINITY;
      bool ok = true;
      int j = r - W + 1;
      if (st) {
        for (; j + 8 <= r + 1; j += 8) {  // 8 taps' LDS loads together, the same order
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = sl[j + u - base];
          bool okb = true;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            okb = okb && fin(v[u]);
            c += (double)v[u];
            cmax = fmax(cmax, c);
            cmin = fmin(cmin, c);
          }
          if (!okb) { ok = false; break; }
        }
      }
      for (; ok && j <= r; ++j) {
        const float v = st ? sl[j - base] : lr[j];
        if (!fin(v)) { ok = false; break; }
        c += (double)v;
        cmax = fmax(cmax, c);
        cmin = fmin(cmin, c);
      }
      if (ok) o = (float)(log(1.0 + (exp(cmax) - 1.0)) - log(1.0 + (exp(cmin) - 1.0)));
    }
  } else {  // factor.py: partial windows, pandas cumsum skips NaN, max/min skip NaN
    const int lo = max(s0, r - W + 1);
    double c = 0.0, cmax = -INFINITY, cmin = INFINITY;
    int n = 0;
    for (int j = lo; j <= r; ++j) {
      const float v = st ? sl[j - base] : lr[j];
      if (!fin(v)) continue;
      c += (double)v;
      cmax = fmax(cmax, c);
      cmin = fmin(cmin, c);
      ++n;
    }
    if (n > 0) o = (float)(log(1.0 + (exp(cmax) - 1.0)) - log(1.0 + (exp(cmin) - 1.0)));
  }
  out[r] = o;
}

// rolling NaN-skipping sum with min valid count; mode 1 = ln(sum) with sum == 0 -> NaN
__global__ __launch_bounds__(256) void rolling_sum_kernel(const float* __restrict__ x,
                                                          const int* __restrict__ seg_lo, int R,
                                                          int W, int minp, double scale, int mode,
                                                          float* __restrict__ out) {
  __shared__ float sx[kDirSpan];
  const int r0 = blockIdx.x * 256, base = r0 - W + 1, span = 255 + W;
  const bool st = span <= kDirSpan;
  if (st) dir_stage(x, R, base, span, sx);
  __syncthreads();
  const int r = r0 + threadIdx.x;
  if (r >= R) return;
  const int lo = max(seg_lo[r], r - W + 1);
  double s = 0.0;
  int n = 0;
  int j = r;
  if (st) {
    for (; j - 8 >= lo - 1; j -= 8) {  // 8 taps' LDS loads together, the same summation order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = sx[j - u - base];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (fin(v[u])) { s += (double)v[u] * scale; ++n; }
    }
  }
  for (; j >= lo; --j) {
    const float v = st ? sx[j - base] : x[j];
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

// ------------------------------------------------------------------------------------------
// Sliding-window (O(1) per row) versions.  A 256-thread block owns kBlockRows consecutive flat
// rows; it stages them plus an H-row halo (H >= the window reach) from HBM into LDS with
// coalesced loads, then every thread walks its own kChunk consecutive rows out of LDS (padded
// layout: one spare word per 16 rows, so the 16-row lane stride hits distinct banks):
//   * the thread's first row gets its window state from one direct pass (<= W taps);
//   * compressed weights (BETA/HSIGMA, DASTD): the newest VALID row has weight 1, older valid
//     rows lam^k (k = valid rows newer than it).  A valid row entering scales all old terms by
//     lam; the row leaving (r - W) has weight lam^(n - 1), so S <- lam S + v_r - lam^(n-1) v_q
//     (errors are damped by lam every step);
//   * positional weights (RSTR): lam^(j - b) with a chunk-fixed base b -- the reference's
//     normalisation by sum(w) cancels the common factor lam^(lo - b).
// Work per output: ~W / kChunk direct taps + O(1), all from LDS; HBM sees each row ~once.
// ------------------------------------------------------------------------------------------
constexpr int kChunk = 16;
constexpr int kBlockRows = 256 * kChunk;
constexpr int kPowMax = 768;   // lam^k table (LDS), k < kPowMax

__device__ __forceinline__ int lds_idx(int p) { return p + (p >> 4); }
__host__ __device__ constexpr int lds_len(int rows) { return rows + (rows >> 4) + 1; }

// Stage rows [g0, g0 + n) of `src` (NaN outside [0, R)) into padded LDS.
__device__ __forceinline__ void stage_f(float* dst, const float* __restrict__ src, int g0, int n,
                                        int R) {
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const int g = g0 + p;
    dst[lds_idx(p)] = (g >= 0 && g < R) ? src[g] : qnanf();
  }
}
__device__ __forceinline__ void stage_i(int* dst, const int* __restrict__ src, int g0, int n,
                                        int R) {
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const int g = g0 + p;
    dst[lds_idx(p)] = (g >= 0 && g < R) ? src[g] : g;
  }
}

__device__ __forceinline__ void fill_pow(double* pw, double lam, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) pw[k] = pow(lam, (double)k);
}

template <int H>
struct Stage2 {  // two float series + seg_lo
  float a[lds_len(H + kBlockRows)], b[lds_len(H + kBlockRows)];
  int seg[lds_len(H + kBlockRows)];
  double pw[kPowMax];
};

template <int H>
__global__ __launch_bounds__(256) void beta_hsigma_scan_kernel(
    const float* __restrict__ y, const float* __restrict__ x, const int* __restrict__ seg_lo,
    int R, int W, double lam, int minp, float* __restrict__ beta, float* __restrict__ hsig) {
  __shared__ Stage2<H> sh;
  const int b0 = blockIdx.x * kBlockRows, g0 = b0 - H;
  const int n = min(H + kBlockRows, R - g0);
  stage_f(sh.a, y, g0, n, R);
  stage_f(sh.b, x, g0, n, R);
  stage_i(sh.seg, seg_lo, g0, n, R);
  fill_pow(sh.pw, lam, W + 1);
  __syncthreads();
  const int r0 = b0 + threadIdx.x * kChunk;
  if (r0 >= R) return;
  const int r1 = min(r0 + kChunk, R);
  auto Y = [&](int r) { return sh.a[lds_idx(r - g0)]; };
  auto X = [&](int r) { return sh.b[lds_idx(r - g0)]; };
  auto S0 = [&](int r) { return sh.seg[lds_idx(r - g0)]; };
  double Sw = 0, Sx = 0, Sy = 0, Sxx = 0, Sxy = 0, Syy = 0;
  int cnt = 0;
  {  // direct state of row r0
    const int lo = max(S0(r0), r0 - W + 1);
    double w = 1.0;
    for (int j = r0; j >= lo; --j) {
      const float yv = Y(j), xv = X(j);
      if (!(fin(yv) && fin(xv))) continue;
      const double xd = xv, yd = yv;
      Sw += w; Sx = fma(w, xd, Sx); Sy = fma(w, yd, Sy);
      Sxx = fma(w * xd, xd, Sxx); Sxy = fma(w * xd, yd, Sxy); Syy = fma(w * yd, yd, Syy);
      w *= lam;
      ++cnt;
    }
  }
  for (int r = r0; r < r1; ++r) {
    if (r > r0) {
      const int s0 = S0(r);
      if (s0 == r) {  // a new stock starts: empty window
        Sw = Sx = Sy = Sxx = Sxy = Syy = 0.0;
        cnt = 0;
      }
      const float yv = Y(r), xv = X(r);
      if (fin(yv) && fin(xv)) {
        const double xd = xv, yd = yv;
        Sw = fma(lam, Sw, 1.0); Sx = fma(lam, Sx, xd); Sy = fma(lam, Sy, yd);
        Sxx = fma(lam, Sxx, xd * xd); Sxy = fma(lam, Sxy, xd * yd); Syy = fma(lam, Syy, yd * yd);
        ++cnt;
      }
      const int q = r - W;
      if (q >= s0) {
        const float yq = Y(q), xq = X(q);
        if (fin(yq) && fin(xq)) {
          const double w = sh.pw[cnt - 1], xd = xq, yd = yq;
          Sw -= w; Sx = fma(-w, xd, Sx); Sy = fma(-w, yd, Sy);
          Sxx = fma(-w * xd, xd, Sxx); Sxy = fma(-w * xd, yd, Sxy); Syy = fma(-w * yd, yd, Syy);
          --cnt;
        }
      }
    }
    float b = qnanf(), h = qnanf();
    if (cnt >= minp && cnt > 2) {
      const double iw = 1.0 / Sw;
      const double mx = Sx * iw, my = Sy * iw;
      const double vxx = Sxx * iw - mx * mx;
      const double cxy = Sxy * iw - mx * my;
      const double vyy = Syy * iw - my * my;
      const double bb = cxy / vxx;
      // weighted residual sum of squares of the fit: Sw (vyy - b cxy)
      const double ssr = fmax(Sw * (vyy - bb * cxy), 0.0);
      b = (float)bb;
      h = (float)sqrt(ssr / (double)(cnt - 2));
    }
    beta[r] = b;
    hsig[r] = h;
  }
}

template <int H>
__global__ __launch_bounds__(256) void dastd_scan_kernel(
    const float* __restrict__ ret, const float* __restrict__ mret, const int* __restrict__ seg_lo,
    int R, int W, double lam, int minp, float* __restrict__ out) {
  __shared__ Stage2<H> sh;
  const int b0 = blockIdx.x * kBlockRows, g0 = b0 - H;
  const int n = min(H + kBlockRows, R - g0);
  stage_f(sh.a, ret, g0, n, R);
  stage_f(sh.b, mret, g0, n, R);
  stage_i(sh.seg, seg_lo, g0, n, R);
  fill_pow(sh.pw, lam, W + 1);
  __syncthreads();
  const int r0 = b0 + threadIdx.x * kChunk;
  if (r0 >= R) return;
  const int r1 = min(r0 + kChunk, R);
  auto E = [&](int r, bool& ok) {
    const float a = sh.a[lds_idx(r - g0)], bm = sh.b[lds_idx(r - g0)];
    ok = fin(a) && fin(bm);
    return (double)a - (double)bm;
  };
  auto S0 = [&](int r) { return sh.seg[lds_idx(r - g0)]; };
  double Sw = 0, Se = 0, See = 0;
  int cnt = 0;
  {
    const int lo = max(S0(r0), r0 - W + 1);
    double w = 1.0;
    for (int j = r0; j >= lo; --j) {
      bool ok;
      const double e = E(j, ok);
      if (!ok) continue;
      Sw += w; Se = fma(w, e, Se); See = fma(w * e, e, See);
      w *= lam;
      ++cnt;
    }
  }
  for (int r = r0; r < r1; ++r) {
    if (r > r0) {
      const int s0 = S0(r);
      if (s0 == r) { Sw = Se = See = 0.0; cnt = 0; }
      bool ok;
      const double e = E(r, ok);
      if (ok) {
        Sw = fma(lam, Sw, 1.0); Se = fma(lam, Se, e); See = fma(lam, See, e * e);
        ++cnt;
      }
      const int q = r - W;
      if (q >= s0) {
        const double eq = E(q, ok);
        if (ok) {
          const double w = sh.pw[cnt - 1];
          Sw -= w; Se = fma(-w, eq, Se); See = fma(-w * eq, eq, See);
          --cnt;
        }
      }
    }
    float o = qnanf();
    if (cnt >= minp) {
      const double m = Se / Sw;
      o = (float)sqrt(fmax(See / Sw - m * m, 0.0));
    }
    out[r] = o;
  }
}

// ------------------------------------------------------------------------------------------
// Anchored-prefix EW window kernels (BETA/HSIGMA, DASTD): no per-chunk direct pass.
//
// With compressed weights (newest valid row 1, lam^k for k valid rows newer), the EW prefix
// from an anchor g0, E_r = lam E_{r-1} + v_r (valid rows only; reset to 0 at a stock start),
// gives every window sum exactly:  S_r = E_r - lam^{n_r} E_{r-W},  n_r = valid rows in
// (r-W, r]  (a window that crosses the stock start is just E_r).  lam^W >= 1/64 for the
// reference's half-lives, so the subtraction costs < 2 bits.  Persistent 256-thread blocks
// loop over tiles of 2048 rows [g0, g0 + 2048) (the first H >= W are halo); thread t owns the
// 8-row chunk t, kept in registers, and prefetches its chunk of the NEXT tile before computing:
//   A. the chunk's affine map E -> lam^c E + B (or B after a reset), c = valid rows;
//   B. inclusive scan of the 256 maps (wave shuffles, then the 4 wave totals in order);
//   C. own rows from the chunk's carry-in, lagged rows r - W (LDS copy of the tile) from the
//      carry-in of chunk (8t - W) / 8, O(1) per output row.
// Measured (5000 x 3780, 1x MI355X, tools/rolling_ab.py): BETA/HSIGMA 0.62 -> 0.21 ms,
// DASTD 0.55 -> 0.16 ms (profiles/r02_rolling_ab.jsonl).
// Work per row ~3 recurrence steps instead of W / 16 direct taps + 1.
// ------------------------------------------------------------------------------------------
template <int NS>
struct EwMap {
  double A;      // lam^(valid rows), multiplier of the carry-in
  double B[NS];  // contribution of the chunk's own rows
  int cnt;       // valid rows since the last reset (or chunk start)
  int reset;     // a stock starts inside: the carry-in is discarded
};

template <int NS>
__device__ __forceinline__ void ew_compose(EwMap<NS>& m, const EwMap<NS>& p) {  // m <- m o p
  if (m.reset) return;
#pragma unroll
  for (int k = 0; k < NS; ++k) m.B[k] = fma(m.A, p.B[k], m.B[k]);
  m.A *= p.A;
  m.cnt += p.cnt;
  m.reset = p.reset;
}

// One step of the map scan on DPP moves instead of ds_bpermute (no LDS round trip per field):
// lanes without a source (row_shr past the row start, rows outside ROW_MASK) compose with the
// identity map, which leaves m unchanged.  Steps row_shr 1 / 2 / 4 / 8, row_bcast:15 into rows
// 1 / 3, row_bcast:31 into rows 2 / 3 form the inclusive scan (associative compose).
template <int CTRL, int ROW_MASK, int NS>
__device__ __forceinline__ void ew_dpp_step(EwMap<NS>& m) {
  EwMap<NS> p;
  p.A = dpp_upd<CTRL, ROW_MASK>(m.A, 1.0);
#pragma unroll
  for (int k = 0; k < NS; ++k) p.B[k] = dpp_upd<CTRL, ROW_MASK>(m.B[k], 0.0);
  p.cnt = __builtin_amdgcn_update_dpp(0, m.cnt, CTRL, ROW_MASK, 0xF, false);
  p.reset = __builtin_amdgcn_update_dpp(0, m.reset, CTRL, ROW_MASK, 0xF, false);
  ew_compose(m, p);
}

template <int NS>
__device__ __forceinline__ EwMap<NS> ew_shfl_up(const EwMap<NS>& m, int d) {
  EwMap<NS> p;
  p.A = __shfl_up(m.A, d, 64);
#pragma unroll
  for (int k = 0; k < NS; ++k) p.B[k] = __shfl_up(m.B[k], d, 64);
  p.cnt = __shfl_up(m.cnt, d, 64);
  p.reset = __shfl_up(m.reset, d, 64);
  return p;
}

// fp32-output finishers: v_rcp_f64 / v_rsq_f64 seeds + one Newton step (~2e-15 relative, far
// below the fp32 rounding of the outputs) instead of the IEEE fp64 division / square-root
// sequences (~12 / ~15 dependent instructions each), which dominated the per-row VALU count.
__device__ __forceinline__ double frcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double fsqrt(double x) {  // x >= 0
  if (!(x > 0.0)) return 0.0;
  double y = __builtin_amdgcn_rsq(x);
  y = fma(0.5 * y, fma(-x * y, y, 1.0), y);
  return x * y;
}

struct BetaOp {  // y ~ 1 + x (ret ~ mret): sums of 1, x, y, xx, xy, yy
  static constexpr int NS = 6;
  // v = 0 for an invalid row (NaN in either series); returns validity
  __device__ static bool value(float yv, float xv, double (&v)[NS]) {
    const bool ok = fin(yv) && fin(xv);
    const double x = ok ? (double)xv : 0.0, y = ok ? (double)yv : 0.0;
    v[0] = ok ? 1.0 : 0.0; v[1] = x; v[2] = y; v[3] = x * x; v[4] = x * y; v[5] = y * y;
    return ok;
  }
  // sanitised rows (inputs already 0 on an invalid row): no per-step selects
  __device__ static void vals(float yv, float xv, double okd, double (&v)[NS]) {
    const double x = xv, y = yv;
    v[0] = okd; v[1] = x; v[2] = y; v[3] = x * x; v[4] = x * y; v[5] = y * y;
  }
  // ew_window_san_kernel: the weight sum of a window is implied by its valid count n
  // (sum_(k<n) lam^k, a table), so only the 5 data sums x, y, xx, xy, yy are carried
  static constexpr int NSX = 5;
  __device__ static void vals_x(float yv, float xv, double (&v)[NSX]) {
    const double x = xv, y = yv;
    v[0] = x; v[1] = y; v[2] = x * x; v[3] = x * y; v[4] = y * y;
  }
  __device__ static void emit_x(const double (&S)[NSX], double iw, int n, int minp, int r,
                                float* o0, float* o1) {
    float b = qnanf(), h = qnanf();
    if (n >= minp && n > 2) {
      const double mx = S[0] * iw, my = S[1] * iw;
      const double vxx = S[2] * iw - mx * mx;
      const double cxy = S[3] * iw - mx * my;
      const double bb = cxy * frcp(vxx);
      // Sw (vyy - b cxy) with Sw vyy = Syy - Sy my and Sw cxy = Sxy - Sx my
      const double ssr = fmax((S[4] - S[1] * my) - bb * (S[3] - S[0] * my), 0.0);
      b = (float)bb;
      h = __builtin_amdgcn_sqrtf((float)ssr * __builtin_amdgcn_rcpf((float)(n - 2)));
    }
    o0[r] = b;
    o1[r] = h;
  }
  __device__ static void emit(const double (&S)[NS], int n, int minp, int r, float* o0, float* o1) {
    float b = qnanf(), h = qnanf();
    if (n >= minp && n > 2) {
      const double iw = frcp(S[0]);
      const double mx = S[1] * iw, my = S[2] * iw;
      const double vxx = S[3] * iw - mx * mx;
      const double cxy = S[4] * iw - mx * my;
      const double vyy = S[5] * iw - my * my;
      const double bb = cxy * frcp(vxx);
      const double ssr = fmax(S[0] * (vyy - bb * cxy), 0.0);
      b = (float)bb;
      // past the cancellation the tail is fp32: ~2 ulp vs the fp64 sqrt (the window
      // subtraction already costs up to 2 bits), 3 instructions instead of 13
      h = __builtin_amdgcn_sqrtf((float)ssr * __builtin_amdgcn_rcpf((float)(n - 2)));
    }
    o0[r] = b;
    o1[r] = h;
  }
};

struct DastdOp {  // e = ret - mret: sums of 1, e, ee; weighted population std
  static constexpr int NS = 3;
  __device__ static bool value(float a, float bm, double (&v)[NS]) {
    const bool ok = fin(a) && fin(bm);
    const double e = ok ? (double)a - (double)bm : 0.0;
    v[0] = ok ? 1.0 : 0.0; v[1] = e; v[2] = e * e;
    return ok;
  }
  __device__ static void vals(float a, float bm, double okd, double (&v)[NS]) {
    const double e = (double)a - (double)bm;
    v[0] = okd; v[1] = e; v[2] = e * e;
  }
  static constexpr int NSX = 2;  // ew_window_san_kernel: the weight sum comes from the count
  __device__ static void vals_x(float a, float bm, double (&v)[NSX]) {
    const double e = (double)a - (double)bm;
    v[0] = e; v[1] = e * e;
  }
  __device__ static void emit_x(const double (&S)[NSX], double iw, int n, int minp, int r,
                                float* o0, float*) {
    float o = qnanf();
    if (n >= minp) {
      const double m = S[0] * iw;
      o = __builtin_amdgcn_sqrtf((float)fmax(S[1] * iw - m * m, 0.0));
    }
    o0[r] = o;
  }
  __device__ static void emit(const double (&S)[NS], int n, int minp, int r, float* o0, float*) {
    float o = qnanf();
    if (n >= minp) {
      const double iw = frcp(S[0]);
      const double m = S[1] * iw;
      o = __builtin_amdgcn_sqrtf((float)fmax(S[2] * iw - m * m, 0.0));
    }
    o0[r] = o;
  }
};


// padded staging index for C-row chunks: one spare word per chunk (odd lane stride C + 1)
template <int C>
__device__ __forceinline__ int ew_idx(int p) { return p + p / C; }

// Persistent, software-pipelined variant: each block loops over tiles of TR staged rows; a
// thread keeps its own C rows in registers (phase A and its own-row steps read them there, the
// LDS copy only serves other threads' lagged rows) and issues the NEXT tile's loads before
// computing the current one, so HBM latency hides behind the scan / window math.
// PF = false (default): no software prefetch of the next tile -- BETA 148 -> 128 VGPRs, 3 -> 4
// waves / SIMD, and the extra waves hide the tile loads better than the prefetch did (5000 x
// 3780: BETA/HSIGMA 0.196 -> 0.173 ms, DASTD 0.131 -> 0.122 ms, bitwise the same outputs,
// profiles/r03_rolling_nopf_ab.jsonl).  PF = true = ew variant 3.
template <class Op, int C, int TR, bool PF = true>
__global__ __launch_bounds__(TR / C) __attribute__((amdgpu_waves_per_eu(PF ? 1 : 4))) void
ew_window_pipe_kernel(
    const float* __restrict__ in_a, const float* __restrict__ in_b,
    const int* __restrict__ seg_lo, int R, int W, int H, double lam, int minp,
    float* __restrict__ o0, float* __restrict__ o1, int ntiles) {
  constexpr int NS = Op::NS, NT = TR / C, LEN = TR + TR / C;
  __shared__ float sa[LEN], sb[LEN];
  __shared__ short sd[LEN];  // rows since the stock start (clamped); -1 = outside [0, R)
  __shared__ double carry[NT][NS];
  __shared__ int ccnt[NT];
  __shared__ EwMap<NS> wtot[NT / 64];
  __shared__ double pw[257];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int k = t; k <= W; k += NT) pw[k] = ipow(lam, k);
  const int p0 = t * C;
  auto load = [&](int tile, float (&xa)[C], float (&xb)[C], short (&xd)[C]) {
    const int g = tile * (TR - H) - H + p0;
    if (g >= 0 && g + C <= R) {
#pragma unroll
      for (int i = 0; i < C; i += 4) {
        const float4 va = *(const float4*)(in_a + g + i), vb = *(const float4*)(in_b + g + i);
        const int4 vs = *(const int4*)(seg_lo + g + i);
        xa[i] = va.x; xa[i + 1] = va.y; xa[i + 2] = va.z; xa[i + 3] = va.w;
        xb[i] = vb.x; xb[i + 1] = vb.y; xb[i + 2] = vb.z; xb[i + 3] = vb.w;
        xd[i] = (short)min(g + i - vs.x, 32767);
        xd[i + 1] = (short)min(g + i + 1 - vs.y, 32767);
        xd[i + 2] = (short)min(g + i + 2 - vs.z, 32767);
        xd[i + 3] = (short)min(g + i + 3 - vs.w, 32767);
      }
    } else {
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int gi = g + i;
        const bool in = gi >= 0 && gi < R;
        xa[i] = in ? in_a[gi] : qnanf();
        xb[i] = in ? in_b[gi] : qnanf();
        xd[i] = (short)(in ? min(gi - seg_lo[gi], 32767) : -1);
      }
    }
  };
  // one row: reset at a stock start, decay only on valid rows (branchless, v = 0 if invalid)
  auto row = [&](float av, float bv, short d, double (&S)[NS], int& c, double& A, int& rs) {
    if (d < 0) return;
    const bool st = d == 0;
    double v[NS];
    const bool ok = Op::value(av, bv, v);
    const double f = st ? 0.0 : (ok ? lam : 1.0);
#pragma unroll
    for (int k = 0; k < NS; ++k) S[k] = fma(f, S[k], v[k]);
    A = st ? (ok ? lam : 1.0) : A * (ok ? lam : 1.0);
    c = (st ? 0 : c) + (ok ? 1 : 0);
    rs |= st;
  };
  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  float ra[C], rb[C];
  short rd[C];
  if constexpr (PF) load(tile, ra, rb, rd);
  for (; tile < ntiles; tile += gridDim.x) {
    if constexpr (!PF) load(tile, ra, rb, rd);
    const int g0 = tile * (TR - H) - H;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const int q = ew_idx<C>(p0 + i);
      sa[q] = ra[i];
      sb[q] = rb[i];
      sd[q] = rd[i];
    }
    float na[C], nb[C];
    short nd[C];
    const int nxt = tile + gridDim.x;
    if constexpr (PF)
      if (nxt < ntiles) load(nxt, na, nb, nd);
    // A. chunk map from registers
    EwMap<NS> m;
    m.A = 1.0;
#pragma unroll
    for (int k = 0; k < NS; ++k) m.B[k] = 0.0;
    m.cnt = 0;
    m.reset = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) row(ra[i], rb[i], rd[i], m.B, m.cnt, m.A, m.reset);
    // B. inclusive scan over the NT chunks
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const EwMap<NS> pm = ew_shfl_up(m, d);
      if (lane >= d) ew_compose(m, pm);
    }
    if (lane == 63) wtot[wid] = m;
    __syncthreads();
    for (int w = wid - 1; w >= 0; --w) ew_compose(m, wtot[w]);
#pragma unroll
    for (int k = 0; k < NS; ++k) carry[t][k] = m.B[k];
    ccnt[t] = m.cnt;
    __syncthreads();
    // C. outputs: own rows (registers) and lagged rows r - W (LDS)
    if (p0 >= H) {
      const int lp = p0 - W, lc = lp / C;
      double E[NS], L[NS];
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        E[k] = t > 0 ? carry[t - 1][k] : 0.0;
        L[k] = lc > 0 ? carry[lc - 1][k] : 0.0;
      }
      int ce = t > 0 ? ccnt[t - 1] : 0, cl = lc > 0 ? ccnt[lc - 1] : 0;
      double dA = 1.0;
      int drs = 0;
      for (int p = lc * C; p < lp; ++p) {
        const int q = ew_idx<C>(p);
        row(sa[q], sb[q], sd[q], L, cl, dA, drs);
      }
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int r = g0 + p0 + i;
        if (rd[i] < 0) break;  // past the end of the panel
        const int q = ew_idx<C>(lp + i);
        row(sa[q], sb[q], sd[q], L, cl, dA, drs);
        row(ra[i], rb[i], rd[i], E, ce, dA, drs);
        double S[NS];
        int nv;
        if (rd[i] >= W) {  // whole window inside the stock: subtract the lagged prefix
          nv = ce - cl;
          const double f = pw[nv];
#pragma unroll
          for (int k = 0; k < NS; ++k) S[k] = fma(-f, L[k], E[k]);
        } else {
          nv = ce;
#pragma unroll
          for (int k = 0; k < NS; ++k) S[k] = E[k];
        }
        Op::emit(S, nv, minp, r, o0, o1);
      }
    }
    __syncthreads();  // LDS tile / carries are rewritten by the next iteration
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < C; ++i) {
        ra[i] = na[i];
        rb[i] = nb[i];
        rd[i] = nd[i];
      }
    }
  }
}

template <class Op, int C, int TR, bool PF = true>
void launch_ew_pipe(const float* a, const float* b, const int* seg, int R, int W, int H,
                    double lam, int minp, float* o0, float* o1, hipStream_t s) {
  static int blocks = 0;
  if (blocks == 0) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ew_window_pipe_kernel<Op, C, TR, PF>, TR / C, 0);
    blocks = max(1, cus * max(per, 1));
  }
  const int ntiles = (R + TR - H - 1) / (TR - H);
  hipLaunchKernelGGL((ew_window_pipe_kernel<Op, C, TR, PF>), dim3(min(ntiles, blocks)), dim3(TR / C), 0,
                     s, a, b, seg, R, W, H, lam, minp, o0, o1, ntiles);
}

// ------------------------------------------------------------------------------------------
// Sanitised-row variant of the anchored-prefix kernel (default since round 4).  The round-3
// kernel spent ~40 VALU instructions per recurrence step, three steps per output row (chunk map,
// own row, lagged row): the finiteness tests, zero selects of both fp64 inputs and the merge
// copies of an exec-masked update (`if (d < 0) return`) were repeated at every step
// (`profiles/r03_pmc_rolling.txt`: 237 VALU / row).  Here the load stage tests each row ONCE:
// an invalid row's inputs become 0 and its validity / stock-start / outside state goes into a
// 16-bit code, so a step is branch-free -- 2 conversions, the value products, 2 selects of the
// decay factor and the NS fmas -- and an outside row is simply "invalid, no reset" (decay 1,
// value 0).  The chunk-map scan composes branch-free (a zero multiplier instead of a masked
// compose) and the window subtraction selects its lag factor instead of branching.  The
// window's weight sum is implied by its valid count (a table), so BETA carries 5 sums (not 6)
// and DASTD 2 (not 3) through the recurrences, the scan and the carries.
// ------------------------------------------------------------------------------------------
// row code: bits 0-13 rows since the stock start (clamped), bit 14 both inputs finite, bit 15
// outside [0, R) (its distance bits all set: neither a stock start nor valid)
constexpr unsigned kCdD = 0x3FFFu, kCdOk = 0x4000u, kCdOut = 0xBFFFu;

// DS: the chunk-map scan on DPP (ew_dpp_step) instead of __shfl_up (A/B variant 12: 113 / 96
// instead of 119 / 102 VGPRs for BETA / DASTD; not timed in round 4 -- tools/gpu_r04zh.sh)
template <class Op, int C, int TR, bool PF = false, bool SL = true, bool DS = false>
__global__ __launch_bounds__(TR / C) __attribute__((amdgpu_waves_per_eu(4))) void
ew_window_san_kernel(
    const float* __restrict__ in_a, const float* __restrict__ in_b,
    const int* __restrict__ seg_lo, int R, int W, int H, double lam, int minp,
    float* __restrict__ o0, float* __restrict__ o1, int ntiles) {
  constexpr int NS = Op::NSX, NT = TR / C, LEN = TR + TR / C;
  __shared__ float sa[LEN], sb[LEN];
  __shared__ unsigned short sd[LEN];
  __shared__ double carry[NT][NS];
  __shared__ int ccnt[NT];
  __shared__ EwMap<NS> wtot[NT / 64];
  __shared__ double pw[257];
  __shared__ double isw[257];  // 1 / sum_(k<n) lam^k: the weight sum of a window with n valid rows
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int k = t; k <= W; k += NT) pw[k] = ipow(lam, k);
  if (t == 0) {  // read after the tile loop's first barriers
    double sw = 0.0, p = 1.0;
    for (int k = 0; k <= W; ++k) {
      isw[k] = k ? 1.0 / sw : 0.0;
      sw += p;
      p *= lam;
    }
  }
  const int p0 = t * C;
  auto code = [](float& a, float& b, int d) -> unsigned {
    const bool ok = fin(a) && fin(b);
    a = ok ? a : 0.f;
    b = ok ? b : 0.f;
    return (unsigned)min(d, (int)kCdD) | (ok ? kCdOk : 0u);
  };
  auto load = [&](int tile, float (&xa)[C], float (&xb)[C], unsigned (&xd)[C]) {
    const int g = tile * (TR - H) - H + p0;
    if (g >= 0 && g + C <= R) {
#pragma unroll
      for (int i = 0; i < C; i += 4) {
        const float4 va = *(const float4*)(in_a + g + i), vb = *(const float4*)(in_b + g + i);
        const int4 vs = *(const int4*)(seg_lo + g + i);
        xa[i] = va.x; xa[i + 1] = va.y; xa[i + 2] = va.z; xa[i + 3] = va.w;
        xb[i] = vb.x; xb[i + 1] = vb.y; xb[i + 2] = vb.z; xb[i + 3] = vb.w;
        xd[i] = code(xa[i], xb[i], g + i - vs.x);
        xd[i + 1] = code(xa[i + 1], xb[i + 1], g + i + 1 - vs.y);
        xd[i + 2] = code(xa[i + 2], xb[i + 2], g + i + 2 - vs.z);
        xd[i + 3] = code(xa[i + 3], xb[i + 3], g + i + 3 - vs.w);
      }
    } else {
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int gi = g + i;
        if (gi >= 0 && gi < R) {
          xa[i] = in_a[gi];
          xb[i] = in_b[gi];
          xd[i] = code(xa[i], xb[i], gi - seg_lo[gi]);
        } else {
          xa[i] = 0.f;
          xb[i] = 0.f;
          xd[i] = kCdOut;
        }
      }
    }
  };
  // one recurrence step E <- f E + v: f = 0 at a stock start, lam on a valid row, 1 otherwise
  auto row = [&](float av, float bv, unsigned cd, double (&S)[NS], int& c) {
    const bool st = (cd & kCdD) == 0u, ok = (cd & kCdOk) != 0u;
    double v[NS];
    Op::vals_x(av, bv, v);
    const double f = st ? 0.0 : (ok ? lam : 1.0);
#pragma unroll
    for (int k = 0; k < NS; ++k) S[k] = fma(f, S[k], v[k]);
    c = (st ? 0 : c) + (ok ? 1 : 0);
  };
  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  float ra[C], rb[C];
  unsigned rd[C];
  if constexpr (PF) load(tile, ra, rb, rd);
  for (; tile < ntiles; tile += gridDim.x) {
    if constexpr (!PF) load(tile, ra, rb, rd);
    const int g0 = tile * (TR - H) - H;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const int q = ew_idx<C>(p0 + i);
      sa[q] = ra[i];
      sb[q] = rb[i];
      sd[q] = (unsigned short)rd[i];
    }
    // PF: the next tile's loads are in flight through the whole tile (raw values: the
    // sanitising code runs when they are consumed, so only 3 x C registers stay live)
    float na[C], nb[C];
    int ns[C];
    const int nxt = tile + gridDim.x, gn = nxt * (TR - H) - H + p0;
    const bool nfast = PF && nxt < ntiles && gn >= 0 && gn + C <= R;
    if constexpr (PF) {
      if (nfast) {
#pragma unroll
        for (int i = 0; i < C; i += 4) {
          const float4 va = *(const float4*)(in_a + gn + i), vb = *(const float4*)(in_b + gn + i);
          const int4 vs = *(const int4*)(seg_lo + gn + i);
          na[i] = va.x; na[i + 1] = va.y; na[i + 2] = va.z; na[i + 3] = va.w;
          nb[i] = vb.x; nb[i + 1] = vb.y; nb[i + 2] = vb.z; nb[i + 3] = vb.w;
          ns[i] = vs.x; ns[i + 1] = vs.y; ns[i + 2] = vs.z; ns[i + 3] = vs.w;
        }
      }
    }
    // A. chunk map from registers (A = lam^valid rows since the last reset / chunk start)
    EwMap<NS> m;
    m.A = 1.0;
#pragma unroll
    for (int k = 0; k < NS; ++k) m.B[k] = 0.0;
    m.cnt = 0;
    m.reset = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const unsigned cd = rd[i];
      const bool st = (cd & kCdD) == 0u, ok = (cd & kCdOk) != 0u;
      row(ra[i], rb[i], cd, m.B, m.cnt);
      m.A = (st ? 1.0 : m.A) * (ok ? lam : 1.0);
      m.reset |= st ? 1 : 0;
    }
    // B. inclusive scan over the NT chunks
    if constexpr (DS) {
      ew_dpp_step<0x111, 0xF>(m);
      ew_dpp_step<0x112, 0xF>(m);
      ew_dpp_step<0x114, 0xF>(m);
      ew_dpp_step<0x118, 0xF>(m);
      ew_dpp_step<0x142, 0xA>(m);
      ew_dpp_step<0x143, 0xC>(m);
    } else {
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const EwMap<NS> pm = ew_shfl_up(m, d);
        if (lane >= d) ew_compose(m, pm);
      }
    }
    if (lane == 63) wtot[wid] = m;
    __syncthreads();
    for (int w = wid - 1; w >= 0; --w) ew_compose(m, wtot[w]);
#pragma unroll
    for (int k = 0; k < NS; ++k) carry[t][k] = m.B[k];
    ccnt[t] = m.cnt;
    __syncthreads();
    // C. outputs: own rows (registers) and lagged rows r - W (LDS).  The empty asm hides the
    // own rows' identity from the optimiser: otherwise it keeps phase A's fp64 values of all C
    // rows alive across the scan for reuse (241 VGPRs, 2 waves / SIMD) instead of re-deriving
    // them (~5 instructions per row, 4 waves / SIMD).
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("" : "+v"(ra[i]), "+v"(rb[i]), "+v"(rd[i]));
    if (p0 >= H) {
      int lp = p0 - W;
      asm volatile("" : "+v"(lp));  // per-tile address math: not 24 hoisted LDS addresses
      const int lc = lp / C;
      double E[NS], L[NS];
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        E[k] = t > 0 ? carry[t - 1][k] : 0.0;
        L[k] = lc > 0 ? carry[lc - 1][k] : 0.0;
      }
      int ce = t > 0 ? ccnt[t - 1] : 0, cl = lc > 0 ? ccnt[lc - 1] : 0;
      for (int p = lc * C; p < lp; ++p) {
        const int q = ew_idx<C>(p);
        row(sa[q], sb[q], sd[q], L, cl);
      }
      if constexpr (SL) {
        // Sliding form: the window sum of row p0 - 1 from the prefixes (as below), then per row
        // S <- f S + v_r - lam^nv v_(r-W): the lagged row costs its value and one fma per sum,
        // not a second recurrence plus the prefix subtraction (~10 fewer VALU per row).  8 steps
        // of drift: ~1e-15 relative, far below the fp32 outputs.
        double S[NS];
        {
          const unsigned dp = sd[ew_idx<C>(p0 - 1)];
          const bool in = (int)(dp & kCdD) >= W;
          const double f = in ? pw[in ? ce - cl : 0] : 0.0;  // index in [0, W] even if not taken
#pragma unroll
          for (int k = 0; k < NS; ++k) S[k] = fma(-f, L[k], E[k]);
        }
#pragma unroll
        for (int i = 0; i < C; ++i) {
          const int r = g0 + p0 + i;
          if (rd[i] & 0x8000u) break;  // past the end of the panel
          row(ra[i], rb[i], rd[i], S, ce);
          const int q = ew_idx<C>(lp + i);
          const unsigned cq = sd[q];
          const bool stq = (cq & kCdD) == 0u, okq = (cq & kCdOk) != 0u;
          cl = (stq ? 0 : cl) + (okq ? 1 : 0);
          // whole window inside the stock: row r - W leaves it; else the window started with
          // the stock and S already is its sum
          const bool in = (int)(rd[i] & kCdD) >= W;
          const int nv = in ? ce - cl : ce;
          const double w = in ? pw[nv] : 0.0;
          double vq[NS];
          Op::vals_x(sa[q], sb[q], vq);
#pragma unroll
          for (int k = 0; k < NS; ++k) S[k] = fma(-w, vq[k], S[k]);
          Op::emit_x(S, isw[nv], nv, minp, r, o0, o1);
        }
      } else {
#pragma unroll
        for (int i = 0; i < C; ++i) {
          const int r = g0 + p0 + i;
          if (rd[i] & 0x8000u) break;  // past the end of the panel
          const int q = ew_idx<C>(lp + i);
          row(sa[q], sb[q], sd[q], L, cl);
          row(ra[i], rb[i], rd[i], E, ce);
          // whole window inside the stock: subtract the lagged prefix; else the window is E
          const bool in = (int)(rd[i] & kCdD) >= W;
          const int nv = in ? ce - cl : ce;
          const double f = in ? pw[nv] : 0.0;
          double S[NS];
#pragma unroll
          for (int k = 0; k < NS; ++k) S[k] = fma(-f, L[k], E[k]);
          Op::emit_x(S, isw[nv], nv, minp, r, o0, o1);
        }
      }
    }
    __syncthreads();  // LDS tile / carries are rewritten by the next iteration
    if constexpr (PF) {
      if (nfast) {
#pragma unroll
        for (int i = 0; i < C; ++i) {
          ra[i] = na[i];
          rb[i] = nb[i];
          rd[i] = code(ra[i], rb[i], gn + i - ns[i]);
        }
      } else if (nxt < ntiles) {
        load(nxt, ra, rb, rd);
      }
    }
  }
}

template <class Op, int C, int TR, bool PF = false, bool SL = true, bool DS = false>
void launch_ew_san(const float* a, const float* b, const int* seg, int R, int W, int H,
                   double lam, int minp, float* o0, float* o1, hipStream_t s) {
  static int blocks = 0;
  if (blocks == 0) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per, ew_window_san_kernel<Op, C, TR, PF, SL, DS>, TR / C, 0);
    blocks = max(1, cus * max(per, 1));
  }
  const int ntiles = (R + TR - H - 1) / (TR - H);
  hipLaunchKernelGGL((ew_window_san_kernel<Op, C, TR, PF, SL, DS>), dim3(min(ntiles, blocks)),
                     dim3(TR / C), 0, s, a, b, seg, R, W, H, lam, minp, o0, o1, ntiles);
}

// A/B geometry of the anchored-prefix kernel (mfa_rolling_set_ew_variant): 0 = sanitised rows,
// 8-row chunks x 256 threads (2048-row tiles), the sliding window update, count-implied weight
// sums and the next tile's loads in flight (BETA 0.142, DASTD 0.096 ms at 5000 x 3780,
// profiles/r04/rolling_ab.jsonl), 7 = the same (kept for the A/B tables), 5 = the round-3
// kernel at the same geometry (and the round-3 CMRA kernel), 1 = 8 x 512 (4096-row tiles: half the halo re-read), 2 = 16 x 256 (4096-row tiles,
// half the scan steps per row), 3 = round-3 geometry with the software prefetch of the next
// tile (3 waves / SIMD), 4 = 4096-row tiles without the prefetch, 6 = sanitised rows, 4096-row
// tiles, 8 = sanitised rows, 4096-row tiles with the prefetch, 9 = variant 0 with the per-row
// prefix subtraction instead of the sliding window update, 10 / 11 = 16-row chunks (slower,
// r04v), 12 = variant 0 with the chunk-map scan on DPP moves (BETA 0.139 vs 0.142, DASTD 0.108
// vs 0.095 ms: not adopted, profiles/r05/r05a/rolling_ab.jsonl).  Variants != 0: MFA_AB builds.
int g_ew_variant = 0;
template <class Op>
void launch_ew(const float* a, const float* b, const int* seg, int R, int W, int H, double lam,
               int minp, float* o0, float* o1, hipStream_t s) {
  if (g_ew_variant == 0 || !MFA_AB) {  // the next tile's loads in flight (BETA 119, DASTD 102 VGPRs)
    launch_ew_san<Op, 8, 2048, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
    return;
  }
#if MFA_AB
  if (g_ew_variant == 6)
    launch_ew_san<Op, 8, 4096>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 7)
    launch_ew_san<Op, 8, 2048, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 8)
    launch_ew_san<Op, 8, 4096, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 9)  // per-row prefix subtraction instead of the sliding form
    launch_ew_san<Op, 8, 2048, false, false>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 10)  // 16-row chunks, 4096-row tiles: half the scan steps and halo
    launch_ew_san<Op, 16, 4096, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 11)  // 16-row chunks, 2048-row tiles on 2-wave workgroups
    launch_ew_san<Op, 16, 2048, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 12)  // the default with the chunk-map scan on DPP moves
    launch_ew_san<Op, 8, 2048, true, true, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 1)
    launch_ew_pipe<Op, 8, 4096>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 2)
    launch_ew_pipe<Op, 16, 4096>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 4)  // A/B: 4096-row tiles without the prefetch (half the halo)
    launch_ew_pipe<Op, 8, 4096, false>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else if (g_ew_variant == 3)  // round-3 default until the 4-wave variant measured faster
    launch_ew_pipe<Op, 8, 2048, true>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
  else
    launch_ew_pipe<Op, 8, 2048, false>(a, b, seg, R, W, H, lam, minp, o0, o1, s);
#endif
}

template <int H>
struct Stage1 {  // one float series + seg_lo
  float a[lds_len(H + kBlockRows)];
  int seg[lds_len(H + kBlockRows)];
  double pw[kPowMax];
};

template <int H>
__global__ __launch_bounds__(256) void rstr_scan_kernel(const float* __restrict__ lr,
                                                        const int* __restrict__ seg_lo, int R,
                                                        int L, int W, double lam, int minp,
                                                        float* __restrict__ out) {
  __shared__ Stage1<H> sh;  // H >= W + L: rows r - W - L + 1 .. r are staged
  const int b0 = blockIdx.x * kBlockRows, g0 = b0 - H;
  const int n = min(H + kBlockRows, R - g0);
  stage_f(sh.a, lr, g0, n, R);
  stage_i(sh.seg, seg_lo, g0, n, R);
  fill_pow(sh.pw, lam, W + kChunk + 1);
  __syncthreads();
  const int r0 = b0 + threadIdx.x * kChunk;
  if (r0 >= R) return;
  const int r1 = min(r0 + kChunk, R);
  auto val = [&](int j, int s0) -> float { return j - L >= s0 ? sh.a[lds_idx(j - L - g0)] : qnanf(); };
  int s0 = sh.seg[lds_idx(r0 - g0)];
  int base = max(s0, r0 - W + 1);  // weights lam^(j - base)
  double num = 0.0, den = 0.0;
  int cnt = 0;
  for (int j = base; j <= r0; ++j) {
    const float v = val(j, s0);
    if (fin(v)) { const double w = sh.pw[j - base]; num = fma(w, (double)v, num); den += w; ++cnt; }
  }
  for (int r = r0; r < r1; ++r) {
    if (r > r0) {
      if (sh.seg[lds_idx(r - g0)] == r) {  // new stock: empty window, fresh base
        s0 = r;
        base = r;
        num = den = 0.0;
        cnt = 0;
      }
      const float v = val(r, s0);
      if (fin(v)) { const double w = sh.pw[r - base]; num = fma(w, (double)v, num); den += w; ++cnt; }
      const int q = r - W;
      if (q >= s0) {  // q >= base always holds here
        const float vq = val(q, s0);
        if (fin(vq)) { const double w = sh.pw[q - base]; num = fma(-w, (double)vq, num); den -= w; --cnt; }
      }
    }
    out[r] = (cnt >= minp) ? (float)(num / den) : qnanf();
  }
}

template <int H>
__global__ __launch_bounds__(256) void rolling_sum_scan_kernel(const float* __restrict__ x,
                                                               const int* __restrict__ seg_lo,
                                                               int R, int W, int minp,
                                                               double scale, int mode,
                                                               float* __restrict__ out) {
  __shared__ Stage1<H> sh;
  const int b0 = blockIdx.x * kBlockRows, g0 = b0 - H;
  const int n = min(H + kBlockRows, R - g0);
  stage_f(sh.a, x, g0, n, R);
  stage_i(sh.seg, seg_lo, g0, n, R);
  __syncthreads();
  const int r0 = b0 + threadIdx.x * kChunk;
  if (r0 >= R) return;
  const int r1 = min(r0 + kChunk, R);
  auto V = [&](int r) { return sh.a[lds_idx(r - g0)]; };
  auto S0 = [&](int r) { return sh.seg[lds_idx(r - g0)]; };
  double s = 0.0;
  int cnt = 0, nz = 0;  // valid count, non-zero count (an all-zero window sums to exactly 0)
  {
    const int lo = max(S0(r0), r0 - W + 1);
    for (int j = r0; j >= lo; --j) {
      const float v = V(j);
      if (fin(v)) { s += (double)v * scale; ++cnt; nz += v != 0.f; }
    }
  }
  for (int r = r0; r < r1; ++r) {
    if (r > r0) {
      const int s0 = S0(r);
      if (s0 == r) { s = 0.0; cnt = 0; nz = 0; }
      const float v = V(r);
      if (fin(v)) { s += (double)v * scale; ++cnt; nz += v != 0.f; }
      const int q = r - W;
      if (q >= s0) {
        const float vq = V(q);
        if (fin(vq)) { s -= (double)vq * scale; --cnt; nz -= vq != 0.f; }
      }
    }
    float o = qnanf();
    if (cnt >= minp) {
      const double sv = nz == 0 ? 0.0 : s;
      if (mode == 1) o = (sv == 0.0) ? qnanf() : (float)log(sv);
      else o = (float)sv;
    }
    out[r] = o;
  }
}

// CMRA = ln(1 + max Z) - ln(1 + min Z) with Z = exp(cumsum) - 1, i.e. max - min of the window's
// cumulative log-return path (no exp / log per tap).  The path offset cancels, so one running
// sum from the chunk's first window start serves every window of the chunk (NaN taps add 0 and
// are counted separately: a full-window CMRA is NaN if any tap is NaN).  Full mode, chunk rows
// r0 + i: window = head[i..] U core U tail[..i-1] with head = the C-1 rows before the common
// core and tail = the rows after r0, so each output costs O(1) after an O(W) core pass.
// Chunks touching a stock start, and the factor.py partial-window mode, walk each window
// directly (still from LDS).
template <int H>
__global__ __launch_bounds__(256) void cmra_scan_kernel(const float* __restrict__ lr,
                                                        const int* __restrict__ seg_lo, int R,
                                                        int W, int partial,
                                                        float* __restrict__ out) {
  __shared__ Stage1<H> sh;
  const int b0 = blockIdx.x * kBlockRows, g0 = b0 - H;
  const int n = min(H + kBlockRows, R - g0);
  stage_f(sh.a, lr, g0, n, R);
  stage_i(sh.seg, seg_lo, g0, n, R);
  __syncthreads();
  const int r0 = b0 + threadIdx.x * kChunk;
  if (r0 >= R) return;
  const int r1 = min(r0 + kChunk, R);
  auto V = [&](int r) { return sh.a[lds_idx(r - g0)]; };
  auto S0 = [&](int r) { return sh.seg[lds_idx(r - g0)]; };
  const int s0 = S0(r0);
  const bool fast = !partial && r0 - W + 1 >= s0 && S0(r1 - 1) == s0 && r1 - r0 == kChunk;
  if (fast) {
    constexpr int C = kChunk;
    const int b = r0 - W + 1;  // first window's start; running sum c_k from b
    double c = 0.0;
    double hmax[C - 1], hmin[C - 1];
    int hnan[C - 1];
    // head rows b .. b + C - 2
#pragma unroll
    for (int i = 0; i < C - 1; ++i) {
      const float v = V(b + i);
      const bool ok = fin(v);
      c += ok ? (double)v : 0.0;
      hmax[i] = c; hmin[i] = c; hnan[i] = ok ? 0 : 1;
    }
#pragma unroll
    for (int i = C - 3; i >= 0; --i) {  // suffix max / min / NaN count over head[i..]
      hmax[i] = fmax(hmax[i], hmax[i + 1]);
      hmin[i] = fmin(hmin[i], hmin[i + 1]);
      hnan[i] += hnan[i + 1];
    }
    double cmax = -1e300, cmin = 1e300;
    int cnan = 0;
    for (int k = b + C - 1; k <= r0; ++k) {  // core
      const float v = V(k);
      const bool ok = fin(v);
      c += ok ? (double)v : 0.0;
      cnan += ok ? 0 : 1;
      cmax = fmax(cmax, c);
      cmin = fmin(cmin, c);
    }
    double tmax = -1e300, tmin = 1e300;
    int tnan = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const int r = r0 + i;
      if (i > 0) {  // tail grows by row r
        const float v = V(r);
        const bool ok = fin(v);
        c += ok ? (double)v : 0.0;
        tnan += ok ? 0 : 1;
        tmax = fmax(tmax, c);
        tmin = fmin(tmin, c);
      }
      const double mx = fmax(fmax(i < C - 1 ? hmax[i] : -1e300, cmax), tmax);
      const double mn = fmin(fmin(i < C - 1 ? hmin[i] : 1e300, cmin), tmin);
      const int nn = (i < C - 1 ? hnan[i] : 0) + cnan + tnan;
      out[r] = nn == 0 ? (float)(mx - mn) : qnanf();
    }
    return;
  }
  for (int r = r0; r < r1; ++r) {
    const int sr = S0(r);
    float o = qnanf();
    if (!partial) {
      if (r - W + 1 >= sr) {
        double c = 0.0, mx = -1e300, mn = 1e300;
        bool ok = true;
        for (int j = r - W + 1; j <= r; ++j) {
          const float v = V(j);
          if (!fin(v)) { ok = false; break; }
          c += (double)v;
          mx = fmax(mx, c);
          mn = fmin(mn, c);
        }
        if (ok) o = (float)(mx - mn);
      }
    } else {  // factor.py: partial windows; pandas cumsum / max / min skip NaN
      double c = 0.0, mx = -1e300, mn = 1e300;
      int cnt = 0;
      for (int j = max(sr, r - W + 1); j <= r; ++j) {
        const float v = V(j);
        if (!fin(v)) continue;
        c += (double)v;
        mx = fmax(mx, c);
        mn = fmin(mn, c);
        ++cnt;
      }
      if (cnt > 0) o = (float)(mx - mn);
    }
    out[r] = o;
  }
}

// CMRA, full windows (the reference's factor_calculator.py:199-234 path), O(1) per row with the
// van Herk / Gil-Werman decomposition over 64-row blocks (one row per lane).  With c the running
// sum of the log returns from the workgroup's first staged row (NaN taps add 0; any NaN in a
// window makes it NaN), the window [a, r] of W > 64 rows is
//   [a, end of a's block] U full blocks U [start of r's block, r]
// so max c = max(suffix-max h[a], block maxima, prefix-max g[r]), likewise min, and CMRA =
// max - min (ln(1 + max Z) - ln(1 + min Z) with Z = exp(c - c_(a-1)) - 1; the offset cancels).
// Per 64-row block a wave does a sum scan, prefix / suffix max and min scans (DPP) and one NaN
// ballot; suffix values and block extrema go to LDS, prefix values stay in registers.  Each workgroup
// owns kVhRows output rows plus a kVhH-row halo (W - 1 <= kVhH), so HBM sees each row ~once.
// Replaced the chunked cmra_scan_kernel (O(W / kChunk) taps per row, latency-bound): A/B mode 2.
constexpr int kVhH = 256;
constexpr int kVhRows = 2048;
constexpr int kVhBlk = (kVhRows + kVhH) / 64;  // 36 staged 64-row blocks (37 KB of LDS: 4 WGs / CU)
constexpr int kVhWaves = 4;
constexpr int kVhBPW = kVhBlk / kVhWaves;      // 9 blocks per wave
static_assert(kVhBlk % kVhWaves == 0 && kVhH % 64 == 0, "block split");

__global__ __launch_bounds__(kVhWaves * 64) void cmra_vhgw_kernel(const float* __restrict__ lr,
                                                                  const int* __restrict__ seg_lo,
                                                                  int R, int W,
                                                                  float* __restrict__ out) {
  __shared__ double hmax[kVhBlk * 64], hmin[kVhBlk * 64];
  __shared__ double bmax[kVhBlk], bmin[kVhBlk];
  __shared__ unsigned long long nanm[kVhBlk];
  __shared__ double wtot[kVhWaves];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g0 = blockIdx.x * kVhRows - kVhH;
  // pass 1: this wave's rows (one per lane per block) and its total
  // (seg_lo of the output rows is loaded here too: pass 3 then waits on no global load)
  float v[kVhBPW];
  int sl[kVhBPW];
  double tot = 0.0;
#pragma unroll
  for (int k = 0; k < kVhBPW; ++k) {
    const int g = g0 + (wid * kVhBPW + k) * 64 + lane;
    v[k] = (g >= 0 && g < R) ? lr[g] : qnanf();
    sl[k] = ((wid * kVhBPW + k) * 64 >= kVhH && g < R) ? seg_lo[g] : 0;
  }
#pragma unroll
  for (int k = 0; k < kVhBPW; ++k) tot += fin(v[k]) ? (double)v[k] : 0.0;
  tot = wave_sum(tot);
  if (lane == 0) wtot[wid] = tot;
  __syncthreads();
  double carry = 0.0;
  for (int w = 0; w < wid; ++w) carry += wtot[w];
  // pass 2: running sum, block prefix (registers) / suffix (LDS) extrema, NaN masks.  All scans
  // are DPP (VALU-only); the suffix scans run as prefix scans of the lane-reversed sums (one
  // ds_bpermute) and store to the mirrored LDS slot.
  double gmax[kVhBPW], gmin[kVhBPW];
  unsigned long long gnan[kVhBPW];
#pragma unroll
  for (int k = 0; k < kVhBPW; ++k) {
    const int blk = wid * kVhBPW + k;
    const bool ok = fin(v[k]);
    const double c = wave_scan_dpp<0>(ok ? (double)v[k] : 0.0) + carry;
    carry = readlane(c, 63);
    const double cr = __shfl(c, 63 - lane, kWave);
    gmax[k] = wave_scan_dpp<1>(c);
    gmin[k] = wave_scan_dpp<2>(c);
    hmax[blk * 64 + 63 - lane] = wave_scan_dpp<1>(cr);
    hmin[blk * 64 + 63 - lane] = wave_scan_dpp<2>(cr);
    const unsigned long long m = __ballot(!ok);
    gnan[k] = m;
    if (lane == 63) { bmax[blk] = gmax[k]; bmin[blk] = gmin[k]; }
    if (lane == 0) nanm[blk] = m;
  }
  __syncthreads();
  // pass 3: outputs (the first kVhH staged rows are halo)
#pragma unroll
  for (int k = 0; k < kVhBPW; ++k) {
    const int blk = wid * kVhBPW + k;
    if (blk * 64 < kVhH) continue;
    const int t = blk * 64 + lane, r = g0 + t;
    if (r >= R) continue;
    float o = qnanf();
    if (r - W + 1 >= sl[k]) {
      const int at = t - W + 1, ba = at >> 6;  // ba < blk since W > 64
      double mx = fmax(hmax[at], gmax[k]), mn = fmin(hmin[at], gmin[k]);
      bool bad = (nanm[ba] >> (at & 63)) != 0 || (gnan[k] & (lane == 63 ? ~0ull : (2ull << lane) - 1)) != 0;
      for (int j = ba + 1; j < blk; ++j) {
        mx = fmax(mx, bmax[j]);
        mn = fmin(mn, bmin[j]);
        bad = bad || nanm[j] != 0;
      }
      if (!bad) o = (float)(mx - mn);
    }
    out[r] = o;
  }
}

// CMRA van Herk / Gil-Werman with TWO rows per lane (128-row blocks; default for W > 128).
// cmra_vhgw_kernel spends ~5 fp64 DPP scans (sum, prefix max / min, suffix max / min) per
// 64-row block, i.e. per row of each lane: 288 VALU instructions per row, VALU pipe ~97 % busy
// (profiles/r03_pmc_rolling.txt).  Here a lane owns rows 2L, 2L+1 of a 128-row block: the pair is
// combined in registers (sum, max / min of its two running sums) and the same five wave scans
// run over the 64 pair aggregates, so each scan serves two rows; the scans are the lean
// variants (common.h wave_scan_sum / wave_scan_ext: 4 instead of 5-6 VALU per step).  Prefix extrema of row 2L take
// the exclusive scan (shifted one lane), suffix extrema of row 2L+1 the exclusive suffix; the NaN
// masks are two ballots per block (even / odd rows).  A window of W >= 129 rows always starts in
// an earlier block than it ends, so [a, r] = suffix(a's block) U full blocks U prefix(r's block).
constexpr int kV2H = 256;
constexpr int kV2Blk = 16;                      // staged 128-row blocks: 2048 rows, 32 KB of LDS
constexpr int kV2Waves = 4;
constexpr int kV2BPW = kV2Blk / kV2Waves;       // 4 blocks per wave
constexpr int kV2Rows = kV2Blk * 128 - kV2H;    // 1792 output rows per workgroup
static_assert(kV2Blk % kV2Waves == 0 && kV2H % 128 == 0, "block split");

__device__ __forceinline__ unsigned long long shr64(unsigned long long m, int s) {
  return s >= 64 ? 0ull : m >> s;
}

__global__ __launch_bounds__(kV2Waves * 64) void cmra_vh2_kernel(const float* __restrict__ lr,
                                                                 const int* __restrict__ seg_lo,
                                                                 int R, int W,
                                                                 float* __restrict__ out) {
  __shared__ double hmax[kV2Blk * 128], hmin[kV2Blk * 128];
  __shared__ double bmax[kV2Blk], bmin[kV2Blk];
  __shared__ unsigned long long nan0[kV2Blk], nan1[kV2Blk];
  __shared__ double wtot[kV2Waves];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g0 = blockIdx.x * kV2Rows - kV2H;
  constexpr double kInf = __builtin_huge_val();
  // pass 1: loads (the wave's rows and seg_lo of its output rows) and the wave total
  float v[kV2BPW][2];
  int sl[kV2BPW][2];
  double tot = 0.0;
#pragma unroll
  for (int k = 0; k < kV2BPW; ++k) {
    const int blk = wid * kV2BPW + k;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int g = g0 + blk * 128 + 2 * lane + i;
      const bool in = g >= 0 && g < R;
      v[k][i] = in ? lr[g] : qnanf();
      sl[k][i] = (blk * 128 >= kV2H && in) ? seg_lo[g] : 0;
    }
  }
#pragma unroll
  for (int k = 0; k < kV2BPW; ++k)
    tot += (fin(v[k][0]) ? (double)v[k][0] : 0.0) + (fin(v[k][1]) ? (double)v[k][1] : 0.0);
  tot = wave_sum(tot);
  if (lane == 0) wtot[wid] = tot;
  __syncthreads();
  double carry = 0.0;
  for (int w = 0; w < wid; ++w) carry += wtot[w];
  // pass 2: running sums, prefix extrema (registers), suffix extrema (LDS), NaN masks
  const unsigned long long lt = (1ull << lane) - 1, le = lane == 63 ? ~0ull : (2ull << lane) - 1;
  double gmax[kV2BPW][2], gmin[kV2BPW][2];
  unsigned long long gn0[kV2BPW], gn1[kV2BPW];
#pragma unroll
  for (int k = 0; k < kV2BPW; ++k) {
    const int blk = wid * kV2BPW + k;
    const bool ok0 = fin(v[k][0]), ok1 = fin(v[k][1]);
    const double d0 = ok0 ? (double)v[k][0] : 0.0, d1 = ok1 ? (double)v[k][1] : 0.0;
    const double c1 = wave_scan_sum(d0 + d1) + carry, c0 = c1 - d1;
    carry = readlane(c1, 63);
    const double phi = vmax64(c0, c1), plo = vmin64(c0, c1);
    const double Mx = wave_scan_ext<true>(phi), Mn = wave_scan_ext<false>(plo);
    // every cross-lane read is executed by ALL lanes, the select comes after (a shuffle inside
    // `lane ? ... : ...` runs with the lanes that skip it disabled, and a disabled lane is not a
    // valid source)
    const double Mxu = __shfl_up(Mx, 1, kWave), Mnu = __shfl_up(Mn, 1, kWave);
    const double Mxe = lane ? Mxu : -kInf, Mne = lane ? Mnu : kInf;
    gmax[k][0] = vmax64(Mxe, c0); gmax[k][1] = Mx;
    gmin[k][0] = vmin64(Mne, c0); gmin[k][1] = Mn;
    // suffix scans as prefix scans of the lane-reversed pair extrema
    const double Rx = wave_scan_ext<true>(__shfl(phi, 63 - lane, kWave));
    const double Rn = wave_scan_ext<false>(__shfl(plo, 63 - lane, kWave));
    const double Sxi = __shfl(Rx, 63 - lane, kWave), Sni = __shfl(Rn, 63 - lane, kWave);
    const double Sxu = __shfl(Rx, (62 - lane) & 63, kWave), Snu = __shfl(Rn, (62 - lane) & 63, kWave);
    const double Sxe = lane < 63 ? Sxu : -kInf, Sne = lane < 63 ? Snu : kInf;
    const int t0 = blk * 128 + 2 * lane;
    hmax[t0] = Sxi; hmax[t0 + 1] = vmax64(c1, Sxe);
    hmin[t0] = Sni; hmin[t0 + 1] = vmin64(c1, Sne);
    const unsigned long long m0 = __ballot(!ok0), m1 = __ballot(!ok1);
    gn0[k] = m0; gn1[k] = m1;
    if (lane == 63) { bmax[blk] = Mx; bmin[blk] = Mn; }
    if (lane == 0) { nan0[blk] = m0; nan1[blk] = m1; }
  }
  __syncthreads();
  // pass 3: outputs (the first kV2H staged rows are halo)
#pragma unroll
  for (int k = 0; k < kV2BPW; ++k) {
    const int blk = wid * kV2BPW + k;
    if (blk * 128 < kV2H) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = blk * 128 + 2 * lane + i, r = g0 + t;
      if (r >= R) continue;
      float o = qnanf();
      if (r - W + 1 >= sl[k][i]) {
        const int at = t - W + 1, ba = at >> 7, ain = at & 127;  // ba < blk since W > 128
        double mx = vmax64(hmax[at], gmax[k][i]), mn = vmin64(hmin[at], gmin[k][i]);
        bool bad = (shr64(nan0[ba], (ain + 1) >> 1) | shr64(nan1[ba], ain >> 1)) != 0 ||
                   (gn0[k] & le) != 0 || (gn1[k] & (i ? le : lt)) != 0;
        for (int j = ba + 1; j < blk; ++j) {
          mx = vmax64(mx, bmax[j]);
          mn = vmin64(mn, bmin[j]);
          bad = bad || (nan0[j] | nan1[j]) != 0;
        }
        if (!bad) o = (float)(mx - mn);
      }
      out[r] = o;
    }
  }
}

// RSTR (factor_calculator.py:127-153): a NaN-renormalised positional-weight mean over the log
// returns lr[k], k in [kl, kr] = [max(seg_lo, r - W + 1 - L), r - L], weights lam^(k - kl) (the
// oldest row weighs 1; the reference's normalisation cancels the common base).  With the
// BACKWARD-anchored decayed sums U[k] = sum_(j >= k) lam^(j - k) x_j (terms shrink away from k,
// so no growth), the window sums are U[kl] - lam^(kr + 1 - kl) U[kr + 1] (numerator: x = lr,
// denominator: x = 1 on valid rows), the valid count a suffix-count difference: O(1) per row.
// Each wave scans its 64-row blocks last to first with lanes holding the block's rows in reverse
// (a forward DPP prefix of lam^-m x'), carries U across blocks, and the waves' regions are joined
// by their carry-ins when read.  Replaced the sliding rstr_scan_kernel (A/B mode 2).
constexpr int kRsH = 512;                       // halo: W + L - 1 <= kRsH
constexpr int kRsRows = 2048;                   // output rows per workgroup
constexpr int kRsBlk = (kRsRows + kRsH) / 64;   // 40 staged 64-row blocks
constexpr int kRsWaves = 4;
constexpr int kRsBPW = kRsBlk / kRsWaves;       // 10 blocks per wave
constexpr int kRsWRows = kRsBPW * 64;           // rows per wave region
static_assert(kRsBlk % kRsWaves == 0 && kRsH % 64 == 0, "block split");

// TWO (default since round 4): pass 2 on 128-row blocks with two rows per lane -- the pair's
// local decayed sum, then ONE DPP scan per block for each of the numerator / denominator serves
// both rows (the exclusive prefix for the first row of the pair is one lane shift): ~half the
// scan instructions per row.
template <bool TWO>
__global__ __launch_bounds__(kRsWaves * 64) void rstr_ew_kernel(const float* __restrict__ lr,
                                                                const int* __restrict__ seg_lo,
                                                                int R, int L, int W, double lam,
                                                                int minp,
                                                                float* __restrict__ out) {
  __shared__ double un[kRsBlk * 64], ud[kRsBlk * 64];
  __shared__ unsigned short cs[kRsBlk * 64];  // valid-row suffix count (region, then tile: <= 2560)
  __shared__ double pw[kRsWRows + 1];
  __shared__ double tn[kRsWaves], td[kRsWaves], in_n[kRsWaves], in_d[kRsWaves];
  __shared__ int tc[kRsWaves], in_c[kRsWaves];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g0 = blockIdx.x * kRsRows - kRsH;
  // lam^k without pow: lam^lane from a DPP product scan, times (lam^64)^(k / 64)
  const double lp = wave_scan_dpp<3>(lane == 0 ? 1.0 : lam), lp1 = lp * lam, lpn = 1.0 / lp;
  {
    const double l64 = readlane(lp1, 63);
    double blk = 1.0;
    for (int b = 0; b * 64 <= kRsWRows; ++b, blk *= l64)
      if (b % kRsWaves == wid && b * 64 + lane <= kRsWRows) pw[b * 64 + lane] = blk * lp;
  }
  // lane m holds block row 63 - m: U_block = lam^m * prefix(lam^-m x') + lam^(m+1) * carry
  const unsigned long long below = lane == 63 ? ~0ull : (2ull << lane) - 1;
  // every load of the workgroup issued up front (the block scans below are a serial chain):
  // this wave's log returns, lane-reversed per block, and seg_lo of its output rows
  float vv[kRsBPW];
  int sl[kRsBPW];
#pragma unroll
  for (int k = 0; k < kRsBPW; ++k) {
    const int g = g0 + (wid * kRsBPW + k) * 64 + 63 - lane;
    vv[k] = (g >= 0 && g < R) ? lr[g] : qnanf();
    const int go = g0 + (wid * kRsBPW + k) * 64 + lane;
    sl[k] = ((wid * kRsBPW + k) * 64 >= kRsH && go < R) ? seg_lo[go] : 0;
  }
  double cn = 0.0, cd = 0.0;
  int cc = 0;
  if constexpr (!TWO) {
#pragma unroll
    for (int k = kRsBPW - 1; k >= 0; --k) {
      const int t = (wid * kRsBPW + k) * 64 + 63 - lane;
      const float v = vv[k];
      const bool ok = fin(v);
      const double zn = wave_scan_sum(ok ? lpn * (double)v : 0.0);
      const double zd = wave_scan_sum(ok ? lpn : 0.0);
      const unsigned long long M = __ballot(ok);
      const double Un = fma(lp, zn, lp1 * cn), Ud = fma(lp, zd, lp1 * cd);
      un[t] = Un;
      ud[t] = Ud;
      cs[t] = (unsigned short)(cc + __popcll(M & below));
      cn = readlane(Un, 63);
      cd = readlane(Ud, 63);
      cc += __popcll(M);
    }
  } else {
    // 128-row blocks, lane m holds the block's reversed positions q = 2m, 2m + 1 (rows 127 - 2m,
    // 126 - 2m); the same row values as vv, re-read pairwise (L1 / L2 hits)
    constexpr int BPW2 = kRsBPW / 2;
    static_assert(kRsBPW % 2 == 0, "pairs of 64-row blocks");
    const double l2 = lam * lam;
    const double lq = wave_scan_dpp<3>(lane == 0 ? 1.0 : l2);  // lam^(2m)
    const double lqn = 1.0 / lq, lq1 = lq * lam, lq2 = lq * l2;
    const unsigned long long lt = (1ull << lane) - 1;
    float x0v[BPW2], x1v[BPW2];
#pragma unroll
    for (int k = 0; k < BPW2; ++k) {
      const int g = g0 + (wid * BPW2 + k) * 128 + 127 - 2 * lane;
      x0v[k] = (g >= 0 && g < R) ? lr[g] : qnanf();
      x1v[k] = (g - 1 >= 0 && g - 1 < R) ? lr[g - 1] : qnanf();
    }
#pragma unroll
    for (int k = BPW2 - 1; k >= 0; --k) {
      const int t0 = (wid * BPW2 + k) * 128 + 127 - 2 * lane, t1 = t0 - 1;
      const bool ok0 = fin(x0v[k]), ok1 = fin(x1v[k]);
      const double xn0 = ok0 ? (double)x0v[k] : 0.0, xn1 = ok1 ? (double)x1v[k] : 0.0;
      const double xd0 = ok0 ? 1.0 : 0.0, xd1 = ok1 ? 1.0 : 0.0;
      // prefix over q at the pair's second position: P_m = lam^2 P_(m-1) + (lam x_q0 + x_q1)
      const double Pn = lq * wave_scan_sum(lqn * fma(lam, xn0, xn1));
      const double Pd = lq * wave_scan_sum(lqn * fma(lam, xd0, xd1));
      const double Pnu = __shfl_up(Pn, 1, kWave), Pdu = __shfl_up(Pd, 1, kWave);
      const double Pne = lane ? Pnu : 0.0, Pde = lane ? Pdu : 0.0;
      // U at position q = prefix(q) + lam^(q+1) U(row after the block)
      const double Un0 = fma(lam, Pne, xn0) + lq1 * cn, Un1 = fma(lq2, cn, Pn);
      const double Ud0 = fma(lam, Pde, xd0) + lq1 * cd, Ud1 = fma(lq2, cd, Pd);
      un[t0] = Un0; un[t1] = Un1;
      ud[t0] = Ud0; ud[t1] = Ud1;
      const unsigned long long M0 = __ballot(ok0), M1 = __ballot(ok1);
      const int c01 = cc + __popcll(M0 & below);
      cs[t0] = (unsigned short)(c01 + __popcll(M1 & lt));
      cs[t1] = (unsigned short)(c01 + __popcll(M1 & below));
      cn = readlane(Un1, 63);
      cd = readlane(Ud1, 63);
      cc += __popcll(M0) + __popcll(M1);
    }
  }
  if (lane == 0) { tn[wid] = cn; td[wid] = cd; tc[wid] = cc; }
  __syncthreads();
  if (threadIdx.x == 0) {  // U / count at the first row after each wave's region
    double a = 0.0, b = 0.0;
    int c = 0;
    for (int w = kRsWaves - 1; w >= 0; --w) {
      in_n[w] = a; in_d[w] = b; in_c[w] = c;
      a = fma(pw[kRsWRows], a, tn[w]);
      b = fma(pw[kRsWRows], b, td[w]);
      c += tc[w];
    }
  }
  __syncthreads();
  // region-relative U / counts -> tile-absolute, once per row (the two window ends below then
  // need no region lookup / integer division): the same fma as a per-read lookup, so the outputs
  // are bitwise unchanged
  {
    const double fn = in_n[wid], fd = in_d[wid];
    const int fc = in_c[wid];
#pragma unroll
    for (int k = 0; k < kRsBPW; ++k) {
      const int t = (wid * kRsBPW + k) * 64 + lane;
      const double f = pw[(wid + 1) * kRsWRows - t];
      un[t] = fma(f, fn, un[t]);
      ud[t] = fma(f, fd, ud[t]);
      cs[t] = (unsigned short)(cs[t] + fc);
    }
  }
  __syncthreads();
  auto full = [&](int t, double& n, double& d, int& c) {
    n = un[t];
    d = ud[t];
    c = cs[t];
  };
#pragma unroll
  for (int k = 0; k < kRsBPW; ++k) {
    const int blk = wid * kRsBPW + k;
    if (blk * 64 < kRsH) continue;
    const int t = blk * 64 + lane, r = g0 + t;
    if (r >= R) continue;
    const int kl = max(sl[k], r - W + 1 - L), kr = r - L;
    float o = qnanf();
    if (kr >= kl) {
      const int tl = kl - g0, tr = kr + 1 - g0;
      double nl, dl, nr, dr;
      int cl, cr;
      full(tl, nl, dl, cl);
      full(tr, nr, dr, cr);
      if (cl - cr >= minp) {
        const double f = pw[tr - tl];
        o = (float)(fma(-f, nr, nl) * frcp(fma(-f, dr, dl)));
      }
    }
    out[r] = o;
  }
}

// ------------------------------------------------------------------------------------------
// Statement-row TTM (factor_calculator.py:392-410, quirk Q18): the rows of a stock form runs of
// one (ts_code, end_date) statement (a point-in-time as-of join keeps end_date non-decreasing),
// the TTM of a run is the NaN-skipping sum of the last 4 runs' values (min_periods 4), and every
// row takes its run's TTM.  Three row-parallel kernels around one int32 prefix sum, no host sync:
//   ttm_flags: run starts (stock change or end_date change) and two error bits (1 = end_date
//              moved backwards inside a stock: a restatement, the caller takes the sort path;
//              2 = one statement with two different values: the pandas path);
//   ttm_runs:  per run its value and stock (written by the run's first row);
//   ttm_rows:  the 4-run window of the row's run, summed newest first in fp64, rounded to fp32
//              like the rolling-sum kernel's output, widened back to fp64.
// Missing end dates (-1) sort last within a stock, as in the pandas path.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ long long ttm_key(long long e) { return e < 0 ? (1LL << 62) : e; }

__global__ __launch_bounds__(256) void ttm_flags_kernel(const int* __restrict__ sid,
                                                        const long long* __restrict__ end_date,
                                                        const float* __restrict__ v, int R,
                                                        int* __restrict__ start,
                                                        int* __restrict__ flags) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  int st = 1, bad = 0;
  if (r > 0) {
    const bool same = sid[r] == sid[r - 1];
    const long long e0 = ttm_key(end_date[r - 1]), e1 = ttm_key(end_date[r]);
    st = !(same && e0 == e1);
    if (same && e1 < e0) bad |= 1;
    if (!st) {
      const float a = v[r], b = v[r - 1];
      if (!(a == b || (a != a && b != b))) bad |= 2;
    }
  }
  start[r] = st;
  if (bad) atomicOr(flags, bad);
}

__global__ __launch_bounds__(256) void ttm_runs_kernel(const int* __restrict__ sid,
                                                       const float* __restrict__ v,
                                                       const int* __restrict__ start,
                                                       const int* __restrict__ run_incl, int R,
                                                       float* __restrict__ vf,
                                                       int* __restrict__ rsid) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !start[r]) return;
  const int q = run_incl[r] - 1;
  vf[q] = v[r];
  rsid[q] = sid[r];
}

__global__ __launch_bounds__(256) void ttm_rows_kernel(const int* __restrict__ run_incl,
                                                       const float* __restrict__ vf,
                                                       const int* __restrict__ rsid, int R,
                                                       double* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int q = run_incl[r] - 1, s0 = rsid[q];
  double s = 0.0;
  int n = 0;
  for (int k = q; k >= 0 && k > q - 4 && rsid[k] == s0; --k) {
    const float x = vf[k];
    if (fin(x)) { s += (double)x; ++n; }
  }
  out[r] = n >= 4 ? (double)(float)s : (double)qnanf();
}

// MLEV = (total_mv + total_ncl) / total_mv (+-inf -> NaN), BLEV = (BE + total_ncl) / BE for BE > 0,
// in fp64 from the fp32 columns, rounded to fp32 (factor_calculator.py:464-509): one pass instead
// of ~12 elementwise tensor launches.
__global__ __launch_bounds__(256) void leverage_kernel(const float* __restrict__ mv,
                                                       const float* __restrict__ ncl,
                                                       const float* __restrict__ be, int R,
                                                       float* __restrict__ mlev,
                                                       float* __restrict__ blev) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const double m = mv[r], n = ncl[r], b = be[r];
  const double ml = (m + n) / m;
  mlev[r] = __builtin_isinf(ml) ? qnanf() : (float)ml;
  blev[r] = b > 0.0 ? (float)((b + n) / b) : qnanf();
}

int g_roll_mode = 0;  // 0 = default (anchored-prefix / van Herk / sliding-window kernels), 1 = direct
                      // per-row kernels (A/B, tests), 2 = round-1 sliding-window BETA / DASTD /
                      // CMRA / RSTR (A/B)

int ew_halo(int W) { return (W + kChunk - 1) / kChunk * kChunk; }

}  // namespace

#define MFA_GRID(R) dim3(((R) + 255) / 256), dim3(256)
#define MFA_SCAN_GRID(R) dim3(((R) + kBlockRows - 1) / kBlockRows), dim3(256)

// mode 2 and ew variants != 0 exist only in MFA_AB builds (hipErrorInvalidValue otherwise)
MFA_API int mfa_rolling_set_mode(int mode) {
  if (!MFA_AB && mode == 2) return (int)hipErrorInvalidValue;
  g_roll_mode = mode;
  return 0;
}
MFA_API int mfa_rolling_set_ew_variant(int v) {
  if (!MFA_AB && v != 0) return (int)hipErrorInvalidValue;
  g_ew_variant = v;
  return 0;
}

MFA_API int mfa_beta_hsigma(const float* y, const float* x, const int* seg_lo, int R, int W,
                            double lam, int minp, float* beta, float* hsig, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W >= 1 && W <= 256) {
    launch_ew<BetaOp>(y, x, seg_lo, R, W, ew_halo(W), lam, minp, beta, hsig, (hipStream_t)s);
#if MFA_AB
  } else if (g_roll_mode == 2 && W <= 256) {
    hipLaunchKernelGGL(beta_hsigma_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, y, x,
                       seg_lo, R, W, lam, minp, beta, hsig);
#endif
  } else
    hipLaunchKernelGGL(beta_hsigma_kernel, MFA_GRID(R), 0, (hipStream_t)s, y, x, seg_lo, R, W, lam,
                       minp, beta, hsig);
  return (int)hipGetLastError();
}
// Rank-invariant BETA/HSIGMA and DASTD (FactorConfig.rank_invariant): the sanitised-row EW kernel
// at a 512-row tile geometry (256 output rows + a 256-row halo) on a VIRTUAL row layout that the
// caller builds (ops/rolling.py, _aligned_layout): every stock's rows sit at virtual positions
// B_s + t - T0_s with B_s a multiple of 256 and t the row's ordinal in the stock's FULL history,
// so the tiles, the 8-row chunks and the scan tree fall on global multiples of 256 whatever
// slice of the history a launch holds.  A date shard whose rows reach 512 back from its first
// owned row then computes every owned row with the same operations in the same order as the
// full panel: bitwise rank-invariant, at ~2x the tile kernel's rows instead of the direct
// kernels' W taps per row.  Rv: virtual rows (a multiple of 256); W <= 255 (the first owned row
// of a tile must see a full window of its own rows in both layouts).
MFA_API int mfa_beta_hsigma_aligned(const float* y, const float* x, const int* seg_lo, int Rv,
                                    int W, double lam, int minp, float* beta, float* hsig,
                                    void* s) {
  if (Rv <= 0) return 0;
  if (W < 1 || W > 255 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  launch_ew_san<BetaOp, 8, 512, true>(y, x, seg_lo, Rv, W, 256, lam, minp, beta, hsig,
                                      (hipStream_t)s);
  return (int)hipGetLastError();
}
MFA_API int mfa_dastd_aligned(const float* ret, const float* mret, const int* seg_lo, int Rv,
                              int W, double lam, int minp, float* out, void* s) {
  if (Rv <= 0) return 0;
  if (W < 1 || W > 255 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  launch_ew_san<DastdOp, 8, 512, true>(ret, mret, seg_lo, Rv, W, 256, lam, minp, out, out,
                                       (hipStream_t)s);
  return (int)hipGetLastError();
}
MFA_API int mfa_rstr(const float* lr, const int* seg_lo, int R, int L, int W, double lam,
                     int minp, float* out, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && L >= 1 && W >= 1 && W + L - 1 <= kRsH && W <= kRsWRows) {
#if MFA_AB
    if (g_ew_variant == 5)  // A/B: the round-3 pass 2 (one row per lane)
      hipLaunchKernelGGL(rstr_ew_kernel<false>, dim3((R + kRsRows - 1) / kRsRows),
                         dim3(kRsWaves * 64), 0, (hipStream_t)s, lr, seg_lo, R, L, W, lam, minp,
                         out);
    else
#endif
      hipLaunchKernelGGL(rstr_ew_kernel<true>, dim3((R + kRsRows - 1) / kRsRows),
                         dim3(kRsWaves * 64), 0, (hipStream_t)s, lr, seg_lo, R, L, W, lam, minp,
                         out);
  }
  else if (g_roll_mode != 1 && W + L <= 512 && W + kChunk + 1 <= kPowMax)
    hipLaunchKernelGGL(rstr_scan_kernel<512>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, L,
                       W, lam, minp, out);
  else
    hipLaunchKernelGGL(rstr_kernel, MFA_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, L, W, lam, minp, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_dastd(const float* ret, const float* mret, const int* seg_lo, int R, int W,
                      double lam, int minp, float* out, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W >= 1 && W <= 256) {
    launch_ew<DastdOp>(ret, mret, seg_lo, R, W, ew_halo(W), lam, minp, out, out, (hipStream_t)s);
#if MFA_AB
  } else if (g_roll_mode == 2 && W <= 256) {
    hipLaunchKernelGGL(dastd_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, ret, mret,
                       seg_lo, R, W, lam, minp, out);
#endif
  } else
    hipLaunchKernelGGL(dastd_kernel, MFA_GRID(R), 0, (hipStream_t)s, ret, mret, seg_lo, R, W, lam,
                       minp, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_cmra(const float* lr, const int* seg_lo, int R, int W, int partial, float* out,
                     void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && !partial && W > 128 && W - 1 <= kV2H && g_ew_variant != 5)
    hipLaunchKernelGGL(cmra_vh2_kernel, dim3((R + kV2Rows - 1) / kV2Rows), dim3(kV2Waves * 64), 0,
                       (hipStream_t)s, lr, seg_lo, R, W, out);
  else if (g_roll_mode == 0 && !partial && W > 64 && W - 1 <= kVhH)
    hipLaunchKernelGGL(cmra_vhgw_kernel, dim3((R + kVhRows - 1) / kVhRows), dim3(kVhWaves * 64), 0,
                       (hipStream_t)s, lr, seg_lo, R, W, out);
  else if (g_roll_mode != 1 && W <= 256 && W >= kChunk)
    hipLaunchKernelGGL(cmra_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, W,
                       partial, out);
  else
    hipLaunchKernelGGL(cmra_kernel, MFA_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, W, partial, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_rolling_sum(const float* x, const int* seg_lo, int R, int W, int minp,
                            double scale, int mode, float* out, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode != 1 && W <= 256)
    hipLaunchKernelGGL(rolling_sum_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, x, seg_lo,
                       R, W, minp, scale, mode, out);
  else
    hipLaunchKernelGGL(rolling_sum_kernel, MFA_GRID(R), 0, (hipStream_t)s, x, seg_lo, R, W, minp,
                       scale, mode, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_ttm_flags(const int* sid, const long long* end_date, const float* v, int R,
                          int* start, int* flags, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(ttm_flags_kernel, MFA_GRID(R), 0, (hipStream_t)s, sid, end_date, v, R, start,
                     flags);
  return (int)hipGetLastError();
}
// run_incl: inclusive prefix sum of `start` (the caller's device scan); vf / rsid: R scratch.
MFA_API int mfa_ttm_finish(const int* sid, const float* v, const int* start, const int* run_incl,
                           int R, float* vf, int* rsid, double* out, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(ttm_runs_kernel, MFA_GRID(R), 0, (hipStream_t)s, sid, v, start, run_incl, R,
                     vf, rsid);
  hipLaunchKernelGGL(ttm_rows_kernel, MFA_GRID(R), 0, (hipStream_t)s, run_incl, vf, rsid, R, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_leverage(const float* mv, const float* ncl, const float* be, int R, float* mlev,
                         float* blev, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(leverage_kernel, MFA_GRID(R), 0, (hipStream_t)s, mv, ncl, be, R, mlev, blev);
  return (int)hipGetLastError();
}
MFA_API int mfa_returns(const float* close, const int* seg_lo, int R, float* ret, float* logret,
                        void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(returns_kernel, MFA_GRID(R), 0, (hipStream_t)s, close, seg_lo, R, ret, logret);
  return (int)hipGetLastError();
}
