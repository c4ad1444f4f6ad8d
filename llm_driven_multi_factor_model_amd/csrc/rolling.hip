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

int g_roll_mode = 0;  // 0 = sliding-window kernels, 1 = direct per-row kernels (A/B, tests)

}  // namespace

#define MFA_GRID(R) dim3(((R) + 255) / 256), dim3(256)
#define MFA_SCAN_GRID(R) dim3(((R) + kBlockRows - 1) / kBlockRows), dim3(256)

MFA_API void mfa_rolling_set_mode(int mode) { g_roll_mode = mode; }

MFA_API int mfa_beta_hsigma(const float* y, const float* x, const int* seg_lo, int R, int W,
                            double lam, int minp, float* beta, float* hsig, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W <= 256)
    hipLaunchKernelGGL(beta_hsigma_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, y, x,
                       seg_lo, R, W, lam, minp, beta, hsig);
  else
    hipLaunchKernelGGL(beta_hsigma_kernel, MFA_GRID(R), 0, (hipStream_t)s, y, x, seg_lo, R, W, lam,
                       minp, beta, hsig);
  return (int)hipGetLastError();
}
MFA_API int mfa_rstr(const float* lr, const int* seg_lo, int R, int L, int W, double lam,
                     int minp, float* out, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W + L <= 512 && W + kChunk + 1 <= kPowMax)
    hipLaunchKernelGGL(rstr_scan_kernel<512>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, L,
                       W, lam, minp, out);
  else
    hipLaunchKernelGGL(rstr_kernel, MFA_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, L, W, lam, minp, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_dastd(const float* ret, const float* mret, const int* seg_lo, int R, int W,
                      double lam, int minp, float* out, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W <= 256)
    hipLaunchKernelGGL(dastd_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, ret, mret,
                       seg_lo, R, W, lam, minp, out);
  else
    hipLaunchKernelGGL(dastd_kernel, MFA_GRID(R), 0, (hipStream_t)s, ret, mret, seg_lo, R, W, lam,
                       minp, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_cmra(const float* lr, const int* seg_lo, int R, int W, int partial, float* out,
                     void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W <= 256 && W >= kChunk)
    hipLaunchKernelGGL(cmra_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, W,
                       partial, out);
  else
    hipLaunchKernelGGL(cmra_kernel, MFA_GRID(R), 0, (hipStream_t)s, lr, seg_lo, R, W, partial, out);
  return (int)hipGetLastError();
}
MFA_API int mfa_rolling_sum(const float* x, const int* seg_lo, int R, int W, int minp,
                            double scale, int mode, float* out, void* s) {
  if (R <= 0) return 0;
  if (g_roll_mode == 0 && W <= 256)
    hipLaunchKernelGGL(rolling_sum_scan_kernel<256>, MFA_SCAN_GRID(R), 0, (hipStream_t)s, x, seg_lo,
                       R, W, minp, scale, mode, out);
  else
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
