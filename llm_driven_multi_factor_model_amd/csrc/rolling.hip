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
// calendar days) exactly as pandas groupby-rolling does.  fp64 accumulation throughout.
//
// Two kernel families:
//   * segment-anchored kernels (the production path, single GPU and date shards alike): prefix
//     sums anchored at fixed ordinal segments of each stock's history, on the segment layout
//     built by ops/rolling.py -- rank-invariant by construction (see the block comment below);
//   * direct per-row kernels: every row sums its own window in one fixed order (the tests'
//     reference kernels and the fallback for windows beyond the segment kernels' limits).
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
};

struct DastdOp {  // e = ret - mret: sums of 1, e, ee; weighted population std
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
};

// ==========================================================================================
// Segment-anchored window kernels: ONE code path for a single GPU and for every date shard.
//
// A descriptor of row r is computed from prefix sums ANCHORED at the start of a fixed-size
// segment of the row's stock history (64 or 256 rows, on ordinals t = the row's position in
// the stock's FULL history), combined in a fixed order.  Rows run on the SEGMENT LAYOUT that
// ops/rolling.py builds (SegLayout): stock s's rows sit at virtual positions B_s + t - T0_s,
// with B_s and T0_s multiples of 256, so a segment boundary falls on the same ordinals whatever
// slice of the history a launch holds; padding positions are NaN and their own stock starts.
// Every output therefore depends only on the stock's rows from its anchor on, through the same
// operations in the same order: a date shard that holds each stock's rows from the anchor of its
// first owned row (halo_rows() in models/factor_engine.py) reproduces the full-panel outputs
// BIT FOR BIT, and the single-GPU run is that same computation -- at tile-kernel cost
// (each row staged once per 2048-row tile plus a 256/512-row halo; O(1)-ish work per row).
// Inputs are in the virtual layout; outputs go straight to the real rows through `omap`
// (virtual position -> real row, -1 on padding).
// ==========================================================================================

// ---- BETA/HSIGMA, DASTD: compressed EW weights (newest valid row 1, lam^k for k valid rows
// newer).  Persistent 256-thread blocks over 2048-row tiles (a 256-row halo + 1792 output
// rows); thread t owns the 8-row chunk t.  The chunk maps E -> lam^c E + B (reset at a stock
// start) are scanned INSIDE each 256-row segment (32 chunks: 5 shuffle steps, no cross-wave
// composition); a row of segment k reads its prefixes anchored at the start of segment k - 1:
// the segment-local prefix composed with segment k - 1's total.  Its window sum is then
// E_r - lam^n E_(r-W) (n valid rows in (r-W, r]; a window crossing the stock start is E_r)
// with r - W inside segments k - 1 .. k for W <= 256.  The lagged row r - W reads the LDS copy
// of the tile; the window slides 8 rows per thread from the prefix pair of its first row.
constexpr int kEwC = 8, kEwTR = 2048, kEwH = 256, kEwNT = kEwTR / kEwC, kEwSegT = 256 / kEwC;

// row code: bits 0-13 rows since the stock start (clamped), bit 14 both inputs finite, bit 15
// outside [0, Rv) (its distance bits all set: neither a stock start nor valid)
constexpr unsigned kCdD = 0x3FFFu, kCdOk = 0x4000u, kCdOut = 0xBFFFu;

template <int C>
__device__ __forceinline__ int ew_idx(int p) { return p + p / C; }  // one spare word per chunk

template <class Op>
__global__ __launch_bounds__(kEwNT) __attribute__((amdgpu_waves_per_eu(4))) void ew_seg_kernel(
    const float* __restrict__ in_a, const float* __restrict__ in_b, const int* __restrict__ seg_v,
    const int* __restrict__ omap, int Rv, int W, double lam, int minp, float* __restrict__ o0,
    float* __restrict__ o1, int ntiles) {
  constexpr int NS = Op::NSX, C = kEwC, NT = kEwNT, TR = kEwTR, H = kEwH, LEN = TR + TR / C;
  __shared__ float sa[LEN], sb[LEN];
  __shared__ unsigned short sd[LEN];
  __shared__ double carry[NT][NS];  // segment-local inclusive chunk maps: B, and
  __shared__ int ccnt[NT];          // valid count | reset << 16 (their A = lam^count)
  __shared__ EwMap<NS> stot[NT / kEwSegT];  // each segment's total map
  __shared__ double pw[257];
  __shared__ double isw[257];  // 1 / sum_(k<n) lam^k: the weight sum of a window with n valid rows
  const int t = threadIdx.x, lane = t & 63;
  for (int k = t; k <= 256; k += NT) pw[k] = ipow(lam, k);
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
    if (g >= 0 && g + C <= Rv) {
#pragma unroll
      for (int i = 0; i < C; i += 4) {
        const float4 va = *(const float4*)(in_a + g + i), vb = *(const float4*)(in_b + g + i);
        const int4 vs = *(const int4*)(seg_v + g + i);
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
        if (gi >= 0 && gi < Rv) {
          xa[i] = in_a[gi];
          xb[i] = in_b[gi];
          xd[i] = code(xa[i], xb[i], gi - seg_v[gi]);
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
  load(tile, ra, rb, rd);
  for (; tile < ntiles; tile += gridDim.x) {
    const int g0 = tile * (TR - H) - H;  // a multiple of 256: segments on ordinal multiples
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const int q = ew_idx<C>(p0 + i);
      sa[q] = ra[i];
      sb[q] = rb[i];
      sd[q] = (unsigned short)rd[i];
    }
    // the next tile's raw loads in flight through this tile (sanitised when consumed)
    float na[C], nb[C];
    int ns[C];
    const int nxt = tile + gridDim.x, gn = nxt * (TR - H) - H + p0;
    const bool nfast = nxt < ntiles && gn >= 0 && gn + C <= Rv;
    if (nfast) {
#pragma unroll
      for (int i = 0; i < C; i += 4) {
        const float4 va = *(const float4*)(in_a + gn + i), vb = *(const float4*)(in_b + gn + i);
        const int4 vs = *(const int4*)(seg_v + gn + i);
        na[i] = va.x; na[i + 1] = va.y; na[i + 2] = va.z; na[i + 3] = va.w;
        nb[i] = vb.x; nb[i + 1] = vb.y; nb[i + 2] = vb.z; nb[i + 3] = vb.w;
        ns[i] = vs.x; ns[i + 1] = vs.y; ns[i + 2] = vs.z; ns[i + 3] = vs.w;
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
    // B. inclusive scan of the chunk maps inside each 32-chunk (256-row) segment
#pragma unroll
    for (int d = 1; d < kEwSegT; d <<= 1) {
      const EwMap<NS> pm = ew_shfl_up(m, d);
      if ((lane & (kEwSegT - 1)) >= d) ew_compose(m, pm);
    }
    if ((t & (kEwSegT - 1)) == kEwSegT - 1) stot[t / kEwSegT] = m;
#pragma unroll
    for (int k = 0; k < NS; ++k) carry[t][k] = m.B[k];
    ccnt[t] = m.cnt | (m.reset << 16);
    __syncthreads();
    // C. outputs of the segments after the first (the halo): own rows from registers, lagged
    // rows r - W from the LDS copy.  The empty asm keeps the optimiser from holding phase A's
    // fp64 row values across the scan (VGPR pressure, see the round-4 sanitised kernel).
#pragma unroll
    for (int i = 0; i < C; ++i) asm volatile("" : "+v"(ra[i]), "+v"(rb[i]), "+v"(rd[i]));
    if (p0 >= H) {
      const int sg = t / kEwSegT;
      int lp = p0 - W;
      asm volatile("" : "+v"(lp));
      const int lc = lp / C;
      // prefix through chunk q anchored at the start of segment sg - 1 (q >= 32 (sg - 1) - 1)
      auto anchored = [&](int q, double (&X)[NS], int& c) {
        if (q < (sg - 1) * kEwSegT) {
#pragma unroll
          for (int k = 0; k < NS; ++k) X[k] = 0.0;
          c = 0;
          return;
        }
        EwMap<NS> mm;
#pragma unroll
        for (int k = 0; k < NS; ++k) mm.B[k] = carry[q][k];
        const int cr = ccnt[q];
        mm.cnt = cr & 0xFFFF;
        mm.reset = cr >> 16;
        mm.A = pw[mm.cnt];  // lam^(valid rows since the segment start or the reset)
        if (q / kEwSegT == sg) ew_compose(mm, stot[sg - 1]);
#pragma unroll
        for (int k = 0; k < NS; ++k) X[k] = mm.B[k];
        c = mm.cnt;
      };
      double E[NS], L[NS];
      int ce, cl;
      anchored(t - 1, E, ce);
      anchored(lc - 1, L, cl);
      for (int p = lc * C; p < lp; ++p) {
        const int q = ew_idx<C>(p);
        row(sa[q], sb[q], sd[q], L, cl);
      }
      // the window sum of row p0 - 1, then per row S <- f S + v_r - lam^nv v_(r-W)
      double S[NS];
      {
        const unsigned dp = sd[ew_idx<C>(p0 - 1)];
        const bool in = (int)(dp & kCdD) >= W;
        const double f = in ? pw[in ? ce - cl : 0] : 0.0;
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
        const bool in = (int)(rd[i] & kCdD) >= W;
        const int nv = in ? ce - cl : ce;
        const double w = in ? pw[nv] : 0.0;
        double vq[NS];
        Op::vals_x(sa[q], sb[q], vq);
#pragma unroll
        for (int k = 0; k < NS; ++k) S[k] = fma(-w, vq[k], S[k]);
        const int ro = omap[r];
        if (ro >= 0) Op::emit_x(S, isw[nv], nv, minp, ro, o0, o1);
      }
    }
    __syncthreads();  // LDS tile / carries are rewritten by the next iteration
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

template <class Op>
void launch_ew_seg(const float* a, const float* b, const int* seg_v, const int* omap, int Rv, int W,
                   double lam, int minp, float* o0, float* o1, hipStream_t s) {
  static int blocks = 0;
  if (blocks == 0) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ew_seg_kernel<Op>, kEwNT, 0);
    blocks = max(1, cus * max(per, 1));
  }
  const int ntiles = (Rv + kEwTR - kEwH - 1) / (kEwTR - kEwH);
  hipLaunchKernelGGL((ew_seg_kernel<Op>), dim3(min(ntiles, blocks)), dim3(kEwNT), 0, s, a, b, seg_v,
                     omap, Rv, W, lam, minp, o0, o1, ntiles);
}

// ---- positional-weight windows: RSTR (ratio of weighted sums) and the STOM / STOQ / STOA
// sums (one pass for all three).  Window of row r: sources [kl, kr] = [max(s0, r - W + 1 - L),
// r - L], source k weighted lam^(k - kl) (RSTR's oldest row weighs 1, quirk Q14; lam = 1 for
// the sums).  With 64-row segments j and the segment-local prefix G_j(p) = sum_(64j <= i <= p)
// lam^(i - 64j) x_i (one DPP scan per segment), the window sum anchored at jl = kl / 64 is
//   S_jl(m) + lam^(64 m) G_jr(kr) - G_jl(kl - 1),   m = jr - jl,
// S_j(m) = T_j + lam^64 T_(j+1) + ... + lam^(64 (m-1)) T_(j+m-1) (T = segment totals) -- a
// left-fold table of <= 9 entries per segment built once per tile, so a row costs one fma and a
// handful of LDS reads whatever its window spans (the RSTR ratio's common factor lam^(kl - 64 jl)
// cancels).  A 256-thread block stages 2048 output rows plus an H-row halo (H >= the reach
// W + L - 1 rounded up to 64), every row loaded once and scanned per 64-row segment.
constexpr int kPosOut = 2048;
constexpr int kPosMF = 9;  // fold-table entries per segment: m = 0 .. 8 (reach <= 512)

template <int H, bool RATIO, int NW>
__global__ __launch_bounds__(256) void poswin_seg_kernel(
    const float* __restrict__ x, const int* __restrict__ seg_v, const int* __restrict__ omap,
    int Rv, int L, int W0, int W1, int W2, int m0, int m1, int m2, double lam, double scale,
    int log_out, float* __restrict__ o0, float* __restrict__ o1, float* __restrict__ o2) {
  constexpr int NSEG = (H + kPosOut) / 64, SPW = NSEG / 4;
  static_assert(NSEG % 4 == 0, "segments split over the 4 waves");
  __shared__ double gn[NSEG * 64];
  __shared__ double gd[RATIO ? NSEG * 64 : 1];
  __shared__ unsigned char gc[NSEG * 64];
  __shared__ double tn[NSEG], td[NSEG];
  __shared__ int tc[NSEG];
  __shared__ double fn[NSEG][kPosMF], fd[RATIO ? NSEG : 1][kPosMF];
  __shared__ int fc[NSEG][kPosMF];
  __shared__ double lpm[kPosMF];  // lam^(64 m)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g0 = blockIdx.x * kPosOut - H;
  // lam^lane and lam^64 from one product scan: the same bits in every workgroup
  const double lp = wave_scan_dpp<3>(lane == 0 ? 1.0 : lam);
  const double l64 = readlane(lp * lam, 63);
  const unsigned long long below = lane == 63 ? ~0ull : (2ull << lane) - 1;
  float v[SPW];
#pragma unroll
  for (int k = 0; k < SPW; ++k) {
    const int g = g0 + (wid * SPW + k) * 64 + lane;
    v[k] = (g >= 0 && g < Rv) ? x[g] : qnanf();
  }
#pragma unroll
  for (int k = 0; k < SPW; ++k) {
    const int s = wid * SPW + k;
    const bool ok = fin(v[k]);
    const double xv = ok ? (double)v[k] * scale : 0.0;
    const double Gn = wave_scan_sum(lp * xv);
    gn[s * 64 + lane] = Gn;
    double Gd = 0.0;
    if constexpr (RATIO) {
      Gd = wave_scan_sum(ok ? lp : 0.0);
      gd[s * 64 + lane] = Gd;
    }
    const int c = __popcll(__ballot(ok) & below);
    gc[s * 64 + lane] = (unsigned char)c;
    if (lane == 63) {
      tn[s] = Gn;
      td[s] = Gd;
      tc[s] = c;
    }
  }
  if (threadIdx.x == 0) {
    double p = 1.0;
    for (int m = 0; m < kPosMF; ++m, p *= l64) lpm[m] = p;
  }
  __syncthreads();
  // the fold tables: one thread per segment, m = 0 .. 8 in order (within the tile)
  if (threadIdx.x < NSEG) {
    const int j = threadIdx.x;
    double an = 0.0, ad = 0.0;
    int ac = 0;
    fn[j][0] = 0.0;
    if constexpr (RATIO) fd[j][0] = 0.0;
    fc[j][0] = 0;
    for (int m = 1; m < kPosMF; ++m) {
      if (j + m - 1 < NSEG) {
        an = fma(lpm[m - 1], tn[j + m - 1], an);
        if constexpr (RATIO) ad = fma(lpm[m - 1], td[j + m - 1], ad);
        ac += tc[j + m - 1];
      }
      fn[j][m] = an;
      if constexpr (RATIO) fd[j][m] = ad;
      fc[j][m] = ac;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPosOut / 256; ++k) {
    const int r = g0 + H + (wid * (kPosOut / 256) + k) * 64 + lane;
    if (r >= Rv) continue;
    const int ro = omap[r];
    if (ro < 0) continue;
    const int s0 = seg_v[r];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int W = w == 0 ? W0 : (w == 1 ? W1 : W2), mp = w == 0 ? m0 : (w == 1 ? m1 : m2);
      float* o = w == 0 ? o0 : (w == 1 ? o1 : o2);
      const int kr = r - L, kl = max(s0, r - W + 1 - L);
      float res = qnanf();
      if (kr >= kl) {
        const int tl = kl - g0, tr = kr - g0, jl = tl >> 6, m = (tr >> 6) - jl;
        const bool mid = (tl & 63) != 0;
        const double f = lpm[m];
        double an = fma(f, gn[tr], fn[jl][m]);
        if (mid) an -= gn[tl - 1];
        int c = fc[jl][m] + gc[tr] - (mid ? gc[tl - 1] : 0);
        if (c >= mp) {
          if constexpr (RATIO) {
            double ad = fma(f, gd[tr], fd[jl][m]);
            if (mid) ad -= gd[tl - 1];
            res = (float)(an * frcp(ad));
          } else {
            res = log_out ? (an == 0.0 ? qnanf() : (float)log(an)) : (float)an;
          }
        }
      }
      o[ro] = res;
    }
  }
}

// ---- CMRA (full windows): max - min of the window's cumulative log returns (the reference's
// ln(1 + max Z) - ln(1 + min Z), Z = exp(cumsum) - 1, is that difference: no exp / log per row),
// c_i = P(i) - P(r - W) over i in [r - W + 1, r], P anchored at the 64-row segment of the
// window's first row; the base P(r - W) cancels in max - min.  P(i) = B_j + G_j(i) on segment j
// (B = the left fold of the segment totals), and since x -> fl(B + x) is monotone, the window
// max is the max of the pieces fl(B_j + max G_j over the piece): the first segment's suffix
// extremum (an LDS table from a lane-reversed DPP scan), whole middle segments, and the last
// segment's prefix extremum (registers: each wave scans the segments it outputs).  Any
// non-finite row in the window (or a window crossing the stock start) gives NaN.  64 < W <= 257.
// Waves: wave w scans halo segment w and output segments 4 + 8w .. 4 + 8w + 7.
template <int H>
__global__ __launch_bounds__(256) void cmra_seg_kernel(const float* __restrict__ x,
                                                       const int* __restrict__ seg_v,
                                                       const int* __restrict__ omap, int Rv, int W,
                                                       float* __restrict__ out) {
  constexpr int HS = H / 64, NSEG = HS + kPosOut / 64, OPW = kPosOut / 256;
  static_assert(HS == 4, "one halo segment per wave");
  __shared__ double g[NSEG * 64], smx[NSEG * 64], smn[NSEG * 64];
  __shared__ unsigned char gbad[NSEG * 64];
  __shared__ double tot[NSEG];
  __shared__ int tbad[NSEG];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g0 = blockIdx.x * kPosOut - H;
  const unsigned long long below = lane == 63 ? ~0ull : (2ull << lane) - 1;
  auto seg_of = [&](int k) { return k == OPW ? wid : HS + wid * OPW + k; };  // k = OPW: halo
  float v[OPW + 1];
#pragma unroll
  for (int k = 0; k <= OPW; ++k) {
    const int gi = g0 + seg_of(k) * 64 + lane;
    v[k] = (gi >= 0 && gi < Rv) ? x[gi] : qnanf();
  }
  double pmx[OPW], pmn[OPW];
#pragma unroll
  for (int k = 0; k <= OPW; ++k) {
    const int s = seg_of(k);
    const bool ok = fin(v[k]);
    const double G = wave_scan_sum(ok ? (double)v[k] : 0.0);
    const int bad = __popcll(__ballot(!ok) & below);
    const double Gr = __shfl(G, 63 - lane, 64);  // lane-reversed: suffix extrema as prefix scans
    const double mxr = wave_scan_ext<true>(Gr), mnr = wave_scan_ext<false>(Gr);
    g[s * 64 + lane] = G;
    smx[s * 64 + lane] = __shfl(mxr, 63 - lane, 64);
    smn[s * 64 + lane] = __shfl(mnr, 63 - lane, 64);
    gbad[s * 64 + lane] = (unsigned char)bad;
    if (lane == 63) {
      tot[s] = G;
      tbad[s] = bad;
    }
    if (k < OPW) {  // an output segment: its prefix extrema stay in registers
      pmx[k] = wave_scan_ext<true>(G);
      pmn[k] = wave_scan_ext<false>(G);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < OPW; ++k) {
    const int tr = seg_of(k) * 64 + lane, r = g0 + tr;
    if (r >= Rv) continue;
    const int ro = omap[r];
    if (ro < 0) continue;
    const int first = r - W + 1;
    float o = qnanf();
    if (first >= seg_v[r]) {
      const int tl = first - g0, jl = tl >> 6, jr = tr >> 6;
      int bad = gbad[tr] - ((tl & 63) ? gbad[tl - 1] : 0);
      for (int j = jl; j < jr; ++j) bad += tbad[j];
      if (bad == 0) {
        double mx = smx[tl], mn = smn[tl], B = tot[jl];
        for (int j = jl + 1; j < jr; ++j) {
          mx = vmax64(mx, B + smx[j * 64]);
          mn = vmin64(mn, B + smn[j * 64]);
          B += tot[j];
        }
        mx = vmax64(mx, B + pmx[k]);
        mn = vmin64(mn, B + pmn[k]);
        o = (float)(mx - mn);
      }
    }
    out[ro] = o;
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

// ---- the segment layout itself (ops/rolling.py SegLayout), in three row-parallel passes
// around one int32 prefix sum instead of ~30 tensor ops:
//   seg_count: on the LAST row of every stock, its padded 256-row block count
//              ((t_last - T0) / 256 + 1, T0 = the stock's first ordinal rounded down to 256);
//   (caller)   incl = inclusive prefix sum of the counts: the virtual base of stock s is
//              256 * incl[first row of s - 1] and Rv = 256 * incl[R - 1];
//   seg_place: every real row r at v = base_s - T0 + t_r: its omap, seg_v and series values;
//              the padding positions (their own stock start, no real row, NaN series values)
//              by the real row before them.
// t_r = the row's full-history ordinal (row_ord; null = r - seg_lo[r], the rows are histories).
struct SegSeries {
  const float* src[4];
  float* dst[4];
  int n;
};

__device__ __forceinline__ int seg_ord(const int* __restrict__ ro, const int* __restrict__ seg_lo,
                                       int r) {
  return ro ? ro[r] : r - seg_lo[r];
}

__global__ __launch_bounds__(256) void seg_count_kernel(const int* __restrict__ seg_lo,
                                                        const int* __restrict__ ro, int R,
                                                        int* __restrict__ nb) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const int sl = seg_lo[r];
  const bool last = r + 1 == R || seg_lo[r + 1] != sl;
  const int T0 = seg_ord(ro, seg_lo, sl) & ~255;
  nb[r] = last ? ((seg_ord(ro, seg_lo, r) - T0) >> 8) + 1 : 0;
}

// padding positions [p0, p1): their own stock start, no real row, NaN series values
__device__ __forceinline__ void seg_pad(int p0, int p1, int* __restrict__ seg_v,
                                        int* __restrict__ omap, const SegSeries& ser) {
  for (int p = p0; p < p1; ++p) {
    if (seg_v) {
      seg_v[p] = p;
      omap[p] = -1;
    }
    for (int k = 0; k < ser.n; ++k) ser.dst[k][p] = qnanf();
  }
}

__global__ __launch_bounds__(256) void seg_place_kernel(const int* __restrict__ seg_lo,
                                                        const int* __restrict__ ro,
                                                        const int* __restrict__ incl, int R,
                                                        int* __restrict__ seg_v,
                                                        int* __restrict__ omap, SegSeries ser) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const int sl = seg_lo[r];
  const int t0 = seg_ord(ro, seg_lo, sl);
  const int bs = sl > 0 ? incl[sl - 1] * 256 : 0;  // the stock's first virtual position
  const int base = bs - (t0 & ~255);
  const int v = base + seg_ord(ro, seg_lo, r);
  if (seg_v) {
    omap[v] = r;
    seg_v[v] = base + t0;
  }
  for (int k = 0; k < ser.n; ++k) ser.dst[k][v] = ser.src[k][r];
  // the padding around this row, written by the row before it: the stock's leading positions
  // by its first row, a gap in the ordinals or the tail of the stock's last block by the row
  // before the gap / the last row (no separate fill pass over all Rv positions)
  if (r == sl) seg_pad(bs, v, seg_v, omap, ser);
  const bool last = r + 1 == R || seg_lo[r + 1] != sl;
  seg_pad(v + 1, last ? incl[r] * 256 : base + seg_ord(ro, seg_lo, r + 1), seg_v, omap, ser);
}

}  // namespace

#define MFA_GRID(R) dim3(((R) + 255) / 256), dim3(256)

// ---- direct per-row kernels (the tests' reference kernels; windows beyond the segment kernels'
// limits; CMRA's partial-window variant; the statement-row TTM of a restated panel)
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

// ---- segment-anchored kernels on the segment layout (Rv: virtual rows, a multiple of 256;
// seg_v: virtual stock start of every virtual row; omap: real output row or -1)
MFA_API int mfa_beta_hsigma_seg(const float* y, const float* x, const int* seg_v, const int* omap,
                                int Rv, int W, double lam, int minp, float* beta, float* hsig,
                                void* s) {
  if (Rv <= 0) return 0;
  if (W < 1 || W > 256 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  launch_ew_seg<BetaOp>(y, x, seg_v, omap, Rv, W, lam, minp, beta, hsig, (hipStream_t)s);
  return (int)hipGetLastError();
}
MFA_API int mfa_dastd_seg(const float* ret, const float* mret, const int* seg_v, const int* omap,
                          int Rv, int W, double lam, int minp, float* out, void* s) {
  if (Rv <= 0) return 0;
  if (W < 1 || W > 256 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  launch_ew_seg<DastdOp>(ret, mret, seg_v, omap, Rv, W, lam, minp, out, out, (hipStream_t)s);
  return (int)hipGetLastError();
}
// RSTR: one window, lag L, weights lam^(k - kl), ratio output.  Reach W + L - 1 <= 512.
MFA_API int mfa_rstr_seg(const float* lr, const int* seg_v, const int* omap, int Rv, int L, int W,
                         double lam, int minp, float* out, void* s) {
  if (Rv <= 0) return 0;
  const int reach = W + L - 1;
  if (W < 1 || L < 0 || reach > 512 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  const dim3 grid((Rv + kPosOut - 1) / kPosOut);
  if (reach <= 256)
    hipLaunchKernelGGL((poswin_seg_kernel<256, true, 1>), grid, dim3(256), 0, (hipStream_t)s, lr,
                       seg_v, omap, Rv, L, W, W, W, minp, minp, minp, lam, 1.0, 0, out, out, out);
  else
    hipLaunchKernelGGL((poswin_seg_kernel<512, true, 1>), grid, dim3(256), 0, (hipStream_t)s, lr,
                       seg_v, omap, Rv, L, W, W, W, minp, minp, minp, lam, 1.0, 0, out, out, out);
  return (int)hipGetLastError();
}
// nw (1..3) NaN-skipping window sums of x * scale sharing one pass (STOM / STOQ / STOA);
// log_out: ln(sum), a zero sum -> NaN.  Every W - 1 <= 512.
MFA_API int mfa_window_sums_seg(const float* x, const int* seg_v, const int* omap, int Rv, int nw,
                                const int* W, const int* minp, double scale, int log_out,
                                float* o0, float* o1, float* o2, void* s) {
  if (Rv <= 0) return 0;
  if (nw < 1 || nw > 3 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  int w[3], m[3], reach = 0;
  float* o[3] = {o0, o1, o2};
  for (int k = 0; k < 3; ++k) {
    w[k] = W[k < nw ? k : 0];
    m[k] = minp[k < nw ? k : 0];
    if (w[k] < 1) return (int)hipErrorInvalidValue;
    reach = max(reach, w[k] - 1);
    if (k >= nw) o[k] = o[0];
  }
  if (reach > 512) return (int)hipErrorInvalidValue;
  const dim3 grid((Rv + kPosOut - 1) / kPosOut);
#define MFA_SUMS(H, N)                                                                          \
  hipLaunchKernelGGL((poswin_seg_kernel<H, false, N>), grid, dim3(256), 0, (hipStream_t)s, x,     \
                     seg_v, omap, Rv, 0, w[0], w[1], w[2], m[0], m[1], m[2], 1.0, scale, log_out, \
                     o[0], o[1], o[2])
  if (reach <= 256) {
    if (nw == 3) MFA_SUMS(256, 3); else if (nw == 2) MFA_SUMS(256, 2); else MFA_SUMS(256, 1);
  } else {
    if (nw == 3) MFA_SUMS(512, 3); else if (nw == 2) MFA_SUMS(512, 2); else MFA_SUMS(512, 1);
  }
#undef MFA_SUMS
  return (int)hipGetLastError();
}
// CMRA, full windows only, 64 < W <= 257.
MFA_API int mfa_cmra_seg(const float* lr, const int* seg_v, const int* omap, int Rv, int W,
                         float* out, void* s) {
  if (Rv <= 0) return 0;
  if (W <= 64 || W > 257 || (Rv % 256) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cmra_seg_kernel<256>, dim3((Rv + kPosOut - 1) / kPosOut), dim3(256), 0,
                     (hipStream_t)s, lr, seg_v, omap, Rv, W, out);
  return (int)hipGetLastError();
}

// ---- segment layout construction (see seg_count / seg_place above)
MFA_API int mfa_seg_count(const int* seg_lo, const int* row_ord, int R, int* nb, void* s) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(seg_count_kernel, MFA_GRID(R), 0, (hipStream_t)s, seg_lo, row_ord, R, nb);
  return (int)hipGetLastError();
}
// incl: inclusive prefix sum of mfa_seg_count's nb; Rv = 256 * incl[R - 1]; nser <= 4 series
// src[k] [R] float32 -> dst[k] [Rv] float32 (virtual positions, NaN padding).
MFA_API int mfa_seg_place(const int* seg_lo, const int* row_ord, const int* incl, int R, int Rv,
                          int* seg_v, int* omap, int nser, const float* const* src,
                          float* const* dst, void* s) {
  if (nser < 0 || nser > 4) return (int)hipErrorInvalidValue;
  SegSeries ser{};
  ser.n = nser;
  for (int k = 0; k < nser; ++k) {
    ser.src[k] = src[k];
    ser.dst[k] = dst[k];
  }
  if (R > 0)
    hipLaunchKernelGGL(seg_place_kernel, MFA_GRID(R), 0, (hipStream_t)s, seg_lo, row_ord, incl, R,
                       seg_v, omap, ser);
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
