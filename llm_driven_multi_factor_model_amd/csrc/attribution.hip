// Portfolio factor exposures for risk attribution, all dates per launch (gfx950).
//
// For a portfolio h_d (weights over the panel's stocks) the exposure to the K = 1 + P + Q factors
// of CrossSection.reg's design matrix (Barra-master/mfm/CrossSection.py:48,74: country column,
// one-hot industries, cap-weighted z-scored styles, :12-20) is
//   x_country = sum_i h_i,   x_ind[j] = sum_{i in j} h_i,   x_style[q] = sum_i h_i z_iq,
//   z_iq = (X_iq - mu_q) / sigma   =>   x_style[q] = (sum_i h_i X_iq - mu_q sum_i h_i) / sigma,
// so the raw panel is read once and never z-scored in memory.  Stocks that are absent or have
// non-finite inputs (the regression's validity rule) contribute nothing.
//
// One 256-thread workgroup per date: fp64 register accumulators for the Q + 1 dense sums, LDS
// atomics for the industry sums (dynamic LDS), a fixed-order workgroup reduction; style sets
// wider than 16 run in blocks of 16 styles.
#include "common.h"

namespace {

using namespace mfa;

// QB styles per launch (template), starting at style q0 of Q; the validity rule still checks all
// Q styles.  The launch with q0 == 0 also writes the country and industry exposures.  Industry
// sums live in dynamic LDS (P doubles), so any P fits (64 K industries = 512 KB would not; the
// host caps P at 8192).
template <int QB, typename T>
__global__ __launch_bounds__(256) void portfolio_exposure_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, const double* __restrict__ h, const double* __restrict__ stats,
    int N, int P, int Q, int q0, int K, double* __restrict__ out) {
  extern __shared__ double segs[];
  __shared__ double red[4][QB + 1];
  const int d = blockIdx.x, tid = threadIdx.x;
  const int Pseg = P > 0 ? P : 1;
  const bool lead = q0 == 0;
  if (lead)
    for (int j = tid; j < Pseg; j += blockDim.x) segs[j] = 0.0;
  __syncthreads();
  const T* Xd = X + (size_t)d * Q * N;
  const T* cd = cap + (size_t)d * N;
  const T* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;
  const double* hd = h + (size_t)d * N;
  double acc[QB + 1];
#pragma unroll
  for (int q = 0; q <= QB; ++q) acc[q] = 0.0;
  for (int n = tid; n < N; n += blockDim.x) {
    const T c = cd[n], r = rd[n];
    const int j = id ? (int)id[n] : 0;
    const double w = hd[n];
    bool ok = (j >= 0) && (j < Pseg) && __builtin_isfinite(c) && (c >= T(0)) &&
              __builtin_isfinite(r) && __builtin_isfinite(w);
    T xf[QB];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      xf[q] = q0 + q < Q ? Xd[(size_t)(q0 + q) * N + n] : T(0);
      ok = ok && __builtin_isfinite(xf[q]);
    }
    if (Q > QB)  // styles outside this launch's block still decide validity
      for (int q = 0; q < Q; ++q)
        if (q < q0 || q >= q0 + QB) ok = ok && __builtin_isfinite(Xd[(size_t)q * N + n]);
    if (!ok || w == 0.0) continue;
    acc[QB] += w;
#pragma unroll
    for (int q = 0; q < QB; ++q) acc[q] = fma(w, (double)xf[q], acc[q]);
    if (P > 0 && lead) atomicAdd(&segs[j], w);
  }
  const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int q = 0; q <= QB; ++q) {
    const double v = wave_sum(acc[q]);
    if (lane == 0) red[wid][q] = v;
  }
  __syncthreads();
  double* o = out + (size_t)d * K;
  const double* st = stats + (size_t)d * (Q + 2);
  if (tid <= QB) {
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w][tid];
    red[0][tid] = s;  // each entry is read back only by its own thread below
  }
  __syncthreads();
  const double hs = red[0][QB];
  const double isig = 1.0 / st[Q];
  if (lead) {
    if (tid == 0) o[0] = hs;
    for (int j = tid; j < P; j += blockDim.x) o[1 + j] = segs[j];
  }
  if (tid < QB && q0 + tid < Q) o[1 + P + q0 + tid] = (red[0][tid] - st[q0 + tid] * hs) * isig;
}

template <typename T>
int portfolio_exposure_dispatch(const T* X, const T* cap, const T* ret, const int16_t* ind,
                                const double* h, const double* stats, int D, int N, int P, int Q,
                                double* out, void* stream) {
  if (D <= 0) return 0;
  if (Q < 1 || P < 0 || P > 8192 || N <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int K = 1 + P + Q;
  const size_t lds = (size_t)(P > 0 ? P : 1) * sizeof(double);
  if (Q > 16) {  // wide style sets: blocks of 16 styles, one launch each (the first adds the
                 // country / industry sums)
    for (int q0 = 0; q0 < Q; q0 += 16)
      hipLaunchKernelGGL((portfolio_exposure_kernel<16, T>), dim3(D), dim3(256), lds, s, X, cap,
                         ret, P > 0 ? ind : nullptr, h, stats, N, P, Q, q0, K, out);
    return (int)hipGetLastError();
  }
  switch (Q) {
#define MFA_Q(qq)                                                                              \
  case qq:                                                                                     \
    hipLaunchKernelGGL((portfolio_exposure_kernel<qq, T>), dim3(D), dim3(256), lds, s, X, cap, \
                       ret, P > 0 ? ind : nullptr, h, stats, N, P, Q, 0, K, out);              \
    break;
    MFA_Q(1) MFA_Q(2) MFA_Q(3) MFA_Q(4) MFA_Q(5) MFA_Q(6) MFA_Q(7) MFA_Q(8)
    MFA_Q(9) MFA_Q(10) MFA_Q(11) MFA_Q(12) MFA_Q(13) MFA_Q(14) MFA_Q(15) MFA_Q(16)
#undef MFA_Q
  }
  return (int)hipGetLastError();
}

// Point-in-time trailing specific volatility (RiskModel.specific_vol_series): for every stock
// n and local date t, the ddof-0 std of the finite values among the W rows ENDING at t of
// ext = [halo (h rows) ; e (D rows)], summed NEWEST FIRST with one rounding per operation
// (count += ok, s1 += x, s2 += fl(x * x); mean = s1 / n, var = fl(s2 / n) - fl(mean * mean)),
// i.e. bitwise the order of the tensor loop it replaces (risk_model.py) -- and so bitwise
// rank-invariant, the property that loop was written for.  One thread per (stock, TD-date
// tile): the tile's TD + W - 1 rows are walked newest to oldest in blocks of 16, the next block's
// loads issued before the current block is summed (the loads are the latency); each row is
// added to the outputs whose window holds it and +0.0 to the others (exact: the sums are never
// -0.0).  Stocks are the contiguous axis, so every load of a wave is one 512-byte row segment.
// The tensor loop moved 3 x W full [D, N] temporaries (~50 ms at 2520 x 5000).
template <int TD>
__global__ __launch_bounds__(256) void trailing_vol_kernel(const double* __restrict__ halo, int h,
                                                           const double* __restrict__ e, int D,
                                                           int N, int W, int minp,
                                                           double* __restrict__ vol) {
  // one rounding per operation, as the tensor loop: the library builds with
  // -ffp-contract=fast (which ignores `#pragma clang fp contract`), and HIP's __dadd_rn /
  // __dmul_rn are plain + / * that it would fuse -- an empty asm on each product blocks that
  constexpr int RB = 16;  // rows per block
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int t0 = blockIdx.y * TD;
  const int nt = D - t0 < TD ? D - t0 : TD;
  auto ld = [&](int i) -> double {  // ext row i (0 outside; such rows are never active)
    if (i < 0 || i >= h + D) return 0.0;
    return i < h ? halo[(size_t)i * N + n] : e[(size_t)(i - h) * N + n];
  };
  double c[TD], s1[TD], s2[TD];
#pragma unroll
  for (int k = 0; k < TD; ++k) {
    c[k] = 0.0;
    s1[k] = 0.0;
    s2[k] = 0.0;
  }
  // row offset o = row - (t0 + h): output k holds it iff k - W < o <= k; rows o = TD-1 .. -(W-1)
  const int o_hi = TD - 1, nrows = TD + W - 1;
  const int nblk = (nrows + RB - 1) / RB;
  double xb[RB], nb[RB];
#pragma unroll
  for (int u = 0; u < RB; ++u) xb[u] = ld(t0 + h + o_hi - u);
  for (int b = 0; b < nblk; ++b) {
    const int ob = o_hi - b * RB;  // offset of the block's first (newest) row
#pragma unroll
    for (int u = 0; u < RB; ++u) nb[u] = b + 1 < nblk ? ld(t0 + h + ob - RB - u) : 0.0;
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int o = ob - u;
      const double x = xb[u];
      const bool fin = __builtin_isfinite(x);
      const double xz = fin ? x : 0.0;
      double sq = __dmul_rn(xz, xz);
      asm volatile("" : "+v"(sq));
#pragma unroll
      for (int k = 0; k < TD; ++k) {
        const bool act = (k >= o) && (k - W < o) && (o > -W);
        c[k] = __dadd_rn(c[k], act && fin ? 1.0 : 0.0);
        s1[k] = __dadd_rn(s1[k], act ? xz : 0.0);
        s2[k] = __dadd_rn(s2[k], act ? sq : 0.0);
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) xb[u] = nb[u];
  }
  const double thr = minp > 1 ? (double)minp : 1.0;
#pragma unroll
  for (int k = 0; k < TD; ++k) {
    if (k < nt) {
      const double mean = __ddiv_rn(s1[k], c[k]);
      double m2 = __dmul_rn(mean, mean);
      asm volatile("" : "+v"(m2));
      const double var = __dsub_rn(__ddiv_rn(s2[k], c[k]), m2);
      const double v = __dsqrt_rn(var > 0.0 ? var : 0.0);
      vol[(size_t)(t0 + k) * N + n] = c[k] >= thr ? v : qnan();
    }
  }
}

}  // namespace

// X [D][Q][N] f32, cap/ret [D][N] f32 (validity only), ind [D][N] int16 (nullable when P == 0),
// h [D][N] f64 portfolio weights, stats [D][Q+2] f64 = (mu_q, sigma, n) from mfa_xs_wls.
// out [D][1+P+Q] f64.
MFA_API int mfa_portfolio_exposure(const float* X, const float* cap, const float* ret,
                                   const int16_t* ind, const double* h, const double* stats, int D,
                                   int N, int P, int Q, double* out, void* stream) {
  return portfolio_exposure_dispatch<float>(X, cap, ret, ind, h, stats, D, N, P, Q, out, stream);
}

// Same with an fp64 panel.
MFA_API int mfa_portfolio_exposure_f64(const double* X, const double* cap, const double* ret,
                                       const int16_t* ind, const double* h, const double* stats,
                                       int D, int N, int P, int Q, double* out, void* stream) {
  return portfolio_exposure_dispatch<double>(X, cap, ret, ind, h, stats, D, N, P, Q, out, stream);
}

// vol [D][N] = trailing point-in-time specific volatility of e [D][N] over W rows ending at each
// date, with halo [h][N] (h = W - 1 rows preceding e; NaN where none).  Bitwise equal to the
// newest-first tensor loop of RiskModel.specific_vol_series.
MFA_API int mfa_trailing_vol(const double* halo, int h, const double* e, int D, int N, int W,
                             int min_periods, double* vol, void* stream) {
  if (D <= 0 || N <= 0) return 0;
  if (W < 1 || h < 0 || (h > 0 && !halo)) return (int)hipErrorInvalidValue;
  constexpr int TD = 16;
  hipLaunchKernelGGL(trailing_vol_kernel<TD>, dim3((N + 255) / 256, (D + TD - 1) / TD), dim3(256),
                     0, (hipStream_t)stream, halo, h, e, D, N, W, min_periods, vol);
  return (int)hipGetLastError();
}
