// Cross-sectional (per-date) reductions for the factor post-processing pipeline (K6, K7, K11).
//
// Reference:
//   winsorize      Barra_factor_cal/post_processing.py:7-24   (clip to mean +- n*std, ddof 1,
//                  NaN-skipping, per date and column)
//   composite      post_processing.py:26-45                   (NaN-renormalised weighted sum)
//   orthogonalize  post_processing.py:47-69                   (per-date OLS residual on [1, X])
//   NLSIZE         factor_calculator.py:237-293               (-residual of SIZE^3 on [1, SIZE])
//   z-score        Barra-master/mfm/CrossSection.py:12-20     (cap-weighted mean, pooled std)
//   bayes_shrink   Barra-master/mfm/utils.py:133-168          (cap-decile Bayesian shrinkage)
//
// Layout: field panels are [F][D][N] fp32 (each (field, date) row contiguous).  One workgroup
// per (field, date) row or per date; fp64 accumulation; deterministic (no float atomics).
#include "common.h"

namespace {

using namespace mfa;

__device__ __forceinline__ bool fin(float v) { return __builtin_isfinite(v); }

// ---- K6: winsorize rows of x [R][N] in place (R = F_sel * D row pointers given by row index)
__global__ __launch_bounds__(256) void winsorize_kernel(float* __restrict__ x, int N, double nstd) {
  __shared__ double scratch[16];
  float* r = x + (size_t)blockIdx.x * N;
  double s = 0.0, c = 0.0;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float v = r[n];
    if (!isnan(v)) { s += v; c += 1.0; }
  }
  s = block_sum(s, scratch);
  c = block_sum(c, scratch);
  const double mean = s / c;
  double ss = 0.0;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float v = r[n];
    if (!isnan(v)) { const double dv = v - mean; ss = fma(dv, dv, ss); }
  }
  ss = block_sum(ss, scratch);
  if (!(c >= 2.0)) return;  // pandas: std NaN -> clip bounds NaN -> no clipping
  const double sd = sqrt(ss / (c - 1.0));
  const double lo = mean - nstd * sd, hi = mean + nstd * sd;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float v = r[n];
    if (!isnan(v)) {
      const double dv = v;
      r[n] = (float)(dv < lo ? lo : (dv > hi ? hi : dv));
    }
  }
}

// ---- composite: out[i] = sum_c w_c x_c[i] (NaN->0) / sum_c w_c notna(x_c[i])   (C <= 8)
struct CompArgs {
  const float* x[8];
  double w[8];
  int C;
};
__global__ __launch_bounds__(256) void composite_kernel(CompArgs a, size_t n, float* __restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double num = 0.0, den = 0.0;
    for (int c = 0; c < a.C; ++c) {
      const float v = a.x[c][i];
      if (!isnan(v)) { num = fma(a.w[c], (double)v, num); den += a.w[c]; }
    }
    out[i] = den != 0.0 ? (float)(num / den) : qnanf();
  }
}

// ---- K7: per-date OLS residual of y on [1, x_1..x_p] (p <= 4), rows with all values finite.
// y [D][N]; X = p pointers to [D][N]; out [D][N] (NaN on excluded rows / dates with < min_rows).
struct OlsArgs {
  const float* x[4];
  int p;
  int log_x0;  // x_1 := ln(x_1) in fp64 (NLSIZE regresses on ln(total_mv))
  int ypow;    // > 0: y := x_1^ypow in fp64 (NLSIZE: SIZE^3), y pointer ignored
};
__global__ __launch_bounds__(256) void ols_resid_kernel(const float* __restrict__ y, OlsArgs a, int N,
                                                        int min_rows, double sign,
                                                        float* __restrict__ out) {
  __shared__ double scratch[16];
  __shared__ double G[5][6];
  const int d = blockIdx.x, p = a.p, m = p + 1;
  const float* yd = y ? y + (size_t)d * N : nullptr;
  double acc[21];  // packed upper Gram (15) + X^T y (5) + count
#pragma unroll
  for (int i = 0; i < 21; ++i) acc[i] = 0.0;
  auto load_row = [&](int n, double (&z)[5], double& yv) -> bool {
    z[0] = 1.0;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < p) {
        const float v = a.x[k][(size_t)d * N + n];
        ok = ok && fin(v);
        z[k + 1] = (k == 0 && a.log_x0) ? log((double)v) : (double)v;
      } else {
        z[k + 1] = 0.0;
      }
    }
    if (a.ypow > 0) {
      yv = z[1];
      for (int e = 1; e < a.ypow; ++e) yv *= z[1];
    } else {
      ok = ok && fin(yd[n]);
      yv = yd[n];
    }
    return ok && __builtin_isfinite(yv) && __builtin_isfinite(z[1]);
  };
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    double z[5], yv;
    if (!load_row(n, z, yv)) continue;
    int idx = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = i; j < 5; ++j) acc[idx++] += z[i] * z[j];
#pragma unroll
    for (int i = 0; i < 5; ++i) acc[15 + i] = fma(z[i], yv, acc[15 + i]);
    acc[20] += 1.0;
  }
#pragma unroll
  for (int i = 0; i < 21; ++i) acc[i] = block_sum(acc[i], scratch);
  const bool enough = acc[20] >= (double)min_rows;
  if (threadIdx.x == 0) {
    int idx = 0;
    for (int i = 0; i < 5; ++i)
      for (int j = i; j < 5; ++j) { G[i][j] = acc[idx]; G[j][i] = acc[idx]; ++idx; }
    for (int i = 0; i < 5; ++i) G[i][5] = acc[15 + i];
    // Gauss-Jordan with partial pivoting on the m x m system (pinv semantics for exact zeros)
    for (int c = 0; c < m; ++c) {
      int piv = c;
      for (int r = c + 1; r < m; ++r)
        if (fabs(G[r][c]) > fabs(G[piv][c])) piv = r;
      if (piv != c)
        for (int k = 0; k <= 5; ++k) { const double t = G[c][k]; G[c][k] = G[piv][k]; G[piv][k] = t; }
      const double pv = G[c][c];
      if (fabs(pv) < 1e-300) { for (int k = 0; k <= 5; ++k) G[c][k] = 0.0; continue; }
      for (int k = 0; k <= 5; ++k) G[c][k] /= pv;
      for (int r = 0; r < m; ++r) {
        if (r == c) continue;
        const double f = G[r][c];
        for (int k = 0; k <= 5; ++k) G[r][k] -= f * G[c][k];
      }
    }
  }
  __syncthreads();
  double b[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) b[i] = i < m ? G[i][5] : 0.0;
  float* od = out + (size_t)d * N;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    double z[5], yv;
    const bool ok = load_row(n, z, yv) && enough;
    double e = yv - b[0];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < p) e -= b[k + 1] * z[k + 1];
    od[n] = ok ? (float)(sign * e) : qnanf();
  }
}

// ---- z-score exactly as CrossSection.style_factor_norm: (x - capweighted mean_q) / pooled std.
// X [D][Q][N] in place; rows invalid when any of x_q / cap non-finite.
__global__ __launch_bounds__(256) void style_norm_kernel(float* __restrict__ X, const float* __restrict__ cap,
                                                         int Q, int N, double* __restrict__ mu_out,
                                                         double* __restrict__ sig_out) {
  __shared__ double scratch[16];
  __shared__ double mus[64];
  const int d = blockIdx.x;
  float* Xd = X + (size_t)d * Q * N;
  const float* cd = cap + (size_t)d * N;
  double sc = 0.0, sx = 0.0, sxx = 0.0, cnt = 0.0;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    bool ok = fin(cd[n]);
    for (int q = 0; q < Q; ++q) ok = ok && fin(Xd[(size_t)q * N + n]);
    if (!ok) continue;
    sc += cd[n];
    cnt += 1.0;
    for (int q = 0; q < Q; ++q) {
      const double v = Xd[(size_t)q * N + n];
      sx += v;
      sxx = fma(v, v, sxx);
    }
  }
  sc = block_sum(sc, scratch);
  sx = block_sum(sx, scratch);
  sxx = block_sum(sxx, scratch);
  cnt = block_sum(cnt, scratch);
  for (int q = 0; q < Q; ++q) {
    double scx = 0.0;
    for (int n = threadIdx.x; n < N; n += blockDim.x) {
      bool ok = fin(cd[n]);
      for (int k = 0; k < Q; ++k) ok = ok && fin(Xd[(size_t)k * N + n]);
      if (ok) scx = fma((double)cd[n], (double)Xd[(size_t)q * N + n], scx);
    }
    scx = block_sum(scx, scratch);
    if (threadIdx.x == 0) mus[q] = scx / sc;
  }
  __syncthreads();
  const double nq = cnt * Q, m = sx / nq;
  const double sig = sqrt(fmax(sxx / nq - m * m, 0.0));
  if (threadIdx.x == 0 && sig_out) sig_out[d] = sig;
  if (mu_out)
    for (int q = threadIdx.x; q < Q; q += blockDim.x) mu_out[(size_t)d * Q + q] = mus[q];
  for (int n = threadIdx.x; n < N; n += blockDim.x)
    for (int q = 0; q < Q; ++q) {
      const float v = Xd[(size_t)q * N + n];
      Xd[(size_t)q * N + n] = (float)((v - mus[q]) / sig);
    }
}

// ---- K11: cap-decile Bayesian shrinkage, one workgroup per date (N <= 8192).
// groups: pd.qcut(cap, G).codes (linear-interpolated quantile edges, right-closed bins, the
// first bin includes the minimum); per group m = sum(vol*cap)/sum(cap), s = sqrt(mean((vol-m)^2));
// out = v*m + (1-v)*|vol| with v = q|vol-m| / (q|vol-m| + s).
// presorted != nullptr (wide universes, N > kBayesLdsN): the caller sorted each date's masked
// caps (+inf = invalid) on the device and the edges are read from there instead of the LDS sort.
__global__ __launch_bounds__(1024) void bayes_shrink_kernel(const float* __restrict__ vol,
                                                            const float* __restrict__ cap, int N,
                                                            int G, double qq, float* __restrict__ out,
                                                            int* __restrict__ group_out,
                                                            const float* __restrict__ presorted) {
  extern __shared__ float lkeys[];  // [NP] sorted caps
  __shared__ double gs[64][4];
  const int d = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const float* vd = vol + (size_t)d * N;
  const float* cd = cap + (size_t)d * N;
  const float* keys = presorted ? presorted + (size_t)d * N : lkeys;
  int nvalid = 0;
  for (int g = tid; g < G * 4; g += nt) gs[g / 4][g % 4] = 0.0;
  if (!presorted) {
    int NP = 1;
    while (NP < N) NP <<= 1;
    for (int i = tid; i < NP; i += nt) {
      const bool ok = i < N && fin(cd[i]) && fin(vd[i]);
      lkeys[i] = ok ? cd[i] : __builtin_inff();
    }
    __syncthreads();
    // bitonic sort ascending
    for (int k = 2; k <= NP; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < NP; i += nt) {
          const int ij = i ^ j;
          if (ij > i) {
            const bool up = (i & k) == 0;
            const float a = lkeys[i], b = lkeys[ij];
            if ((a > b) == up) { lkeys[i] = b; lkeys[ij] = a; }
          }
        }
        __syncthreads();
      }
  }
  __syncthreads();
  {
    int c = 0;
    for (int i = tid; i < N; i += nt) c += fin(keys[i]) ? 1 : 0;
    __shared__ int cs[32];
    c = wave_sum(c);
    if ((tid & 63) == 0) cs[tid >> 6] = c;
    __syncthreads();
    nvalid = 0;
    for (int w = 0; w < (nt + 63) / 64; ++w) nvalid += cs[w];
  }
  // quantile edges (numpy 'linear'): e_g = sorted[(n-1) g / G] interpolated
  auto edge = [&](int g) -> double {
    const double pos = (double)(nvalid - 1) * g / G;
    const int lo = (int)floor(pos);
    const int hi = min(lo + 1, nvalid - 1);
    const double fr = pos - lo;
    return (double)keys[lo] + ((double)keys[hi] - (double)keys[lo]) * fr;
  };
  int* grp = group_out ? group_out + (size_t)d * N : nullptr;
  for (int i = tid; i < N; i += nt) {
    int g = -1;
    if (fin(cd[i]) && fin(vd[i])) {
      const double c = cd[i];
      g = 0;
      for (int k = 1; k < G; ++k)
        if (c > edge(k)) g = k;
      atomicAdd(&gs[g][0], (double)vd[i] * c);
      atomicAdd(&gs[g][1], c);
    }
    if (grp) grp[i] = g;
  }
  __syncthreads();
  for (int i = tid; i < N; i += nt) {
    if (!(fin(cd[i]) && fin(vd[i]))) continue;
    const double c = cd[i];
    int g = 0;
    for (int k = 1; k < G; ++k)
      if (c > edge(k)) g = k;
    const double mg = gs[g][0] / gs[g][1];
    const double dv = (double)vd[i] - mg;
    atomicAdd(&gs[g][2], dv * dv);
    atomicAdd(&gs[g][3], 1.0);
  }
  __syncthreads();
  for (int i = tid; i < N; i += nt) {
    float o = qnanf();
    if (fin(cd[i]) && fin(vd[i])) {
      const double c = cd[i];
      int g = 0;
      for (int k = 1; k < G; ++k)
        if (c > edge(k)) g = k;
      const double mg = gs[g][0] / gs[g][1];
      const double sg = sqrt(gs[g][2] / gs[g][3]);
      const double a = qq * fabs((double)vd[i] - mg);
      const double v = a / (a + sg);
      o = (float)(v * mg + (1.0 - v) * fabs((double)vd[i]));
    }
    out[(size_t)d * N + i] = o;
  }
}

}  // namespace

MFA_API int mfa_winsorize(float* x, int rows, int N, double nstd, void* stream) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(winsorize_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, x, N, nstd);
  return (int)hipGetLastError();
}

MFA_API int mfa_composite(const float* const* xs, const double* w, int C, size_t n, float* out,
                          void* stream) {
  if (C < 1 || C > 8) return (int)hipErrorInvalidValue;
  CompArgs a;
  for (int c = 0; c < 8; ++c) { a.x[c] = c < C ? xs[c] : nullptr; a.w[c] = c < C ? w[c] : 0.0; }
  a.C = C;
  const int grid = (int)min((size_t)4096, (n + 255) / 256);
  hipLaunchKernelGGL(composite_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, (hipStream_t)stream, a, n, out);
  return (int)hipGetLastError();
}

MFA_API int mfa_ols_resid(const float* y, const float* const* xs, int p, int D, int N, int min_rows,
                          double sign, int log_x0, int ypow, float* out, void* stream) {
  if (D <= 0) return 0;
  if (p < 0 || p > 4 || (ypow > 0 && p < 1) || (ypow <= 0 && y == nullptr)) return (int)hipErrorInvalidValue;
  OlsArgs a;
  for (int k = 0; k < 4; ++k) a.x[k] = k < p ? xs[k] : nullptr;
  a.p = p;
  a.log_x0 = log_x0;
  a.ypow = ypow;
  hipLaunchKernelGGL(ols_resid_kernel, dim3(D), dim3(256), 0, (hipStream_t)stream, y, a, N, min_rows,
                     sign, out);
  return (int)hipGetLastError();
}

MFA_API int mfa_style_norm(float* X, const float* cap, int D, int Q, int N, double* mu, double* sig,
                           void* stream) {
  if (D <= 0) return 0;
  if (Q > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(style_norm_kernel, dim3(D), dim3(256), 0, (hipStream_t)stream, X, cap, Q, N, mu, sig);
  return (int)hipGetLastError();
}

MFA_API int mfa_bayes_shrink(const float* vol, const float* cap, int D, int N, int G, double q,
                             float* out, int* groups, void* stream) {
  if (D <= 0) return 0;
  if (N > 16384 || G < 1 || G > 64) return (int)hipErrorInvalidValue;
  int NP = 1;
  while (NP < N) NP <<= 1;
  hipLaunchKernelGGL(bayes_shrink_kernel, dim3(D), dim3(1024), NP * sizeof(float), (hipStream_t)stream,
                     vol, cap, N, G, q, out, groups, (const float*)nullptr);
  return (int)hipGetLastError();
}

// Any N: `sorted` [D][N] = each date's caps with invalid (vol, cap) pairs set to +inf, sorted
// ascending (the caller's device sort); the kernel takes the decile edges from it.
MFA_API int mfa_bayes_shrink_presorted(const float* vol, const float* cap, const float* sorted,
                                       int D, int N, int G, double q, float* out, int* groups,
                                       void* stream) {
  if (D <= 0) return 0;
  if (N <= 0 || G < 1 || G > 64 || sorted == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bayes_shrink_kernel, dim3(D), dim3(1024), 0, (hipStream_t)stream, vol, cap,
                     N, G, q, out, groups, sorted);
  return (int)hipGetLastError();
}
