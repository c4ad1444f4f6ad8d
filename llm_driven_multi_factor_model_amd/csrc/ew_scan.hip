// Expanding-window exponentially-weighted Newey-West covariance series as a blocked scan (K8),
// plus the decayed prefix mean used by the volatility-regime adjustment (K10).
//
// Reference: Barra-master/mfm/utils.py:16-50 (Newey_West on one prefix) called for EVERY
// prefix f[:t], t = 1..T, by MFM.Newey_West_by_time (MFM.py:80-101): O(T^2 K^2) Python.
//
// Here every prefix is produced in O(T K^2) from decayed moments (lambda = 0.5^(1/tau)):
//   Z   = sum_u l^(n-1-u)              m  = sum_u l^(n-1-u) f_u       S0 = sum_u l^(n-1-u) f_u f_u^T
//   A_i = sum_{u>=i} l^(n-1-u) f_{u-i} f_u^T   a_i = sum_{u>=i} l^(n-1-u) f_{u-i}
//   b_i = sum_{u>=i} l^(n-1-u) f_u             z_i = sum_{u>=i} l^(n-1-u)
//   mu = m/Z,  G0 = S0/Z - mu mu^T,  Gi = (A_i - a_i mu^T - mu b_i^T + z_i mu mu^T)/Z
//   V  = G0 + sum_i (1 - i/(q+1)) (Gi + Gi^T)
// Work decomposition: thread = one (k,l) output entry, which carries its own scalar copy of
// every moment it needs (18 fp64 at q = 2); dates are cut into chunks of CH rows:
//   pass A  chunk-local decayed sums      grid (chunks, ceil(K^2/256))
//   pass B  exclusive scan of chunk carries (sequential over chunks, parallel over moments)
//   pass C  re-scan each chunk from its carry and write V_t      grid (out chunks, ...)
// The output range [t_lo, t_hi) lets each data-parallel rank emit only its own date shard.
#include "common.h"

namespace {

using namespace mfa;

constexpr int CH = 32;        // dates per chunk
constexpr int MAXQ = 4;       // max Newey-West lag
constexpr int NSTATE = 2 + 7 * MAXQ + 4;  // per-thread moment count (upper bound)

// state layout per thread (k,l):
//   0 Z | 1 S0 | 2 mk | 3 ml | then per lag i (0-based ii): A_kl, A_lk, a_k, a_l, b_k, b_l, z
struct NwDims {
  int T, K, q;
  double lam;
};

__device__ __forceinline__ int st_idx(int ii, int w) { return 4 + ii * 7 + w; }

template <bool STAGE_OUT>
__device__ void nw_run_chunk(const double* __restrict__ Fs,  // LDS rows [t0-q, t1)
                             int t0, int t1, int k, int l, const NwDims& dm, double* s,
                             double* __restrict__ V, int t_lo, int t_hi, int qoff) {
  const int K = dm.K, q = dm.q;
  const double lam = dm.lam;
  for (int u = t0; u < t1; ++u) {
    const double* fu = Fs + (size_t)(u - t0 + qoff) * K;
    const double fk = fu[k], fl = fu[l];
    s[0] = fma(lam, s[0], 1.0);
    s[1] = fma(lam, s[1], fk * fl);
    s[2] = fma(lam, s[2], fk);
    s[3] = fma(lam, s[3], fl);
#pragma unroll
    for (int ii = 0; ii < MAXQ; ++ii) {
      if (ii >= q) break;
      const int i = ii + 1;
      double* si = s + st_idx(ii, 0);
      const bool has = u >= i;
      const double gk = has ? Fs[(size_t)(u - i - t0 + qoff) * K + k] : 0.0;
      const double gl = has ? Fs[(size_t)(u - i - t0 + qoff) * K + l] : 0.0;
      si[0] = fma(lam, si[0], gk * fl);
      si[1] = fma(lam, si[1], gl * fk);
      si[2] = fma(lam, si[2], gk);
      si[3] = fma(lam, si[3], gl);
      si[4] = fma(lam, si[4], has ? fk : 0.0);
      si[5] = fma(lam, si[5], has ? fl : 0.0);
      si[6] = fma(lam, si[6], has ? 1.0 : 0.0);
    }
    if (STAGE_OUT && u >= t_lo && u < t_hi) {
      const int n = u + 1;  // prefix length
      double v;
      if (n <= q || n <= K) {
        v = qnan();
      } else {
        const double iz = 1.0 / s[0];
        const double mk = s[2] * iz, ml = s[3] * iz;
        v = s[1] * iz - mk * ml;
#pragma unroll
        for (int ii = 0; ii < MAXQ; ++ii) {
          if (ii >= q) break;
          const int i = ii + 1;
          const double* si = s + st_idx(ii, 0);
          // G_i[k][l] + G_i[l][k]
          const double gkl = si[0] - si[2] * ml - mk * si[5] + si[6] * mk * ml;
          const double glk = si[1] - si[3] * mk - ml * si[4] + si[6] * ml * mk;
          v = fma(1.0 - (double)i / (q + 1), (gkl + glk) * iz, v);
        }
      }
      V[(size_t)(u - t_lo) * K * K + (size_t)k * K + l] = v;
    }
  }
}

__device__ void stage_rows(const double* __restrict__ F, double* Fs, int t0, int t1, int q, int K) {
  const int lo = t0 - q;
  const int rows = t1 - lo;
  for (int e = threadIdx.x; e < rows * K; e += blockDim.x) {
    const int r = e / K, c = e % K;
    const int t = lo + r;
    Fs[e] = t >= 0 ? F[(size_t)t * K + c] : 0.0;
  }
}

// pass A: chunk-local sums.  C[chunk][m][kk] (m = moment index, kk = k*K+l)
__global__ __launch_bounds__(256) void nw_chunk_sums(const double* __restrict__ F, NwDims dm,
                                                     int nchunks, double* __restrict__ C) {
  extern __shared__ double Fs[];
  const int c = blockIdx.x;
  const int t0 = c * CH, t1 = min(dm.T, t0 + CH);
  stage_rows(F, Fs, t0, t1, dm.q, dm.K);
  __syncthreads();
  const int KK = dm.K * dm.K;
  const int kk = blockIdx.y * blockDim.x + threadIdx.x;
  if (kk >= KK) return;
  double s[NSTATE];
#pragma unroll
  for (int i = 0; i < NSTATE; ++i) s[i] = 0.0;
  nw_run_chunk<false>(Fs, t0, t1, kk / dm.K, kk % dm.K, dm, s, nullptr, 0, 0, dm.q);
  const int ns = 4 + 7 * dm.q;
#pragma unroll
  for (int m = 0; m < NSTATE; ++m)
    if (m < ns) C[((size_t)c * ns + m) * KK + kk] = s[m];
}

// pass B: in-place exclusive scan over chunks: C[c] <- sum_{c'<c} l^(t0_c - t1_c') C[c']
__global__ __launch_bounds__(256) void nw_carry_scan(NwDims dm, int nchunks, double* __restrict__ C) {
  const int KK = dm.K * dm.K;
  const int ns = 4 + 7 * dm.q;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (m, kk)
  if (e >= ns * KK) return;
  double carry = 0.0;
  for (int c = 0; c < nchunks; ++c) {
    const int len = min(dm.T, (c + 1) * CH) - c * CH;
    double* p = C + (size_t)c * ns * KK + e;
    const double loc = *p;
    *p = carry;
    carry = fma(pow(dm.lam, (double)len), carry, loc);
  }
}

// pass C: outputs for chunks overlapping [t_lo, t_hi)
__global__ __launch_bounds__(256) void nw_emit(const double* __restrict__ F, NwDims dm,
                                               const double* __restrict__ C, int c_first,
                                               int t_lo, int t_hi, double* __restrict__ V) {
  extern __shared__ double Fs[];
  const int c = c_first + blockIdx.x;
  const int t0 = c * CH, t1 = min(dm.T, t0 + CH);
  stage_rows(F, Fs, t0, t1, dm.q, dm.K);
  __syncthreads();
  const int KK = dm.K * dm.K;
  const int kk = blockIdx.y * blockDim.x + threadIdx.x;
  if (kk >= KK) return;
  const int ns = 4 + 7 * dm.q;
  double s[NSTATE];
#pragma unroll
  for (int m = 0; m < NSTATE; ++m) s[m] = m < ns ? C[((size_t)c * ns + m) * KK + kk] : 0.0;
  nw_run_chunk<true>(Fs, t0, t1, kk / dm.K, kk % dm.K, dm, s, V, t_lo, t_hi, dm.q);
}

// Decayed prefix mean with validity: out[t] = sum_{s<=t, ok} l^(t-s) x_s / sum_{s<=t, ok} l^(t-s)
// (VRA factor-volatility multiplier, MFM.py:149-160).  One wave; chunked two-level scan.
__global__ __launch_bounds__(64) void ew_prefix_mean(const double* __restrict__ x, int T, double lam,
                                                     double* __restrict__ out) {
  const int lane = threadIdx.x;
  const int per = (T + 63) / 64;
  const int a = lane * per, b = min(T, a + per);
  double num = 0.0, den = 0.0;
  for (int t = a; t < b; ++t) {
    const double v = x[t];
    const bool ok = __builtin_isfinite(v);
    num = fma(lam, num, ok ? v : 0.0);
    den = fma(lam, den, ok ? 1.0 : 0.0);
  }
  // exclusive scan of (num, den) carries across lanes: carry_l = sum_{l'<l} lam^(len after) ...
  const double dec = pow(lam, (double)(b > a ? b - a : 0));
  double cn = num, cd = den, dk = dec;  // inclusive combine (decay-weighted)
  for (int off = 1; off < 64; off <<= 1) {
    const double pn = __shfl_up(cn, off, 64), pd = __shfl_up(cd, off, 64), pk = __shfl_up(dk, off, 64);
    if (lane >= off) {
      cn = fma(pn, dk, cn);
      cd = fma(pd, dk, cd);
      dk = dk * pk;
    }
  }
  double en = __shfl_up(cn, 1, 64), ed = __shfl_up(cd, 1, 64);
  if (lane == 0) { en = 0.0; ed = 0.0; }
  num = en; den = ed;
  for (int t = a; t < b; ++t) {
    const double v = x[t];
    const bool ok = __builtin_isfinite(v);
    num = fma(lam, num, ok ? v : 0.0);
    den = fma(lam, den, ok ? 1.0 : 0.0);
    out[t] = den > 0.0 ? num / den : qnan();
  }
}

}  // namespace

// F: [T][K] fp64 factor-return series (global calendar, all dates up to t_hi).
// V: [t_hi - t_lo][K][K] fp64; V[t - t_lo] = Newey-West(F[:t+1]) (NaN where t+1 <= q or <= K).
// ws: workspace of mfa_nw_workspace_bytes(T, K, q) bytes.
MFA_API size_t mfa_nw_workspace_bytes(int T, int K, int q) {
  const int nch = (T + CH - 1) / CH;
  return (size_t)nch * (4 + 7 * q) * K * K * sizeof(double);
}

MFA_API int mfa_nw_series(const double* F, int T, int K, int q, double tau, int t_lo, int t_hi,
                          double* V, void* ws, void* stream) {
  if (T <= 0 || t_hi <= t_lo) return 0;
  if (q < 0 || q > MAXQ || K <= 0 || t_lo < 0 || t_hi > T) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  NwDims dm{T, K, q, pow(0.5, 1.0 / tau)};
  // only chunks up to the one containing t_hi-1 are needed
  const int nch = (t_hi - 1) / CH + 1;
  const int KK = K * K;
  const size_t lds = (size_t)(CH + q) * K * sizeof(double);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  double* C = (double*)ws;
  dim3 blk(256);
  hipLaunchKernelGGL(nw_chunk_sums, dim3(nch, (KK + 255) / 256), blk, lds, s, F, dm, nch, C);
  const int ns = 4 + 7 * q;
  hipLaunchKernelGGL(nw_carry_scan, dim3((ns * KK + 255) / 256), blk, 0, s, dm, nch, C);
  const int c_first = t_lo / CH;
  hipLaunchKernelGGL(nw_emit, dim3(nch - c_first, (KK + 255) / 256), blk, lds, s, F, dm, C,
                     c_first, t_lo, t_hi, V);
  return (int)hipGetLastError();
}

MFA_API int mfa_ew_prefix_mean(const double* x, int T, double tau, double* out, void* stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ew_prefix_mean, dim3(1), dim3(64), 0, (hipStream_t)stream, x, T,
                     pow(0.5, 1.0 / tau), out);
  return (int)hipGetLastError();
}
