// Expanding-window exponentially-weighted Newey-West covariance series as a blocked scan (K8),
// plus the decayed prefix mean used by the volatility-regime adjustment (K10).
//
// Reference: Barra-master/mfm/utils.py:16-50 (Newey_West on one prefix, any lag count q < T)
// called for EVERY prefix f[:t], t = 1..T, by MFM.Newey_West_by_time (MFM.py:80-101):
// O(T^2 K^2) Python.
//
// Here every prefix is produced in O(T K^2 q) from decayed moments (l = 0.5^(1/tau)); with
// n = u + 1 the prefix length at date u and M[u] = sum_{s<=u} l^(u-s) f_s the decayed sum series:
//   Z(n) = (1 - l^n) / (1 - l)                          mu = M[u] / Z(n)
//   S0   = sum_s l^(u-s) f_s f_s^T                        G0 = S0 / Z - mu mu^T
//   A_i  = sum_{s>=i} l^(u-s) f_{s-i} f_s^T               a_i = M[u-i]
//   b_i  = M[u] - l^(u+1-i) M[i-1]                        z_i = Z(n-i)
//   G_i  = (A_i - a_i mu^T - mu b_i^T + z_i mu mu^T) / Z
//   V    = G0 + sum_{i=1..q} (1 - i/(q+1)) (G_i + G_i^T)
// Only S0 and the A_i are carried per (k,l) entry (1 + 2q fp64); the lag-shifted sums a_i, b_i,
// z_i come from the K-vector series M (one small scan) and Z's closed form.  Lags are processed
// in groups of at most G per launch triple, each group ADDING its terms to V, so q is limited
// only by the LDS rows [t0 - q, t1) of a chunk, never by registers.
// Work decomposition: thread = one (k,l) output entry; dates are cut into chunks of CH rows:
//   pass A  chunk-local decayed sums                 grid (chunks, ceil(K^2/256))
//   pass B  exclusive scan of chunk carries          sequential over chunks, parallel over moments
//   pass C  re-scan each chunk from its carry and write / accumulate V_t
// The output range [t_lo, t_hi) lets each data-parallel rank emit only its own date shard.
#include "common.h"

namespace {

using namespace mfa;

constexpr int CH = 32;  // dates per chunk (fewer for wide K: nw_chunk)
constexpr int G = 8;    // lags per launch group (register state: 1 + 2G fp64 per thread)

struct NwDims {
  int T, K, q;      // series length, factors, total lag count (weights 1 - i/(q+1))
  int i0, i1;       // this launch's lag group [i0, i1), 1-based lags
  double lam;
  int org;          // first date of the scanned range: chunk c = [org + c ch, org + (c+1) ch)
  int ch;           // dates per chunk (nw_chunk(K, q): CH unless a chunk's LDS image is too big)
};

// LDS image of a chunk: F rows [t0 - i1 + 1, t1) and M rows [t0 - i1 + 1, t1), then M rows
// [0, i1 - 1) (the b_i boundary terms, from Mg: the GLOBAL series' first rows).  Rows before
// date 0 are zero.  F and M are indexed by global date (a shard passes base pointers offset so
// that only its rows [org - q, T) are ever read).
__device__ void stage_rows(const double* __restrict__ F, const double* __restrict__ M,
                           const double* __restrict__ Mg, double* Fs, double* Ms, double* M0,
                           int t0, int t1, const NwDims& dm, bool want_m) {
  const int K = dm.K;
  const int lo = t0 - (dm.i1 - 1);
  const int rows = t1 - lo;
  for (int e = threadIdx.x; e < rows * K; e += blockDim.x) {
    const int r = e / K, c = e % K;
    const int t = lo + r;
    Fs[e] = t >= 0 ? F[(size_t)t * K + c] : 0.0;
    if (want_m) Ms[e] = t >= 0 ? M[(size_t)t * K + c] : 0.0;
  }
  if (want_m)
    for (int e = threadIdx.x; e < (dm.i1 - 1) * K; e += blockDim.x) {
      const int t = e / K;
      M0[e] = t < dm.T ? Mg[e] : 0.0;
    }
}

// Advance the (k,l) state over dates [t0, t1).  s[0] = S0 (group 0 only), s[1 + 2g + {0,1}] =
// A_{i0+g}[k][l], A_{i0+g}[l][k].  EMIT: write (or add) V for dates in [t_lo, t_hi).
// tab (EMIT only): per date u of the chunk, tab[(u - t0) * (1 + G)] = 1 / Z(n) and
// tab[(u - t0) * (1 + G) + 1 + g] = l^(n - i0 - g): one pow per (date, lag) per block instead of
// per (date, lag, k, l) thread
template <bool EMIT>
__device__ void nw_run_chunk(const double* Fs, const double* Ms, const double* M0, int t0, int t1,
                             int k, int l, const NwDims& dm, double (&s)[1 + 2 * G],
                             double* __restrict__ V, int t_lo, int t_hi, bool add,
                             const double* tab = nullptr) {
  const int K = dm.K, q = dm.q;
  const int off = dm.i1 - 1;  // LDS row of date t0
  const double lam = dm.lam;
  const double il = 1.0 / (1.0 - lam);
  const bool base = dm.i0 == 1;
  for (int u = t0; u < t1; ++u) {
    const int r = u - t0 + off;
    const double fk = Fs[r * K + k], fl = Fs[r * K + l];
    if (base) s[0] = fma(lam, s[0], fk * fl);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int i = dm.i0 + g;
      if (i >= dm.i1) break;
      const bool has = u >= i;
      const double gk = has ? Fs[(r - i) * K + k] : 0.0;
      const double gl = has ? Fs[(r - i) * K + l] : 0.0;
      s[1 + 2 * g] = fma(lam, s[1 + 2 * g], gk * fl);
      s[2 + 2 * g] = fma(lam, s[2 + 2 * g], gl * fk);
    }
    if (EMIT && u >= t_lo && u < t_hi) {
      const int n = u + 1;  // prefix length
      double* vo = V + (size_t)(u - t_lo) * K * K + (size_t)k * K + l;
      if (n <= q || n <= K) {
        if (base) *vo = qnan();
        continue;
      }
      const double* tu = tab + (u - t0) * (1 + G);
      const double iz = tu[0];
      const double mk = Ms[r * K + k] * iz, ml = Ms[r * K + l] * iz;
      double v = base ? s[0] * iz - mk * ml : 0.0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int i = dm.i0 + g;
        if (i >= dm.i1) break;
        const double ak = Ms[(r - i) * K + k], al = Ms[(r - i) * K + l];  // a_i = M[u-i]
        const double dec = tu[1 + g];
        const double bk = Ms[r * K + k] - dec * M0[(i - 1) * K + k];     // b_i
        const double bl = Ms[r * K + l] - dec * M0[(i - 1) * K + l];
        const double zi = (1.0 - dec) * il;                               // z_i = Z(n - i)
        // G_i[k][l] + G_i[l][k]
        const double gkl = s[1 + 2 * g] - ak * ml - mk * bl + zi * mk * ml;
        const double glk = s[2 + 2 * g] - al * mk - ml * bk + zi * ml * mk;
        v = fma(1.0 - (double)i / (q + 1), (gkl + glk) * iz, v);
      }
      *vo = add ? *vo + v : v;
    }
  }
}

__device__ __forceinline__ int nstate(const NwDims& dm) {
  return (dm.i0 == 1 ? 1 : 0) + 2 * (dm.i1 - dm.i0);
}

// moment m of the compact carry layout -> register slot
__device__ __forceinline__ int slot_of(const NwDims& dm, int m) {
  return dm.i0 == 1 ? m : m + 1;
}

// pass A: chunk-local sums.  C[chunk][m][kk] (m = compact moment index, kk = k*K+l)
__global__ __launch_bounds__(256) void nw_chunk_sums(const double* __restrict__ F, NwDims dm,
                                                     double* __restrict__ C) {
  extern __shared__ double Fs[];
  const int c = blockIdx.x;
  const int t0 = dm.org + c * dm.ch, t1 = min(dm.T, t0 + dm.ch);
  stage_rows(F, nullptr, nullptr, Fs, nullptr, nullptr, t0, t1, dm, false);
  __syncthreads();
  const int KK = dm.K * dm.K;
  const int kk = blockIdx.y * blockDim.x + threadIdx.x;
  if (kk >= KK) return;
  double s[1 + 2 * G];
#pragma unroll
  for (int i = 0; i < 1 + 2 * G; ++i) s[i] = 0.0;
  nw_run_chunk<false>(Fs, nullptr, nullptr, t0, t1, kk / dm.K, kk % dm.K, dm, s, nullptr, 0, 0,
                      false);
  const int ns = nstate(dm);
#pragma unroll
  for (int m = 0; m < 1 + 2 * G; ++m)
    if (m < ns) C[((size_t)c * ns + m) * KK + kk] = s[slot_of(dm, m)];
}

// pass B: in-place exclusive scan over chunks: C[c] <- Cin + sum_{c'<c} l^(t0_c - t1_c') C[c']
// (Cin: the state at date org - 1 carried in from earlier shards, decayed along; null = 0).
// Ctot (optional): the inclusive total at date T - 1 (a shard's contribution to later shards).
__global__ __launch_bounds__(256) void nw_carry_scan(NwDims dm, int nchunks, double* __restrict__ C,
                                                     const double* __restrict__ Cin,
                                                     double* __restrict__ Ctot) {
  const int KK = dm.K * dm.K;
  const int ns = nstate(dm);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (m, kk)
  if (e >= ns * KK) return;
  const double dch = pow(dm.lam, (double)dm.ch);
  double carry = Cin ? Cin[e] : 0.0;
  for (int c = 0; c < nchunks; ++c) {
    const int t0 = dm.org + c * dm.ch;
    const int len = min(dm.T, t0 + dm.ch) - t0;
    double* p = C + (size_t)c * ns * KK + e;
    const double loc = *p;
    *p = carry;
    carry = fma(len == dm.ch ? dch : pow(dm.lam, (double)len), carry, loc);
  }
  if (Ctot) Ctot[e] = carry;
}

// pass C: outputs for chunks overlapping [t_lo, t_hi)
__global__ __launch_bounds__(256) void nw_emit(const double* __restrict__ F,
                                               const double* __restrict__ M,
                                               const double* __restrict__ Mg, NwDims dm,
                                               const double* __restrict__ C, int c_first,
                                               int t_lo, int t_hi, double* __restrict__ V,
                                               int add) {
  extern __shared__ double Fs[];
  const int c = c_first + blockIdx.x;
  const int t0 = dm.org + c * dm.ch, t1 = min(dm.T, t0 + dm.ch);
  const int rows = t1 - t0 + dm.i1 - 1;
  double* Ms = Fs + (size_t)rows * dm.K;
  double* M0 = Ms + (size_t)rows * dm.K;
  double* tab = M0 + (size_t)(dm.i1 - 1) * dm.K;  // [ch][1 + G]
  stage_rows(F, M, Mg, Fs, Ms, M0, t0, t1, dm, true);
  for (int e = threadIdx.x; e < (t1 - t0) * (1 + G); e += blockDim.x) {
    const int du = e / (1 + G), g = e % (1 + G);
    const double n = (double)(t0 + du + 1);
    tab[e] = g == 0 ? (1.0 - dm.lam) / (1.0 - pow(dm.lam, n)) : pow(dm.lam, n - (dm.i0 + g - 1));
  }
  __syncthreads();
  const int KK = dm.K * dm.K;
  const int kk = blockIdx.y * blockDim.x + threadIdx.x;
  if (kk >= KK) return;
  const int ns = nstate(dm);
  double s[1 + 2 * G];
#pragma unroll
  for (int m = 0; m < 1 + 2 * G; ++m) s[m] = 0.0;
#pragma unroll
  for (int m = 0; m < 1 + 2 * G; ++m)
    if (m < ns) s[slot_of(dm, m)] = C[((size_t)c * ns + m) * KK + kk];
  nw_run_chunk<true>(Fs, Ms, M0, t0, t1, kk / dm.K, kk % dm.K, dm, s, V, t_lo, t_hi, add != 0,
                     tab);
}

// Decayed running sums of K series over rows [t_s, T): M[t][k] = l^(t-t_s+1) init[k] +
// sum_{t_s<=s<=t} l^(t-s) x[s][k] (no masking; init null = 0; x, M indexed by global row).
// One wave per column; lane-chunked two-level scan.
__global__ __launch_bounds__(64) void ew_cumsum_cols(const double* __restrict__ x, int t_s, int T,
                                                    int K, double lam,
                                                    const double* __restrict__ init,
                                                    double* __restrict__ M) {
  const int k = blockIdx.x, lane = threadIdx.x;
  const int per = (T - t_s + 63) / 64;
  const int a = min(T, t_s + lane * per), b = min(T, a + per);
  double num = 0.0;
  for (int t = a; t < b; ++t) num = fma(lam, num, x[(size_t)t * K + k]);
  double cn = num, dk = pow(lam, (double)(b - a));
  for (int off = 1; off < 64; off <<= 1) {
    const double pn = __shfl_up(cn, off, 64), pk = __shfl_up(dk, off, 64);
    if (lane >= off) {
      cn = fma(pn, dk, cn);
      dk = dk * pk;
    }
  }
  double en = __shfl_up(cn, 1, 64);
  if (lane == 0) en = 0.0;
  if (init) en = fma(pow(lam, (double)(a - t_s)), init[k], en);  // carried-in state, decayed
  for (int t = a; t < b; ++t) {
    en = fma(lam, en, x[(size_t)t * K + k]);
    M[(size_t)t * K + k] = en;
  }
}

// Mtot[k] = sum_{t_s<=s<T} l^(T-1-s) x[s][k]: a shard's own contribution to M[T - 1].
__global__ __launch_bounds__(64) void ew_cumsum_tail(const double* __restrict__ x, int t_s, int T,
                                                    int K, double lam, double* __restrict__ Mtot) {
  const int k = blockIdx.x, lane = threadIdx.x;
  double acc = 0.0;
  for (int t = t_s + lane; t < T; t += 64) acc = fma(pow(lam, (double)(T - 1 - t)), x[(size_t)t * K + k], acc);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) Mtot[k] = acc;
}

// Decayed prefix mean with validity: out[t] = sum_{s<=t, ok} l^(t-s) x_s / sum_{s<=t, ok} l^(t-s)
// (VRA factor-volatility multiplier, MFM.py:149-160).  One wave; chunked two-level scan.
__global__ __launch_bounds__(64) void ew_prefix_mean(const double* __restrict__ x, int T, double lam,
                                                     double* __restrict__ out,
                                                     const double* __restrict__ init = nullptr,
                                                     double* __restrict__ tot = nullptr) {
  const int lane = threadIdx.x;
  const int per = (T + 63) / 64;
  const int a = min(T, lane * per), b = min(T, a + per);
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
  if (tot && lane == 63) { tot[0] = cn; tot[1] = cd; }  // own totals at date T - 1
  double en = __shfl_up(cn, 1, 64), ed = __shfl_up(cd, 1, 64);
  if (lane == 0) { en = 0.0; ed = 0.0; }
  if (init) {  // (num, den) carried in at date -1 of this shard, decayed to a - 1
    const double da = pow(lam, (double)a);
    en = fma(da, init[0], en);
    ed = fma(da, init[1], ed);
  }
  num = en; den = ed;
  if (out)
    for (int t = a; t < b; ++t) {
      const double v = x[t];
      const bool ok = __builtin_isfinite(v);
      num = fma(lam, num, ok ? v : 0.0);
      den = fma(lam, den, ok ? 1.0 : 0.0);
      out[t] = den > 0.0 ? num / den : qnan();
    }
}

// LDS doubles of the emit pass's chunk image (the larger of the two passes) at ch dates per
// chunk and lags up to q
size_t nw_lds_doubles(int ch, int K, int q) {
  return (size_t)(2 * (ch + q) + q) * K + (size_t)ch * (1 + G);
}
// Dates per chunk: CH, halved (down to 4) while a chunk's LDS image exceeds the CU's 160 KB --
// a function of (K, q) only, so every shard and rank chunks the same way; K <= ~190 at q = 2
// keeps CH (bitwise the round-5 scan)
int nw_chunk(int K, int q) {
  int ch = CH;
  while (ch > 4 && nw_lds_doubles(ch, K, q) * sizeof(double) > 160 * 1024) ch >>= 1;
  return ch;
}

size_t nw_carry_bytes(int T, int K, int q) {
  const int ch = nw_chunk(K, q);
  const int nch = (T + ch - 1) / ch;
  const int g = q < G ? q : G;
  return (size_t)nch * (1 + 2 * g) * K * K * sizeof(double);
}

}  // namespace

// F: [T][K] fp64 factor-return series (global calendar, all dates up to t_hi).
// V: [t_hi - t_lo][K][K] fp64; V[t - t_lo] = Newey-West(F[:t+1]) (NaN where t+1 <= q or <= K).
// ws: workspace of mfa_nw_workspace_bytes(T, K, q) bytes (chunk carries + the M series).
MFA_API size_t mfa_nw_workspace_bytes(int T, int K, int q) {
  return nw_carry_bytes(T, K, q) + (size_t)T * K * sizeof(double);
}

// Largest lag count the kernels accept for K factors (LDS rows of one chunk).
MFA_API int mfa_nw_max_lags(int K) {
  int q = 0;
  while (nw_lds_doubles(4, K, q + 1) * sizeof(double) <= 160 * 1024) ++q;
  return q;
}

MFA_API int mfa_nw_series(const double* F, int T, int K, int q, double tau, int t_lo, int t_hi,
                          double* V, void* ws, void* stream) {
  if (T <= 0 || t_hi <= t_lo) return 0;
  if (q < 0 || K <= 0 || t_lo < 0 || t_hi > T || q > mfa_nw_max_lags(K))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const double lam = pow(0.5, 1.0 / tau);
  // the scan always covers all T dates (the caller passes the series length), so a rank that
  // emits only its own window [t_lo, t_hi) computes every date bitwise like the one-process
  // run (same chunking and carries); the extra scan is ~0.1 ms at T = 2520
  const int Tn = T;
  const int ch = nw_chunk(K, q);
  const int nch = (Tn - 1) / ch + 1;
  const int KK = K * K;
  double* C = (double*)ws;
  double* M = (double*)((char*)ws + nw_carry_bytes(Tn, K, q));
  hipLaunchKernelGGL(ew_cumsum_cols, dim3(K), dim3(64), 0, s, F, 0, Tn, K, lam,
                     (const double*)nullptr, M);
  const int c_first = t_lo / ch;
  dim3 blk(256);
  // lag groups [i0, i1): group 0 also carries S0 and writes V; later groups add their lags
  for (int i0 = 1, grp = 0; grp == 0 || i0 <= q; i0 += G, ++grp) {
    const int i1 = std::min(q + 1, i0 + G);
    NwDims dm{Tn, K, q, i0, i1, lam, 0, ch};
    const int ns = (i0 == 1 ? 1 : 0) + 2 * (i1 - i0);
    const size_t ldsA = (size_t)(ch + i1 - 1) * K * sizeof(double);
    const size_t ldsC = ((size_t)(2 * (ch + i1 - 1) + (i1 - 1)) * K + ch * (1 + G)) * sizeof(double);
    hipLaunchKernelGGL(nw_chunk_sums, dim3(nch, (KK + 255) / 256), blk, ldsA, s, F, dm, C);
    hipLaunchKernelGGL(nw_carry_scan, dim3((ns * KK + 255) / 256), blk, 0, s, dm, nch, C,
                       (const double*)nullptr, (double*)nullptr);
    hipLaunchKernelGGL(nw_emit, dim3(nch - c_first, (KK + 255) / 256), blk, ldsC, s, F, M, M, dm,
                       C, c_first, t_lo, t_hi, V, grp > 0 ? 1 : 0);
  }
  return (int)hipGetLastError();
}

// Carried state of the sharded scan: for every lag group g (groups of G lags, [1 + 8g, ...)),
// nstate(g) x K x K moments (S0 for group 0, then A_i[k][l], A_i[l][k] per lag), concatenated.
MFA_API size_t mfa_nw_state_doubles(int K, int q) {
  size_t n = 0;
  for (int i0 = 1, grp = 0; grp == 0 || i0 <= q; i0 += G, ++grp) {
    const int i1 = std::min(q + 1, i0 + G);
    n += (size_t)((i0 == 1 ? 1 : 0) + 2 * (i1 - i0)) * K * K;
  }
  return n;
}

// Shard workspace: chunk carries of [T0, T1) + the M series rows [T0 - q, T1).
MFA_API size_t mfa_nw_shard_workspace_bytes(int T0, int T1, int K, int q) {
  const int h = q > 1 ? q : 1;
  const int lo = T0 - h > 0 ? T0 - h : 0;
  return nw_carry_bytes(T1 - T0, K, q) + (size_t)(T1 - lo) * K * sizeof(double);
}

// One date shard [T0, T1) of the expanding-window Newey-West series (SURVEY 2.5 time-axis
// scan across ranks).  With h = max(q, 1): Fsh = rows [max(0, T0 - h), T1) of F (the halo +
// the shard); Mh: the GLOBAL decayed sums M[t] = sum_{s<=t} l^(t-s) f_s for rows [max(0, T0 - h), T0)
// (null when T0 == 0); Mg: global M rows [0, min(q, T1)) (b_i boundary terms).
// Cin: carried state at date T0 - 1 (mfa_nw_state_doubles layout; null = zero, i.e. T0 == 0).
// Outputs (each optional): V [T1 - T0][K][K] for the shard's dates; Ctot = the shard's own
// contribution to the state at date T1 - 1 (chunk sums of [T0, T1) including the halo lag
// products, NOT including Cin); Mtot = sum_{T0<=s<T1} l^(T1-1-s) f_s.
MFA_API int mfa_nw_series_shard(const double* Fsh, const double* Mh, const double* Mg, int T0,
                                int T1, int K, int q, double tau, const double* Cin, double* V,
                                double* Ctot, double* Mtot, void* ws, void* stream) {
  if (T1 <= T0) return 0;
  if (q < 0 || K <= 0 || T0 < 0 || q > mfa_nw_max_lags(K)) return (int)hipErrorInvalidValue;
  if (V && T0 > 0 && Mh == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const double lam = pow(0.5, 1.0 / tau);
  const int h = q > 1 ? q : 1;
  const int lo = T0 - h > 0 ? T0 - h : 0;
  const int ch = nw_chunk(K, q);
  const int nch = (T1 - T0 - 1) / ch + 1;
  const int KK = K * K;
  const double* Fb = Fsh - (size_t)lo * K;  // indexed by global date (rows >= lo only)
  double* C = (double*)ws;
  double* Mw = (double*)((char*)ws + nw_carry_bytes(T1 - T0, K, q));
  double* Mb = Mw - (size_t)lo * K;         // indexed by global date
  if (V) {
    if (T0 > lo) {
      const hipError_t e = hipMemcpyAsync(Mw, Mh, (size_t)(T0 - lo) * K * sizeof(double),
                                          hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return (int)e;
    }
    // own rows of M: carried M[T0 - 1] (the halo's last row) decayed along
    hipLaunchKernelGGL(ew_cumsum_cols, dim3(K), dim3(64), 0, s, Fb, T0, T1, K, lam,
                       T0 > 0 ? Mb + (size_t)(T0 - 1) * K : (const double*)nullptr, Mb);
  }
  if (Mtot)  // own contribution only: rescan with no carried state
    hipLaunchKernelGGL(ew_cumsum_tail, dim3(K), dim3(64), 0, s, Fb, T0, T1, K, lam, Mtot);
  dim3 blk(256);
  size_t off = 0;
  for (int i0 = 1, grp = 0; grp == 0 || i0 <= q; i0 += G, ++grp) {
    const int i1 = std::min(q + 1, i0 + G);
    NwDims dm{T1, K, q, i0, i1, lam, T0, ch};
    const int ns = (i0 == 1 ? 1 : 0) + 2 * (i1 - i0);
    const size_t ldsA = (size_t)(ch + i1 - 1) * K * sizeof(double);
    const size_t ldsC = ((size_t)(2 * (ch + i1 - 1) + (i1 - 1)) * K + ch * (1 + G)) * sizeof(double);
    hipLaunchKernelGGL(nw_chunk_sums, dim3(nch, (KK + 255) / 256), blk, ldsA, s, Fb, dm, C);
    if (Ctot)  // own contribution: scan from zero, keep the total, then rescan from Cin below
      hipLaunchKernelGGL(nw_carry_scan, dim3((ns * KK + 255) / 256), blk, 0, s, dm, nch, C,
                         (const double*)nullptr, Ctot + off);
    if (V) {
      if (Ctot)
        hipLaunchKernelGGL(nw_chunk_sums, dim3(nch, (KK + 255) / 256), blk, ldsA, s, Fb, dm, C);
      hipLaunchKernelGGL(nw_carry_scan, dim3((ns * KK + 255) / 256), blk, 0, s, dm, nch, C,
                         Cin ? Cin + off : (const double*)nullptr, (double*)nullptr);
      hipLaunchKernelGGL(nw_emit, dim3(nch, (KK + 255) / 256), blk, ldsC, s, Fb, Mb, Mg, dm, C, 0,
                         T0, T1, V, grp > 0 ? 1 : 0);
    }
    off += (size_t)ns * KK;
  }
  return (int)hipGetLastError();
}

// Shard of the decayed prefix mean: init = (num, den) carried in at date -1 (null = 0), out =
// the shard's prefix means (nullable), tot = its own (num, den) totals at date T - 1 (nullable).
MFA_API int mfa_ew_prefix_mean_shard(const double* x, int T, double tau, const double* init,
                                     double* out, double* tot, void* stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ew_prefix_mean, dim3(1), dim3(64), 0, (hipStream_t)stream, x, T,
                     pow(0.5, 1.0 / tau), out, init, tot);
  return (int)hipGetLastError();
}

MFA_API int mfa_ew_prefix_mean(const double* x, int T, double tau, double* out, void* stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ew_prefix_mean, dim3(1), dim3(64), 0, (hipStream_t)stream, x, T,
                     pow(0.5, 1.0 / tau), out);
  return (int)hipGetLastError();
}
