// Batched, fused cross-sectional WLS factor-return regression (Barra CNE5/USE4 style) for gfx950.
//
// Reference semantics: Barra-master/mfm/CrossSection.py:12-20 (style z-score: cap-weighted mean,
// ONE pooled ddof-0 std) and :57-108 (sqrt-cap WLS, industry-neutral constraint
// sum_j s_j f_j = 0 via the K x (K-1) matrix R, pinv solve, f = Omega r, e = r - X f,
// unweighted R^2).
//
// MI355X-first design (nothing mirrors the reference's dense N x N weight matrix):
//   * one workgroup of `nw` waves per date, every date of the shard in ONE launch;  with
//     nw = 4 about 512 dates are in flight chip-wide (~130 MB at N=5000), so the second pass
//     over a date is served from the 256 MB Infinity Cache instead of HBM;
//   * pass 1 streams the date once (coalesced [D][Q][N] fp32 styles, int16 industry ids) and
//     accumulates RAW fp64 moments in registers; the z-scored Gram is derived algebraically
//     from them, so standardisation costs no extra pass;
//   * the one-hot industry block is never materialised: it is a segmented sum accumulated with
//     native LDS ds_add_f64 atomics into a [P][Q+3] table;
//   * the constrained normal equations are solved STRUCTURALLY: after eliminating the pivot
//     industry, the industry block is diag(W) + rho a a^T, inverted by Sherman-Morrison, and
//     only the (1+Q) x (1+Q) Schur complement (country + styles) is Cholesky-factorised in
//     fp64.  Exactly-empty industries get f = 0 (pinv semantics); near-singular dates are
//     flagged for the host-side pseudo-inverse fallback;
//   * pass 2 re-streams the date (MALL-hot) to write fp32 specific returns and R^2.
#include "common.h"

namespace {

using namespace mfa;

enum XsStatus : int {
  XS_NO_ROWS = 1,        // no valid stock on the date
  XS_PIVOT_EMPTY = 2,    // constraint pivot industry has zero capital
  XS_NEAR_SINGULAR = 4,  // Schur Cholesky lost > 12 digits: host refines with pinv
  XS_ZERO_PIVOT = 8,     // exactly-zero pivots / empty industries (pinv semantics -> f = 0)
  XS_BAD_SIGMA = 16,     // pooled style std is zero / NaN
};

struct XsDims {
  int D, N, P, Pseg, has_ind, pivot_mode;
  double tol;
};

__device__ __forceinline__ bool finite_f(float v) { return __builtin_isfinite(v); }

__device__ __forceinline__ void lds_add(double* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Reduce a compile-time register array across the workgroup into out[0..CNT) (LDS, zeroed by
// the caller).  Chunks of 8 values go through a per-wave [8][65] fp64 LDS tile, which keeps the
// register footprint flat (a shuffle butterfly over ~80 fp64 accumulators costs ~110 VGPRs).
template <int CNT>
__device__ __forceinline__ void wg_reduce(const double (&v)[CNT], double* wbuf, double* out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int a = lane & 7, slice = lane >> 3;
#pragma unroll
  for (int c0 = 0; c0 < CNT; c0 += 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (c0 + i < CNT) wbuf[i * 65 + lane] = v[c0 + i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += wbuf[a * 65 + slice * 8 + i];
    t += __shfl_xor(t, 8, kWave);
    t += __shfl_xor(t, 16, kWave);
    t += __shfl_xor(t, 32, kWave);
    if (slice == 0 && c0 + a < CNT) lds_add(out + c0 + a, t);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int Q>
struct Layout {
  static constexpr int NS = Q + 3;            // per-industry channels: W, A_q, B, s
  static constexpr int NG = Q * (Q + 1) / 2;  // packed symmetric raw Gram
  static constexpr int NACC = NG + 2 * Q + 4; // Swxx | Swxr | Scx | Sc Sx Sxx n
  static constexpr int ND = Q + 1;            // dense block: country + styles
};

template <int Q>
__global__ __launch_bounds__(256) void xs_wls_kernel(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, XsDims dm, double* __restrict__ fout,
    float* __restrict__ eout, double* __restrict__ r2out, double* __restrict__ stats,
    int* __restrict__ status) {
  using L = Layout<Q>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, ND = L::ND;
  extern __shared__ double lds[];
  const int d = blockIdx.x;
  const int tid = threadIdx.x;
  const int nthr = blockDim.x;
  const int wid = tid >> 6;
  const int N = dm.N, Pseg = dm.Pseg, P = dm.P;
  const int K = 1 + P + Q;

  // ---- LDS carve (doubles) ----
  double* seg = lds;                 // [Pseg][NS]
  double* acc = seg + Pseg * NS;     // [NACC] reduced raw moments
  double* mu = acc + NACC;           // [Q]
  double* Swx = mu + Q;              // [Q]
  double* misc = Swx + Q;            // [16] scalars
  double* MDD = misc + 16;           // [ND][ND+1]  dense block, then its Cholesky factor
  double* hD = MDD + ND * (ND + 1);  // [ND]
  double* MID = hD + ND;             // [Pseg][ND+1]  M_ID | h_I
  double* Y = MID + Pseg * (ND + 1); // [Pseg][ND+1]  M_II^{-1} [M_ID | h_I]
  double* f = Y + Pseg * (ND + 1);   // [K]
  double* wbuf = f + K + ((K & 1) ? 1 : 0);  // per-wave [8][65] reduction tiles
  double* mywbuf = wbuf + wid * 8 * 65;

  for (int i = tid; i < Pseg * NS + NACC; i += nthr) lds[i] = 0.0;
  __syncthreads();

  const float* Xd = X + (size_t)d * Q * N;
  const float* cd = cap + (size_t)d * N;
  const float* rd = ret + (size_t)d * N;
  const int16_t* id = dm.has_ind ? ind + (size_t)d * N : nullptr;

  // ---- pass 1: raw fp64 moments (registers) + segmented industry sums (LDS atomics) ----
  double v[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) v[i] = 0.0;
  for (int n = tid; n < N; n += nthr) {
    const float cf = cd[n];
    const float rf = rd[n];
    const int j = id ? (int)id[n] : 0;
    float xf[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) xf[q] = Xd[(size_t)q * N + n];
    bool ok = (j >= 0) && (j < Pseg) && finite_f(cf) && (cf >= 0.f) && finite_f(rf);
#pragma unroll
    for (int q = 0; q < Q; ++q) ok = ok && finite_f(xf[q]);
    if (!ok) continue;
    const double c = cf, r = rf, w = sqrt(c);
    double x[Q], wx[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) { x[q] = xf[q]; wx[q] = w * x[q]; }
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int s = 0; s <= q; ++s) v[q * (q + 1) / 2 + s] = fma(wx[q], x[s], v[q * (q + 1) / 2 + s]);
    double sx = 0.0, sxx = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      v[NG + q] = fma(wx[q], r, v[NG + q]);
      v[NG + Q + q] = fma(c, x[q], v[NG + Q + q]);
      sx += x[q];
      sxx = fma(x[q], x[q], sxx);
    }
    v[NG + 2 * Q + 0] += c;
    v[NG + 2 * Q + 1] += sx;
    v[NG + 2 * Q + 2] += sxx;
    v[NG + 2 * Q + 3] += 1.0;
    double* sj = seg + j * NS;
    lds_add(sj + 0, w);
#pragma unroll
    for (int q = 0; q < Q; ++q) lds_add(sj + 1 + q, wx[q]);
    lds_add(sj + Q + 1, w * r);
    lds_add(sj + Q + 2, c);
  }
  wg_reduce<NACC>(v, mywbuf, acc);
  __syncthreads();

  // ---- moments -> standardised system (Q << 64 : lane-parallel in wave 0 + all-thread loops) ----
  const double Sc = acc[NG + 2 * Q + 0];
  const double nval = acc[NG + 2 * Q + 3];
  const double nq = nval * Q;
  const double mx = acc[NG + 2 * Q + 1] / nq;
  const double sigma = sqrt(fmax(acc[NG + 2 * Q + 2] / nq - mx * mx, 0.0));
  const double isig = 1.0 / sigma;
  int st = 0;
  if (!(nval > 0.0)) st |= XS_NO_ROWS;
  if (!(sigma > 0.0) || !__builtin_isfinite(sigma)) st |= XS_BAD_SIGMA;

  if (tid < Q) {
    double t = 0.0;
    for (int jj = 0; jj < Pseg; ++jj) t += seg[jj * NS + 1 + tid];
    Swx[tid] = t;
    mu[tid] = acc[NG + Q + tid] / Sc;
  }
  if (tid == 0) {
    double Sw = 0.0, Swr = 0.0;
    for (int jj = 0; jj < Pseg; ++jj) { Sw += seg[jj * NS]; Swr += seg[jj * NS + Q + 1]; }
    misc[0] = Sw;
    misc[1] = Swr;
  }
  __syncthreads();
  const double Sw = misc[0], Swr = misc[1];
  // dense block (country, styles) of X~' W X~ and rhs; x~ = (x - mu) / sigma
  for (int e = tid; e < ND * ND; e += nthr) {
    const int u = e / ND, w = e % ND;
    double m;
    if (u == 0 && w == 0) m = Sw;
    else if (u == 0 || w == 0) {
      const int q = (u == 0 ? w : u) - 1;
      m = (Swx[q] - mu[q] * Sw) * isig;
    } else {
      const int q = u - 1, s = w - 1;
      const int hi = q > s ? q : s, lo = q > s ? s : q;
      m = (acc[hi * (hi + 1) / 2 + lo] - mu[q] * Swx[s] - mu[s] * Swx[q] + mu[q] * mu[s] * Sw) *
          isig * isig;
    }
    MDD[u * (ND + 1) + w] = m;
  }
  if (tid < ND) hD[tid] = tid == 0 ? Swr : (acc[NG + tid - 1] - mu[tid - 1] * Swr) * isig;
  for (int e = tid; e < Pseg * Q; e += nthr) {  // standardise the segmented style sums in place
    const int jj = e / Q, q = e % Q;
    double* p = seg + jj * NS;
    p[1 + q] = (p[1 + q] - mu[q] * p[0]) * isig;
  }
  __syncthreads();

  // ---- constraint + structured solve ----
  int jp = -1;  // pivot industry (0-based)
  if (P > 0) {
    if (dm.pivot_mode == 1) {
      jp = P - 1;  // reference: always the last industry (CrossSection.py:69)
    } else {
      for (int jj = P - 1; jj >= 0; --jj)
        if (seg[jj * NS + Q + 2] > 0.0) { jp = jj; break; }
      if (jp < 0) jp = P - 1;
    }
    if (!(seg[jp * NS + Q + 2] > 0.0)) st |= XS_PIVOT_EMPTY;
  }
  const double sp = P > 0 ? seg[jp * NS + Q + 2] : 1.0;
  const double rho = P > 0 ? seg[jp * NS] : 0.0;
  // M_ID = G_ID + a_j G_pD ;  h_I = B_j + a_j B_p ;  a_j = -s_j / s_p
  for (int e = tid; e < P * (ND + 1); e += nthr) {
    const int jj = e / (ND + 1), u = e % (ND + 1);
    double m = 0.0;
    if (jj != jp && seg[jj * NS] > 0.0) {
      const double aj = -seg[jj * NS + Q + 2] / sp;
      if (u == 0) m = seg[jj * NS] + aj * seg[jp * NS];
      else if (u <= Q) m = seg[jj * NS + u] + aj * seg[jp * NS + u];
      else m = seg[jj * NS + Q + 1] + aj * seg[jp * NS + Q + 1];
    }
    MID[e] = m;
  }
  __syncthreads();
  if (P > 0 && tid == 0) {  // Sherman-Morrison scalars over the active industry set I
    double den = 0.0;
    for (int jj = 0; jj < P; ++jj) {
      const double W = seg[jj * NS];
      if (jj == jp || !(W > 0.0)) continue;
      const double aj = -seg[jj * NS + Q + 2] / sp;
      den = fma(aj * rho, aj / W, den);
    }
    misc[2] = rho / (1.0 + den);  // kappa
  }
  __syncthreads();
  // Y[:, u] = M_II^{-1} MID[:, u] = t - kappa (a.t) a~ ,  t = MID[:, u] / W
  if (P > 0 && tid <= ND) {
    const int u = tid;
    const double kappa = misc[2];
    double at = 0.0;
    for (int jj = 0; jj < P; ++jj) {
      const double W = seg[jj * NS];
      if (jj == jp || !(W > 0.0)) continue;
      const double aj = -seg[jj * NS + Q + 2] / sp;
      at = fma(aj, MID[jj * (ND + 1) + u] / W, at);
    }
    for (int jj = 0; jj < P; ++jj) {
      const double W = seg[jj * NS];
      double y = 0.0;
      if (jj != jp && W > 0.0) {
        const double aj = -seg[jj * NS + Q + 2] / sp;
        y = (MID[jj * (ND + 1) + u] - kappa * at * aj) / W;
      }
      Y[jj * (ND + 1) + u] = y;
    }
  }
  __syncthreads();
  // Schur complement S = M_DD - M_ID^T Y_D ; rhs = h_D - M_ID^T y
  if (P > 0) {
    for (int e = tid; e < ND * (ND + 1); e += nthr) {
      const int u = e / (ND + 1), w = e % (ND + 1);
      if (w < u) continue;  // upper incl. rhs column; lower mirrored below
      double t = 0.0;
      for (int jj = 0; jj < P; ++jj) t = fma(MID[jj * (ND + 1) + u], Y[jj * (ND + 1) + w], t);
      if (w < ND) MDD[u * (ND + 1) + w] -= t;
      else hD[u] -= t;
    }
    __syncthreads();
  }
  // Cholesky of the (1+Q) x (1+Q) Schur complement, single wave, pinv semantics for zero pivots
  if (wid == 0) {
    const int lane = tid;
    if (lane < ND)  // mirror upper -> lower
      for (int w = 0; w < lane; ++w) MDD[lane * (ND + 1) + w] = MDD[w * (ND + 1) + lane];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double dmax = 0.0;
    for (int k = 0; k < ND; ++k) dmax = fmax(dmax, fabs(MDD[k * (ND + 1) + k]));
    const double ztol = dm.tol * dmax;
    const double diag0 = lane < ND ? MDD[lane * (ND + 1) + lane] : 0.0;
    unsigned int skip = 0u;
    for (int k = 0; k < ND; ++k) {
      const double dk = MDD[k * (ND + 1) + k];
      const double d0k = __shfl(diag0, k, kWave);
      const bool zero = !(dk > ztol);
      __builtin_amdgcn_wave_barrier();
      if (zero) {
        skip |= 1u << k;
        if (lane >= k && lane < ND) MDD[lane * (ND + 1) + k] = 0.0;
        st |= (d0k > ztol) ? XS_NEAR_SINGULAR : XS_ZERO_PIVOT;
      } else {
        if (dk < 1e-12 * d0k) st |= XS_NEAR_SINGULAR;
        const double l = sqrt(dk);
        if (lane > k && lane < ND) MDD[lane * (ND + 1) + k] /= l;
        if (lane == k) MDD[k * (ND + 1) + k] = l;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (!zero && lane > k && lane < ND) {
        const double lik = MDD[lane * (ND + 1) + k];
        for (int w = k + 1; w <= lane; ++w) MDD[lane * (ND + 1) + w] -= lik * MDD[w * (ND + 1) + k];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) {  // tiny triangular solves, one lane
      for (int k = 0; k < ND; ++k) {
        double t = hD[k];
        for (int w = 0; w < k; ++w) t -= MDD[k * (ND + 1) + w] * hD[w];
        hD[k] = ((skip >> k) & 1u) ? 0.0 : t / MDD[k * (ND + 1) + k];
      }
      for (int k = ND - 1; k >= 0; --k) {
        double t = hD[k];
        for (int w = k + 1; w < ND; ++w) t -= MDD[w * (ND + 1) + k] * hD[w];
        hD[k] = ((skip >> k) & 1u) ? 0.0 : t / MDD[k * (ND + 1) + k];
      }
    }
    if (lane == 0) misc[3] = (double)st;
  }
  __syncthreads();
  st |= (int)misc[3];
  // assemble f = R g : country, industries (g_I = y - Y_D g_D, pivot from the constraint), styles
  if (tid < Q) f[1 + P + tid] = hD[1 + tid];
  if (tid == 0) f[0] = hD[0];
  for (int jj = tid; jj < P; jj += nthr) {
    double g = Y[jj * (ND + 1) + ND];
    for (int u = 0; u < ND; ++u) g -= Y[jj * (ND + 1) + u] * hD[u];
    f[1 + jj] = g;  // zero for the pivot and for empty industries (Y rows are zero)
  }
  __syncthreads();
  if (P > 0 && tid == 0) {
    double t = 0.0;
    for (int jj = 0; jj < P; ++jj)
      if (jj != jp) t = fma(-seg[jj * NS + Q + 2] / sp, f[1 + jj], t);
    f[1 + jp] = t;
  }
  __syncthreads();
  const bool bad = (st & (XS_NO_ROWS | XS_BAD_SIGMA | XS_PIVOT_EMPTY)) != 0;
  if (bad)
    for (int i = tid; i < K; i += nthr) f[i] = qnan();
  __syncthreads();

  // ---- pass 2: specific returns + R^2 (date is hot in L2 / Infinity Cache) ----
  double beta[Q];
  double cst = f[0];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    beta[q] = f[1 + P + q] * isig;
    cst -= beta[q] * mu[q];
  }
  double se = 0.0, see = 0.0, sr = 0.0, srr = 0.0;
  float* ed = eout ? eout + (size_t)d * N : nullptr;
  for (int n = tid; n < N; n += nthr) {
    const float cf = cd[n];
    const float rf = rd[n];
    const int j = id ? (int)id[n] : 0;
    float xf[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) xf[q] = Xd[(size_t)q * N + n];
    bool ok = (j >= 0) && (j < Pseg) && finite_f(cf) && (cf >= 0.f) && finite_f(rf);
#pragma unroll
    for (int q = 0; q < Q; ++q) ok = ok && finite_f(xf[q]);
    float eo = qnanf();
    if (ok) {
      double e = (double)rf - cst - (P > 0 ? f[1 + j] : 0.0);
#pragma unroll
      for (int q = 0; q < Q; ++q) e = fma(-beta[q], (double)xf[q], e);
      se += e;
      see = fma(e, e, see);
      sr += rf;
      srr = fma((double)rf, (double)rf, srr);
      eo = (float)e;
    }
    if (ed) ed[n] = eo;
  }
  se = wave_sum(se);
  see = wave_sum(see);
  sr = wave_sum(sr);
  srr = wave_sum(srr);
  double* red = acc;  // reuse (raw moments no longer needed)
  __syncthreads();
  if (tid < 4) red[tid] = 0.0;
  __syncthreads();
  if ((tid & 63) == 0) { lds_add(red + 0, se); lds_add(red + 1, see); lds_add(red + 2, sr); lds_add(red + 3, srr); }
  __syncthreads();
  for (int i = tid; i < K; i += nthr) fout[(size_t)d * K + i] = f[i];
  if (tid == 0) {
    const double ve = red[1] / nval - (red[0] / nval) * (red[0] / nval);
    const double vr = red[3] / nval - (red[2] / nval) * (red[2] / nval);
    r2out[d] = bad ? qnan() : 1.0 - ve / vr;
    status[d] = st;
  }
  if (stats) {
    double* sd = stats + (size_t)d * (Q + 2);
    if (tid < Q) sd[tid] = mu[tid];
    if (tid == Q) sd[Q] = sigma;
    if (tid == Q + 1) sd[Q + 1] = nval;
  }
}

template <int Q>
size_t lds_bytes(int Pseg, int K, int nw) {
  using L = Layout<Q>;
  const size_t nd = (size_t)Pseg * L::NS + L::NACC + 2 * Q + 16 + L::ND * (L::ND + 1) + L::ND +
                    2 * (size_t)Pseg * (L::ND + 1) + K + 1 + (size_t)nw * 8 * 65;
  return nd * sizeof(double);
}

template <int Q>
hipError_t launch_q(const float* X, const float* cap, const float* ret, const int16_t* ind,
                    XsDims dm, int nw, double* f, float* e, double* r2, double* stats,
                    int* status, hipStream_t s) {
  const size_t bytes = lds_bytes<Q>(dm.Pseg, 1 + dm.P + Q, nw);
  if (bytes > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xs_wls_kernel<Q>, dim3(dm.D), dim3(64 * nw), bytes, s, X, cap, ret, ind, dm,
                     f, e, r2, stats, status);
  return hipGetLastError();
}

}  // namespace

// X: [D][Q][N] fp32 styles, cap/ret: [D][N] fp32, ind: [D][N] int16 industry id (<0 = absent;
// may be null when P == 0).  Outputs: f [D][1+P+Q] fp64 (country, industries, styles),
// e [D][N] fp32 specific returns (nullable), r2 [D] fp64, stats [D][Q+2] fp64 = (mu_q, sigma,
// n_valid) (nullable), status [D] int32 bit flags (XsStatus).
// pivot_mode: 0 = last non-empty industry (default), 1 = always the last industry (reference).
// waves: waves per date-workgroup (1, 2, 4; 0 = auto from N).
MFA_API int mfa_xs_wls(const float* X, const float* cap, const float* ret, const int16_t* ind,
                       int D, int N, int P, int Q, int pivot_mode, double tol, int waves,
                       double* f, float* e, double* r2, double* stats, int* status,
                       void* stream) {
  if (D <= 0) return 0;
  if (Q < 1 || Q > 16 || P < 0 || P > 128 || N <= 0) return (int)hipErrorInvalidValue;
  XsDims dm;
  dm.D = D; dm.N = N; dm.P = P;
  dm.has_ind = P > 0 ? 1 : 0;
  dm.Pseg = P > 0 ? P : 1;
  dm.pivot_mode = pivot_mode;
  dm.tol = tol;
  int nw = waves;
  if (nw <= 0) nw = N >= 2048 ? 4 : (N >= 512 ? 2 : 1);
  if (nw != 1 && nw != 2 && nw != 4) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  switch (Q) {
#define MFA_Q(qq) \
  case qq: return (int)launch_q<qq>(X, cap, ret, ind, dm, nw, f, e, r2, stats, status, s);
    MFA_Q(1) MFA_Q(2) MFA_Q(3) MFA_Q(4) MFA_Q(5) MFA_Q(6) MFA_Q(7) MFA_Q(8)
    MFA_Q(9) MFA_Q(10) MFA_Q(11) MFA_Q(12) MFA_Q(13) MFA_Q(14) MFA_Q(15) MFA_Q(16)
#undef MFA_Q
  }
  return (int)hipErrorInvalidValue;
}
