// Monte-Carlo eigenfactor bias statistic for wide factor sets (64 < K <= 160) on gfx950.
//
// Reference: Barra-master/mfm/utils.py:55-92 (eigen_risk_adj), as csrc/eigen.hip: per (date,
// sim) the bias ratios v[k] = V[:,k]^T D0 V[:,k] / Lambda[k] of A = S C_z S (descending).
#include "common.h"
#include "tridiag.h"
#include "wide_gram.h"

namespace {

using namespace mfa;

// ---------------- multi-wave tridiagonal bias solver (64 < K <= 144) ----------------
// Wide factor sets (e.g. SW-L2 industries, K = 140) with mode 5's four phases and arithmetic on
// ONE workgroup of NW waves per (date, sim).  Layout 0 (mc_bias_wide_kernel, default for
// K <= 96): lane t owns row t of A = S C_z S in registers (KP doubles); layout 1
// (mc_bias_wide2_kernel below, default for K > 96): two lanes per row.  The packed reflector
// rows and the tridiagonal tables live in LDS (~87 KB at K = 140: one workgroup per CU).
// What changes against the one-wave kernel is only where lanes meet: the Householder column
// norm, u^T p and the Gershgorin / pivot bounds are block reductions (per-wave DPP totals, then
// the NW partials in wave order: deterministic), the pivot row's entries are LDS broadcasts, and
// every cross-wave LDS exchange is behind a barrier (2 per Householder step, each carrying one
// reduction's partials and one broadcast vector; 4 until round 6).  Replaces
// rocSOLVER's batched syevd (~27 us per 140 x 140 problem at the GPU's throughput) for the bias
// statistic; eigenvalues, eigenvectors and back-transform are per lane as before.
// Multisection rounds before the Laguerre loop: bits 4-6 of the kernels' `abl` argument
// (mfa_eigen_wide_set_ablation(r << 4)); 0 = off until measured (the Laguerre phase is ~1/3 of
// the K = 140 solver, profiles/r04/wide_bias_ab.jsonl).

template <int NW>
__device__ __forceinline__ double block_total(double v, double* red, int t) {
  v = wave_total(v);
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) s += red[w];
  return s;
}
template <int NW, bool MAX>
__device__ __forceinline__ double block_ext(double v, double* red, int t) {
  v = MAX ? wave_max(v) : wave_min(v);
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) s = MAX ? fmax(s, red[w]) : fmin(s, red[w]);
  return s;
}

template <int KP, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(1))) void
mc_bias_wide_kernel(const double* __restrict__ D0, int K, int M, const double* __restrict__ Cz,
                    const int* __restrict__ dvalid, double* __restrict__ vout, int abl) {
  static_assert(KP % 8 == 0 && KP <= NW * 64, "KP: multiple of 8, at most one row per lane");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int d = blockIdx.x / M, m = blockIdx.x % M, t = threadIdx.x;
  double* vo = vout + ((size_t)d * M + m) * K;
  if (!dvalid[d]) {
    for (int k = t; k < K; k += NW * 64) vo[k] = qnan();
    return;
  }
  const int nrow = (tri2_rows_doubles<KP>(K) + 1) & ~1;
  double* R = sm;                          // packed reflector rows
  double* wb = R + nrow;                   // [NW*64] broadcast p; Sturm counts later
  double* xb = wb + NW * 64;               // [NW*64] broadcast column s
  double2* tb = (double2*)(xb + NW * 64);  // [KP] {alpha_i, beta_{i-1}^2}
  double* be = (double*)(tb + KP);         // [KP] beta_i
  double* ta = be + KP;                    // [KP] tau_s
  double* dd = ta + KP;                    // [NW*64] sqrt(D0)
  double* gs = dd + NW * 64;               // [NW*64] diagonal of A, descending; Laguerre x later
  double* red = gs + NW * 64;              // [2][NW] block-reduction partials (double-buffered)
  double* bc = red + 2 * NW;               // [2] pivot-row broadcasts (alpha, x_{s+1})
  const int li = t < K ? t : 0;
  double a[KP];
  const double* c = Cz + (size_t)m * K * K;
  const double* d0 = D0 + (size_t)d * K;
  const double di = t < K ? sqrt(fmax(d0[t], 0.0)) : 0.0;
  dd[t] = di;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    a[j] = (j < K && t < K) ? di * c[j * K + li] * dd[j] : 0.0;
    if ((j & 7) == 7) lds_batch();
  }
  {
    const double g = t < K ? di * c[li * K + li] * di : 0.0;
    wb[t] = g;
    __syncthreads();
    if (t < K) {  // descending rank of the diagonal (ties by index): initial guesses
      int rank = 0;
      for (int j = 0; j < K; ++j) {
        const double h = wb[j];
        rank += (h > g) || (h == g && j < t);
      }
      gs[rank] = g;
    }
    __syncthreads();
  }
  // ---- 1. Householder tridiagonalisation (rows in registers, u broadcast from its row) ----
  auto steps = [&](auto J0c) {
    constexpr int J0 = decltype(J0c)::value;
    for (int s = J0; s < J0 + 8 && s < K; ++s) {
      double xs = a[J0];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (J0 + k < KP) {
          double tt = a[J0 + k];
          asm volatile("" : "+v"(tt));
          xs = s == J0 + k ? tt : xs;
        }
      const bool act = t > s && t < K;
      const double x = act ? xs : 0.0;
      xb[t] = x;
      if (t == s) bc[0] = xs;
      const double v = wave_total(t > s + 1 && t < K ? x * x : 0.0);
      if ((t & 63) == 0) red[t >> 6] = v;
      __syncthreads();  // A: column s, alpha, the sigma partials
      double sig = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) sig += red[w];
      const double alpha = bc[0], x0 = s + 1 < K ? xb[s + 1] : 0.0;
      double u = 0.0, tau = 0.0, beta = x0;
      if (sig != 0.0) {
        const double n2 = fma(x0, x0, sig);
        const double nrm = n2 * rsq_nr(n2);
        beta = x0 >= 0.0 ? -nrm : nrm;
        tau = rcp_nr(nrm * (nrm + fabs(x0)));
        u = act ? (t == s + 1 ? x0 - beta : x) : 0.0;
      }
      if (t == 0) {
        tb[s] = double2{alpha, s > 0 ? be[s - 1] * be[s - 1] : 0.0};
        be[s] = beta;
        ta[s] = tau;
      }
      if (s + 2 >= K) {  // no reflection (tau = 0)
        __syncthreads();
        continue;
      }
      double* us = R + tri2_row_off<KP>(s) - J0;  // us[j], j in [J0, KP)
      if (t >= J0 && t < KP) us[t] = u;
      double p0 = 0.0, p1 = 0.0;  // p = tau (A x - beta A[:, s+1]) = tau A u
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 xx = *(const double2*)(xb + j);
        p0 = fma(a[j], xx.x, p0);
        p1 = fma(a[j + 1], xx.y, p1);
        if (((j - J0) & 7) == 6) lds_batch();
      }
      double as1 = a[J0];  // column s + 1
#pragma unroll
      for (int k = 1; k < 9; ++k)
        if (J0 + k < KP) {
          double tt = a[J0 + k];
          asm volatile("" : "+v"(tt));
          as1 = s + 1 == J0 + k ? tt : as1;
        }
      const double p = act ? tau * fma(-beta, as1, p0 + p1) : 0.0;
      const double v2 = wave_total(u * p);
      if ((t & 63) == 0) red[NW + (t >> 6)] = v2;
      wb[t] = p;
      __syncthreads();  // B: p, the u^T p partials, the reflector row
      double up = red[NW];
#pragma unroll
      for (int w = 1; w < NW; ++w) up += red[NW + w];
      const double kk = 0.5 * tau * up;
      const double w2 = fma(-2.0 * kk, u, p);  // A -= u p^T + (p - 2 kk u) u^T
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 pp = *(const double2*)(wb + j), uu = *(const double2*)(us + j);
        a[j] = fma(-u, pp.x, fma(-w2, uu.x, a[j]));
        a[j + 1] = fma(-u, pp.y, fma(-w2, uu.y, a[j + 1]));
        if (((j - J0) & 7) == 6) lds_batch();
      }
      // no barrier after the update (mc_bias_wide2_kernel below has the hazard argument)
    }
  };
  if ((abl & 4) == 0) {
    [&]<int... G>(std::integer_sequence<int, G...>) {
      (steps(std::integral_constant<int, 8 * G>{}), ...);
    }(std::make_integer_sequence<int, KP / 8>{});
  } else {  // timing ablation: T = the sorted diagonal with a weak coupling, no reflectors
    const double g = gs[t];
    if (t < KP) {
      tb[t] = double2{g, t > 0 ? 1e-12 * g * g : 0.0};
      be[t] = 1e-6 * g;
      ta[t] = 0.0;
    }
    __syncthreads();
  }
  // ---- 2. eigenvalue of rank t (descending), as mode 5 ----
  double lo_l = 0.0, hi_l = 0.0, b2max = 0.0;
  if (t < K) {
    const double ad = tb[t].x;
    const double r = (t > 0 ? fabs(be[t - 1]) : 0.0) + (t + 1 < K ? fabs(be[t]) : 0.0);
    lo_l = ad - r;
    hi_l = ad + r;
    b2max = tb[t].y;
  } else {
    lo_l = tb[0].x;
    hi_l = tb[0].x;
  }
  const double gl = block_ext<NW, false>(lo_l, red, t);
  const double gu = block_ext<NW, true>(hi_l, red + NW, t);
  __syncthreads();
  const double b2 = block_ext<NW, true>(b2max, red, t);
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, b2);
  constexpr double kEps = 2.220446049250313e-16;
  const double abstol = kEps * tnorm + pivmin;  // LAPACK's accuracy (eigen.hip, mode 5)
  const int jt = K - 1 - t;
  double lo = gl - 2.0 * kEps * tnorm - pivmin, hi = gu + 2.0 * kEps * tnorm + pivmin;
  double x = t < K ? fmin(fmax(gs[t], lo), hi) : 0.5 * (lo + hi);
  double G = 0.0, H = 0.0;
  int cnt = sturm_gh_p(tb, K, x, G, H);
  __syncthreads();  // every lane has read its gs slot
  double* xsv = gs;
  int* csv = (int*)wb;
  xsv[t] = x;
  csv[t] = cnt;
  __syncthreads();
  for (int l = 0; l < K; ++l) {
    const double xl = xsv[l];
    const int cl = csv[l];
    if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
  }
  // multisection: every lane samples the count at its bracket's midpoint and every lane
  // tightens its bracket with all K samples (the diagonal is a poor guess when C_z is far from
  // the identity, e.g. T_sim ~ 2 K: the Laguerre loop otherwise starts with long bisections)
  for (int rd = 0; rd < ((abl >> 4) & 7); ++rd) {
    const double xm = 0.5 * (lo + hi);
    double Gm, Hm;
    const int cm = sturm_gh_p(tb, K, xm, Gm, Hm);
    __syncthreads();
    xsv[t] = xm;
    csv[t] = cm;
    __syncthreads();
    for (int l = 0; l < K; ++l) {
      const double xl = xsv[l];
      const int cl = csv[l];
      if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
    }
  }
  if ((abl >> 4) != 0 && !(x > lo && x < hi)) {  // the guess fell out: restart mid-bracket
    x = 0.5 * (lo + hi);
    cnt = sturm_gh_p(tb, K, x, G, H);
  }
  double lam = x;
  if (t < K && (abl & 1) == 0) {
    int prev = -1;
    double sprev = __builtin_inf();
    for (int it = 0; it < 512; ++it) {
      bool lag = false;
      double xn = 0.0;
      if (cnt == jt || cnt == jt + 1) {
        xn = laguerre_toward(x, G, H, K, cnt == jt);
        double st = fabs(xn - x);
        if (prev == cnt && st >= 1.5 * sprev) {
          xn = fma(8.0, xn - x, x);
          st *= 8.0;
        }
        lag = __builtin_isfinite(xn) && xn >= lo && xn <= hi;
        if (lag && prev == cnt && (st <= 1e-8 * fabs(x) || st <= abstol) && st <= 0.25 * sprev) {
          x = xn;
          break;
        }
        sprev = lag ? st : __builtin_inf();
      }
      if (!lag) { xn = 0.5 * (lo + hi); sprev = __builtin_inf(); }
      if (hi - lo <= 2.0 * kEps * (fabs(lo) + fabs(hi)) + abstol) { x = 0.5 * (lo + hi); break; }
      prev = lag ? cnt : -1;
      x = xn;
      cnt = sturm_gh_p(tb, K, x, G, H);
      if (cnt <= jt) lo = x; else hi = x;
    }
    lam = x;
  }
  if (abl & 2) {  // timing ablation: no eigenvectors / back-transform
    if (t < K) vo[t] = lam;
    return;
  }
  // ---- 3. eigenvector of T at lam: twisted factorisation in the y registers only ----
  double y[KP];
  if (t < K) {
    double dp = 0.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i < K) {
        const double2 tt = tb[i];
        dp = guard_pivot(i == 0 ? tt.x - lam : (tt.x - lam) - tt.y * rcp_nr1(dp), pivmin);
      }
      y[i] = i < K ? dp : 0.0;
    }
    double dm = 0.0, gmin = 0.0;
    int r = K - 1;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < K) {
        const double ai = tb[i].x - lam;
        dm = guard_pivot(i == K - 1 ? ai : ai - tb[i + 1].y * rcp_nr1(dm), pivmin);
        const double g = fabs(y[i] + dm - ai);
        if (i == K - 1 || g < gmin) { gmin = g; r = i; }
      }
    }
    double cz = 1.0, nrm = 1.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < r) {
        cz = -be[i] * cz * rcp_nr1(y[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
    }
    dm = 0.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < K && i > r) {
        const double ai = tb[i].x - lam;
        dm = guard_pivot(i == K - 1 ? ai : ai - tb[i + 1].y * rcp_nr1(dm), pivmin);
        y[i] = dm;
      }
    }
    cz = 1.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i == r) y[i] = 1.0;
      if (i > r && i < K) {
        cz = -be[i - 1] * cz * rcp_nr1(y[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
      if (i >= K) y[i] = 0.0;
    }
    const double sc = rsq_nr(nrm);
#pragma unroll
    for (int i = 0; i < KP; ++i) y[i] *= sc;
  } else {
#pragma unroll
    for (int i = 0; i < KP; ++i) y[i] = 0.0;
  }
  // ---- 4. back-transform with the packed reflector rows and the bias ratio ----
  auto back = [&](auto J0c, int s_hi) {
    constexpr int J0 = decltype(J0c)::value;
    for (int s = s_hi; s >= J0; --s) {
      if (s + 2 >= K) continue;
      const double tau = ta[s];
      if (tau == 0.0) continue;
      const double* us = R + tri2_row_off<KP>(s) - J0;
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        t0 = fma(uu.x, y[j], t0);
        t1 = fma(uu.y, y[j + 1], t1);
        if (((j - J0) & 7) == 6) lds_batch();
      }
      const double f = tau * (t0 + t1);
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        y[j] = fma(-f, uu.x, y[j]);
        y[j + 1] = fma(-f, uu.y, y[j + 1]);
        if (((j - J0) & 7) == 6) lds_batch();
      }
    }
  };
  [&]<int... G>(std::integer_sequence<int, G...>) {
    constexpr int NG = KP / 8;
    (back(std::integral_constant<int, 8 * (NG - 1 - G)>{}, 8 * (NG - 1 - G) + 7), ...);
  }(std::make_integer_sequence<int, KP / 8>{});
  if (t < K) {
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < KP; ++j)
      if (j < K) v = fma(dd[j] * dd[j], y[j] * y[j], v);
    vo[t] = v / lam;
  }
}

// ---------------- two lanes per row (wide variant 1) ----------------
// The row-per-lane kernel needs 2 x KP registers for a 144-column row (a, then y): 32+ of them
// live in AGPRs and the eigenvector phase spills to scratch, at one 3-wave workgroup per CU.
// Here lanes 2i and 2i+1 share row i: lane half h holds columns [h HP, h HP + HP) (HP = KP / 2)
// of the row in phase 1 and entries [h HP, h HP + HP) of the eigenvector in phases 3-4, so a lane
// keeps HP = 72 doubles.  Row-level scalars (x, u, p, w, the eigenvalue) are computed by both
// lanes of a pair with identical arithmetic; partial dot products over the two halves are
// summed with one DPP lane swap (a + b == b + a bitwise); sequential recurrences that cross
// the halves (the eigenvector below / above the twist) run over the upper / lower half in turn
// and hand their carry to the partner lane.  Same operations in the same order as the
// row-per-lane kernel except the two-half split of each dot product.
__device__ __forceinline__ double pair_swap(double v) { return dpp_mov<0xB1>(v); }  // lane ^ 1
__device__ __forceinline__ int pair_swap_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
}

// EIG: batched symmetric eigendecomposition with the same machinery (eigh of wide F0): D0 = the
// input matrices [B][K][K] (symmetrised), M = 1, vout = w [B][K] descending, Uout [B][K][K]
// with U[:, k] = eigenvector k; a matrix with a non-finite entry gives NaN.  The caller checks
// U^T U = I (clustered spectra) and re-solves what fails.
template <int KP, int NW, bool EIG = false>
__global__ __launch_bounds__(NW * 64) void mc_bias_wide2_kernel(
    const double* __restrict__ D0, int K, int M, const double* __restrict__ Cz,
    const int* __restrict__ dvalid, double* __restrict__ vout, int abl,
    double* __restrict__ Uout = nullptr) {
  constexpr int HP = KP / 2;
  static_assert(KP % 16 == 0 && KP <= NW * 32, "KP: multiple of 16, two lanes per row");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int d = blockIdx.x / M, m = blockIdx.x % M, t = threadIdx.x;
  const int i = t >> 1, h = t & 1;  // row, half
  double* vo = vout + ((size_t)d * M + m) * K;
  const double* Ain = D0 + (size_t)d * K * K;  // EIG input matrix
  if constexpr (EIG) {
    bool fin = true;
    for (int e = t; e < K * K; e += NW * 64) fin = fin && __builtin_isfinite(Ain[e]);
    double* redx = sm;  // before any other use of the LDS
    if (block_total<NW>(fin ? 0.0 : 1.0, redx, t) != 0.0) {
      for (int k = t; k < K; k += NW * 64) vo[k] = qnan();
      for (int e = t; e < K * K; e += NW * 64) Uout[(size_t)d * K * K + e] = qnan();
      return;
    }
    __syncthreads();  // the partials slot is reused as reflector storage below
  } else if (!dvalid[d]) {
    for (int k = t; k < K; k += NW * 64) vo[k] = qnan();
    return;
  }
  const int nrow = (tri2_rows_doubles<KP>(K) + 1) & ~1;
  double* R = sm;                          // packed reflector rows (column-interleaved halves)
  double* wb = R + nrow;                   // [KP] broadcast p (interleaved); Sturm counts later
  double* xb = wb + KP;                    // [KP] broadcast column s (interleaved)
  double2* tb = (double2*)(xb + KP);       // [KP] {alpha_i, beta_{i-1}^2}
  double* be = (double*)(tb + KP);         // [KP] beta_i
  double* ta = be + KP;                    // [KP] tau_s
  double* dd = ta + KP;                    // [KP] sqrt(D0)
  double* gs = dd + KP;                    // [KP] diagonal of A, descending; Laguerre x later
  double* red = gs + KP;                   // [2][NW] block-reduction partials
  double* bc = red + 2 * NW;               // [2] pivot-row broadcasts
  const bool row_ok = i < K;
  const int li = row_ok ? i : 0;
  const bool lead = h == 0 && i < KP;      // the lane that writes row-indexed LDS slots
  double a[HP];
  const double* c = Cz + (size_t)m * K * K;
  const double* d0 = D0 + (size_t)d * K;
  const double di = (row_ok && !EIG) ? sqrt(fmax(d0[li], 0.0)) : 0.0;
  if (lead) dd[i] = di;
  __syncthreads();
#pragma unroll
  for (int jj = 0; jj < HP; ++jj) {
    const int j = 2 * jj + h;  // phase 1: lane h holds the columns of parity h
    if constexpr (EIG)  // this lane's half of row i of the symmetrised input
      a[jj] = (j < K && row_ok) ? 0.5 * (Ain[li * K + j] + Ain[j * K + li]) : 0.0;
    else
      a[jj] = (j < K && row_ok) ? di * c[j * K + li] * dd[j] : 0.0;
    if ((jj & 7) == 7) lds_batch();
  }
  {
    const double g = row_ok ? (EIG ? Ain[li * K + li] : di * c[li * K + li] * di) : 0.0;
    if (lead) wb[i] = g;
    __syncthreads();
    if (lead && row_ok) {
      int rank = 0;
      for (int j = 0; j < K; ++j) {
        const double q = wb[j];
        rank += (q > g) || (q == g && j < i);
      }
      gs[rank] = g;
    }
    __syncthreads();
  }
  // ---- 1. Householder tridiagonalisation ----
  // Lane h holds the columns j = 2 jj + h of its row (register jj), so both lanes of a pair keep
  // (KP - s) / 2 live columns at step s: the loops below run over registers [J0 / 2, HP) instead
  // of a contiguous half that stays whole until s passes HP.  Vectors broadcast through the LDS
  // (the column x, p, the reflector rows) are stored de-interleaved, entry j at
  // (j & 1) * half + (j >> 1), so a lane reads its parity's entries as contiguous double2.
  // Two barriers per step, each carrying a block reduction:
  //   A: column s (x, rows > s) and the partials of sigma = |x_{s+2..}|^2;
  //   B: p = tau A u and the partials of u^T p.
  // u differs from x only at s + 1 (u_{s+1} = x_{s+1} - beta), so p = tau (A x - beta A[:, s+1])
  // is formed from the broadcast x before u is published; the reflector row u (written after A)
  // feeds the rank-2 update after B, in the form A -= u p^T + (p - 2 kk u) u^T
  // (= u w^T + w u^T with w = p - kk u, kk = tau u^T p / 2: no per-element w).
  // No barrier after the update: every LDS slot a step writes before its barrier A (x, alpha, the
  // sigma partials) was last read before the previous step's barrier B, and the slots it writes
  // between A and B (p, the u^T p partials, its reflector row) were last read after the previous
  // B, which no wave leaves behind before reaching this A.
  auto steps = [&](auto J0c) {
    constexpr int J0 = decltype(J0c)::value;
    constexpr int JH = J0 / 2;          // first register holding a column >= J0
    constexpr int L2 = (KP - J0) / 2;   // half length of the packed reflector rows of group J0
    for (int s = J0; s < J0 + 8 && s < K; ++s) {
      double xo = a[JH];  // column 2 (s >> 1) + h
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        double tt = a[JH + k];
        asm volatile("" : "+v"(tt));
        xo = (s >> 1) == JH + k ? tt : xo;
      }
      const double xp = pair_swap(xo);
      const double xs = h == (s & 1) ? xo : xp;  // column s of row i, on both lanes of the pair
      const bool act = i > s && row_ok;
      const double x = act ? xs : 0.0;
      if (lead) xb[(i & 1) * HP + (i >> 1)] = x;
      if (t == 2 * s) bc[0] = xs;
      double v = wave_total(h == 0 && i > s + 1 && row_ok ? x * x : 0.0);
      if ((t & 63) == 0) red[t >> 6] = v;
      __syncthreads();  // A
      double sig = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) sig += red[w];
      const double alpha = bc[0];
      const double x0 = s + 1 < K ? xb[((s + 1) & 1) * HP + ((s + 1) >> 1)] : 0.0;
      double u = 0.0, tau = 0.0, beta = x0;
      if (sig != 0.0) {
        const double n2 = fma(x0, x0, sig);
        const double nrm = n2 * rsq_nr(n2);
        beta = x0 >= 0.0 ? -nrm : nrm;
        tau = rcp_nr(nrm * (nrm + fabs(x0)));
        u = act ? (i == s + 1 ? x0 - beta : x) : 0.0;
      }
      if (t == 0) {
        tb[s] = double2{alpha, s > 0 ? be[s - 1] * be[s - 1] : 0.0};
        be[s] = beta;
        ta[s] = tau;
      }
      if (s + 2 >= K) {  // x has at most one entry: no reflection (tau = 0)
        __syncthreads();  // the next step's x / partials overwrite what this step read after A
        continue;
      }
      double* us = R + tri2_row_off<KP>(s);  // entries j in [J0, KP), de-interleaved
      if (lead && i >= J0) us[(i & 1) * L2 + ((i - J0) >> 1)] = u;
      const double* xh = xb + h * HP;
      double p0 = 0.0, p1 = 0.0;
#pragma unroll
      for (int jj = JH; jj < HP; jj += 2) {
        const double2 xx = *(const double2*)(xh + jj);
        p0 = fma(a[jj], xx.x, p0);
        p1 = fma(a[jj + 1], xx.y, p1);
        if (((jj - JH) & 7) == 6) lds_batch();
      }
      double yo = a[JH];  // column s + 1 of row i
#pragma unroll
      for (int k = 1; k < 5; ++k)
        if (JH + k < HP) {
          double tt = a[JH + k];
          asm volatile("" : "+v"(tt));
          yo = ((s + 1) >> 1) == JH + k ? tt : yo;
        }
      const double yp = pair_swap(yo);
      const double as1 = h == ((s + 1) & 1) ? yo : yp;
      const double pl = p0 + p1, pr = pair_swap(pl);
      const double p = act ? tau * fma(-beta, as1, h ? pr + pl : pl + pr) : 0.0;
      double v2 = wave_total(h == 0 ? u * p : 0.0);
      if ((t & 63) == 0) red[NW + (t >> 6)] = v2;
      if (lead) wb[(i & 1) * HP + (i >> 1)] = p;
      __syncthreads();  // B
      double up = red[NW];
#pragma unroll
      for (int w = 1; w < NW; ++w) up += red[NW + w];
      const double kk = 0.5 * tau * up;
      const double w2 = fma(-2.0 * kk, u, p);
      const double* ph = wb + h * HP;
      const double* uh = us + h * L2 - JH;
#pragma unroll
      for (int jj = JH; jj < HP; jj += 2) {
        const double2 pp = *(const double2*)(ph + jj);
        const double2 uu = *(const double2*)(uh + jj);
        a[jj] = fma(-u, pp.x, fma(-w2, uu.x, a[jj]));
        a[jj + 1] = fma(-u, pp.y, fma(-w2, uu.y, a[jj + 1]));
        if (((jj - JH) & 7) == 6) lds_batch();
      }
    }
  };
  if ((abl & 4) == 0) {
    [&]<int... G>(std::integer_sequence<int, G...>) {
      (steps(std::integral_constant<int, 8 * G>{}), ...);
    }(std::make_integer_sequence<int, KP / 8>{});
  } else {
    if (lead) {
      const double g = gs[i];
      tb[i] = double2{g, i > 0 ? 1e-12 * g * g : 0.0};
      be[i] = 1e-6 * g;
      ta[i] = 0.0;
    }
    __syncthreads();
  }
  // T padded to KP with decoupled rows (alpha = 1e300, beta = 0): the eigenvector recurrences
  // below run over all KP entries without per-entry K tests (their unrolled K masks otherwise
  // overflow the scalar registers); the padded pivots are ~1e300, their twist candidates never
  // win and their eigenvector entries come out 0 (beta = 0).  Sturm counts still use K.
  if (lead && i >= K) {
    tb[i] = double2{1e300, 0.0};
    be[i] = 0.0;
  }
  if (t == 0) be[K - 1] = 0.0;
  // ---- 2. eigenvalue of rank i (descending), both lanes of the pair ----
  double lo_l = 0.0, hi_l = 0.0, b2max = 0.0;
  if (row_ok) {
    const double ad = tb[i].x;
    const double r = (i > 0 ? fabs(be[i - 1]) : 0.0) + (i + 1 < K ? fabs(be[i]) : 0.0);
    lo_l = ad - r;
    hi_l = ad + r;
    b2max = tb[i].y;
  } else {
    lo_l = tb[0].x;
    hi_l = tb[0].x;
  }
  const double gl = block_ext<NW, false>(lo_l, red, t);
  const double gu = block_ext<NW, true>(hi_l, red + NW, t);
  __syncthreads();
  const double b2 = block_ext<NW, true>(b2max, red, t);
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, b2);
  constexpr double kEps = 2.220446049250313e-16;
  // LAPACK's absolute eigenvalue accuracy eps ||T|| (eigen.hip, mode 5); abl bit 8 clear on
  // the F0 eigh (mfa_eigen_wide_set_eig_abstol(0), A/B) restores round 4's 1e-22 ||T||
  const double abstol = ((EIG && !(abl & 256)) ? 1e-22 * tnorm : kEps * tnorm) + pivmin;
  const int jt = K - 1 - i;
  double lo = gl - 2.0 * kEps * tnorm - pivmin, hi = gu + 2.0 * kEps * tnorm + pivmin;
  double x = row_ok ? fmin(fmax(gs[li], lo), hi) : 0.5 * (lo + hi);
  double G = 0.0, H = 0.0;
  int cnt = sturm_gh_p(tb, K, x, G, H);
  __syncthreads();
  double* xsv = gs;
  int* csv = (int*)wb;
  if (lead) {
    xsv[i] = x;
    csv[i] = cnt;
  }
  __syncthreads();
  for (int l = 0; l < K; ++l) {
    const double xl = xsv[l];
    const int cl = csv[l];
    if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
  }
  for (int rd = 0; rd < ((abl >> 4) & 7); ++rd) {  // multisection, as in the row kernel
    const double xm = 0.5 * (lo + hi);
    double Gm, Hm;
    const int cm = sturm_gh_p(tb, K, xm, Gm, Hm);
    __syncthreads();
    if (lead) {
      xsv[i] = xm;
      csv[i] = cm;
    }
    __syncthreads();
    for (int l = 0; l < K; ++l) {
      const double xl = xsv[l];
      const int cl = csv[l];
      if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
    }
  }
  if ((abl >> 4) != 0 && !(x > lo && x < hi)) {
    x = 0.5 * (lo + hi);
    cnt = sturm_gh_p(tb, K, x, G, H);
  }
  double lam = x;
  if (row_ok && (abl & 1) == 0) {
    int prev = -1;
    double sprev = __builtin_inf();
    for (int it = 0; it < 512; ++it) {
      bool lag = false;
      double xn = 0.0;
      if (cnt == jt || cnt == jt + 1) {
        xn = laguerre_toward(x, G, H, K, cnt == jt);
        double st = fabs(xn - x);
        if (prev == cnt && st >= 1.5 * sprev) {
          xn = fma(8.0, xn - x, x);
          st *= 8.0;
        }
        lag = __builtin_isfinite(xn) && xn >= lo && xn <= hi;
        if (lag && prev == cnt && (st <= 1e-8 * fabs(x) || ((!EIG || (abl & 256)) && st <= abstol)) &&
            st <= 0.25 * sprev) { x = xn; break; }
        sprev = lag ? st : __builtin_inf();
      }
      if (!lag) { xn = 0.5 * (lo + hi); sprev = __builtin_inf(); }
      if (hi - lo <= 2.0 * kEps * (fabs(lo) + fabs(hi)) + abstol) { x = 0.5 * (lo + hi); break; }
      prev = lag ? cnt : -1;
      x = xn;
      cnt = sturm_gh_p(tb, K, x, G, H);
      if (cnt <= jt) lo = x; else hi = x;
    }
    lam = x;
  }
  if (!EIG && (abl & 2)) {
    if (lead && row_ok) vo[i] = lam;
    return;
  }
  // ---- 3. eigenvector of T at lam, entries [h HP, h HP + HP) in this lane ----
  double y[HP];
  double nrm = 0.0;  // this half's sum of squares, the twist entry's 1 added at the end
  {
    // forward pivots of the whole recurrence, kept for this half
    double dp = 0.0;
#pragma unroll
    for (int q = 0; q < KP; ++q) {
      const double2 tt = tb[q];
      dp = guard_pivot(q == 0 ? tt.x - lam : (tt.x - lam) - tt.y * rcp_nr1(dp), pivmin);
      if (q < HP) y[q] = h == 0 ? dp : y[q];
      else y[q - HP] = h == 1 ? dp : y[q - HP];
      if ((q & 3) == 3) lds_batch();  // the table loads stay 4 steps ahead, not 144
    }
    // backward pivots of the whole recurrence; the twist candidates of this half
    double dm = 0.0, gmin = __builtin_inf();
    int r = -1;
#pragma unroll
    for (int q = KP - 1; q >= 0; --q) {
      const double ai = tb[q].x - lam;
      dm = guard_pivot(q == KP - 1 ? ai : ai - tb[q + 1].y * rcp_nr1(dm), pivmin);
      const bool mine = (q < HP) == (h == 0);
      const double yq = q < HP ? y[q] : y[q - HP];
      const double g = fabs(yq + dm - ai);
      if (mine && (r < 0 || g < gmin)) { gmin = g; r = q; }
      if ((q & 3) == 0) lds_batch();
    }
    // the pair's twist: the upper half's candidate wins ties (the descending scan meets it first)
    const double go = pair_swap(gmin);
    const int ro = pair_swap_i(r);
    const double gu2 = h ? gmin : go, gl2 = h ? go : gmin;
    const int ru2 = h ? r : ro, rl2 = h ? ro : r;
    r = (ru2 >= 0 && !(gl2 < gu2)) || rl2 < 0 ? ru2 : rl2;
    // below the twist, descending: the upper half first, its carry handed to the lower half
    double cz = 1.0;
#pragma unroll
    for (int q = KP - 1; q >= HP; --q) {
      if (h == 1 && q < r) {
        cz = -be[q] * cz * rcp_nr1(y[q - HP]);
        nrm = fma(cz, cz, nrm);
        y[q - HP] = cz;
      }
      if ((q & 3) == 0) lds_batch();
    }
    {
      const double cu = pair_swap(cz);
      if (h == 0) cz = r > HP ? cu : 1.0;
    }
#pragma unroll
    for (int q = HP - 1; q >= 0; --q) {
      if (h == 0 && q < r) {
        cz = -be[q] * cz * rcp_nr1(y[q]);
        nrm = fma(cz, cz, nrm);
        y[q] = cz;
      }
      if ((q & 3) == 0) lds_batch();
    }
    // above the twist: backward pivots into this half's slots
    dm = 0.0;
#pragma unroll
    for (int q = KP - 1; q >= 0; --q) {
      if (q > r) {
        const double ai = tb[q].x - lam;
        dm = guard_pivot(q == KP - 1 ? ai : ai - tb[q + 1].y * rcp_nr1(dm), pivmin);
        if (q < HP) y[q] = h == 0 ? dm : y[q];
        else y[q - HP] = h == 1 ? dm : y[q - HP];
      }
      if ((q & 3) == 0) lds_batch();
    }
    // ascending from the twist: the lower half first, its carry handed to the upper half
    cz = 1.0;
#pragma unroll
    for (int q = 0; q < HP; ++q) {
      if (h == 0) {
        if (q == r) y[q] = 1.0;
        if (q > r) {
          cz = -be[q - 1] * cz * rcp_nr1(y[q]);
          nrm = fma(cz, cz, nrm);
          y[q] = cz;
        }
      }
      if ((q & 3) == 3) lds_batch();
    }
    {
      const double cl = pair_swap(cz);
      if (h == 1) cz = r < HP ? cl : 1.0;
    }
#pragma unroll
    for (int q = HP; q < KP; ++q) {
      if (h == 1) {
        if (q == r) y[q - HP] = 1.0;
        if (q > r) {
          cz = -be[q - 1] * cz * rcp_nr1(y[q - HP]);
          nrm = fma(cz, cz, nrm);
          y[q - HP] = cz;
        }
      }
      if ((q & 3) == 3) lds_batch();
    }
    const double no = pair_swap(nrm);
    const double sc = rsq_nr(1.0 + (h ? no + nrm : nrm + no));
#pragma unroll
    for (int q = 0; q < HP; ++q) y[q] *= sc;
    if (!row_ok) {
#pragma unroll
      for (int q = 0; q < HP; ++q) y[q] = 0.0;
    }
    // to the reflector rows' interleaved layout, in place: lane h trades the entries of the other
    // parity with its partner, after which register 2 m holds entry 2 m + h and register 2 m + 1
    // entry HP + 2 m + h (interleaved position jj at register yr(jj) below)
#pragma unroll
    for (int m = 0; m < HP / 2; ++m) {
      const double rv = pair_swap(h ? y[2 * m] : y[2 * m + 1]);
      if (h) y[2 * m] = rv; else y[2 * m + 1] = rv;
      __builtin_amdgcn_sched_barrier(0);  // one pair at a time (no register pressure spike)
    }
  }
  // ---- 4. back-transform (interleaved, as phase 1) and the bias ratio ----
  constexpr auto yr = [](int jj) { return jj < HP / 2 ? 2 * jj : 2 * (jj - HP / 2) + 1; };
  auto back = [&](auto J0c, int s_hi) {
    constexpr int J0 = decltype(J0c)::value;
    constexpr int JH = J0 / 2, L2 = (KP - J0) / 2;
    for (int s = s_hi; s >= J0; --s) {
      if (s + 2 >= K) continue;
      const double tau = ta[s];
      if (tau == 0.0) continue;
      const double* uh = R + tri2_row_off<KP>(s) + h * L2 - JH;
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int jj = JH; jj < HP; jj += 2) {
        const double2 uu = *(const double2*)(uh + jj);
        t0 = fma(uu.x, y[yr(jj)], t0);
        t1 = fma(uu.y, y[yr(jj + 1)], t1);
        if (((jj - JH) & 7) == 6) lds_batch();
      }
      const double tl = t0 + t1, tr = pair_swap(tl);
      const double f = tau * (h ? tr + tl : tl + tr);
#pragma unroll
      for (int jj = JH; jj < HP; jj += 2) {
        const double2 uu = *(const double2*)(uh + jj);
        y[yr(jj)] = fma(-f, uu.x, y[yr(jj)]);
        y[yr(jj + 1)] = fma(-f, uu.y, y[yr(jj + 1)]);
        if (((jj - JH) & 7) == 6) lds_batch();
      }
    }
  };
  [&]<int... G>(std::integer_sequence<int, G...>) {
    constexpr int NG = KP / 8;
    (back(std::integral_constant<int, 8 * (NG - 1 - G)>{}, 8 * (NG - 1 - G) + 7), ...);
  }(std::make_integer_sequence<int, KP / 8>{});
  if constexpr (EIG) {  // w (descending by row rank) and U[:, i] = eigenvector i
    if (row_ok) {
      if (h == 0) vo[i] = lam;
      double* Ub = Uout + (size_t)d * K * K;
#pragma unroll
      for (int jj = 0; jj < HP; ++jj) {
        const int j = 2 * jj + h;
        if (j < K) Ub[(size_t)j * K + i] = y[yr(jj)];
      }
    }
    return;
  }
  double v = 0.0;
#pragma unroll
  for (int jj = 0; jj < HP; ++jj) {
    const double dj = dd[2 * jj + h];  // 0 for the padded entries
    v = fma(dj * dj, y[yr(jj)] * y[yr(jj)], v);
    if ((jj & 7) == 7) lds_batch();
  }
  const double vo2 = pair_swap(v);
  if (lead && row_ok) vo[i] = (v + vo2) / lam;
}

size_t bias_wide2_lds(int K, int KP, int NW) {
  int n = 0;
  for (int s = 0; s + 2 < K; ++s) n += KP - 8 * (s / 8);
  return ((size_t)((n + 1) & ~1) + 8 * KP + 2 * NW + 2) * sizeof(double);
}

size_t bias_wide_lds(int K, int KP, int NW) {
  int n = 0;
  for (int s = 0; s + 2 < K; ++s) n += KP - 8 * (s / 8);
  return ((size_t)((n + 1) & ~1) + 2 * NW * 64 + 2 * KP + 2 * KP + 3 * NW * 64 + 2 * NW + 2) *
         sizeof(double);
}


__global__ __launch_bounds__(64) void wide_bias_sum_kernel(const double* __restrict__ vin, int K,
                                                           int M, double* __restrict__ S) {
  const int d = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += 64) {
    double s = 0.0;
    for (int m = 0; m < M; ++m) s += vin[((size_t)d * M + m) * K + k];
    S[(size_t)d * K + k] += s;
  }
}

// ---------------- wide eigh: orthogonality check + device Jacobi re-solve ----------------
// After the tridiagonal EIG kernel, one 256-thread workgroup per matrix: err = max |U^T U - I|
// from the fp64 matrix cores (wide_gram_block over 64-row blocks of U), and a matrix with a
// finite input and !(err <= tol) -- non-orthogonal twisted-factorisation vectors of a clustered
// spectrum, or a NaN from a solver failure on a finite matrix -- is re-solved in place by a
// cyclic round-robin Jacobi: A (symmetrised) in the scratch `ws` [B][K][K], V in U itself, both
// global (L2-resident while the workgroup runs).  Replaces the host-side U^T U check, the
// torch.nonzero host sync and the rocSOLVER re-solve of round 4; matrices that pass exit after
// the check.  Deterministic (fixed rotation order, no atomics).
// Rotation of pair (p, q), zeroing A_pq: J_pp = J_qq = c, J_pq = s, J_qp = -s
// (Golub-Van Loan sym.schur2); A <- J^T A J on 2 x 2 pair blocks, V <- V J.
template <int KP>
__global__ __launch_bounds__(256) void eigh_wide_fix_kernel(const double* __restrict__ Ain, int K,
                                                            double tol, double psd_tol,
                                                            double* __restrict__ w,
                                                            double* __restrict__ U,
                                                            double* __restrict__ ws,
                                                            int* __restrict__ fixed) {
  using G = WideCov<KP>;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ double Z[64][KP + 2];
  __shared__ double red[4];
  __shared__ double cs_c[KP / 2 + 1], cs_s[KP / 2 + 1];
  __shared__ int idx[KP + 2];
  const double* A = Ain + (size_t)b * K * K;
  double* Ub = U + (size_t)b * K * K;
  double* S = ws + (size_t)b * K * K;
  bool fin = true;
  for (int e = tid; e < K * K; e += 256) fin = fin && __builtin_isfinite(A[e]);
  if (block_total<4>(fin ? 0.0 : 1.0, red, tid) != 0.0) {  // the EIG kernel wrote NaN already
    if (tid == 0 && fixed) fixed[b] = 0;
    return;
  }
  // ---- err = max |U^T U - I| ----
  f64x4g acc[G::TPW];
#pragma unroll
  for (int u = 0; u < G::TPW; ++u) acc[u] = f64x4g{0.0, 0.0, 0.0, 0.0};
  for (int r0 = 0; r0 < K; r0 += 64) {
    __syncthreads();
    for (int e = tid; e < 64 * KP; e += 256) {
      const int r = e / KP, c = e - r * KP;
      Z[r][c] = (r0 + r < K && c < K) ? Ub[(size_t)(r0 + r) * K + c] : 0.0;
    }
    __syncthreads();
    wide_gram_block<KP>(Z, wv, lane, acc);
  }
  double err = 0.0;
#pragma unroll
  for (int u = 0; u < G::TPW; ++u) {
    const int t = wv + G::NW * u;
    if (t < G::NT) {
      const int ti = G::ti(t), tj = G::tj(t);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 16 * ti + (lane >> 4) + 4 * e, j = 16 * tj + (lane & 15);
        if (i < K && j < K) {
          const double g = fabs(acc[u][e] - (i == j ? 1.0 : 0.0));
          err = (g > err || g != g) ? g : err;  // NaN propagates
        }
      }
    }
  }
  err = block_ext<4, true>(err != err ? INFINITY : err, red, tid);
  if (err <= tol) {
    if (tid == 0 && fixed) fixed[b] = 0;
    return;
  }
  // psd_tol >= 0 (the eigen adjustment): an indefinite matrix is an invalid date whose
  // eigenvectors are never read -- flagged 2, not re-solved (uniform: w is global)
  if (psd_tol >= 0.0 && w[(size_t)b * K + K - 1] < -psd_tol * fabs(w[(size_t)b * K])) {
    if (tid == 0 && fixed) fixed[b] = 2;
    return;
  }
  // ---- Jacobi re-solve ----
  const int Ke = K + (K & 1), np = Ke / 2;
  for (int e = tid; e < K * K; e += 256) {
    const int i = e / K, j = e - i * K;
    S[e] = 0.5 * (A[e] + A[(size_t)j * K + i]);
    Ub[e] = i == j ? 1.0 : 0.0;
  }
  for (int k = tid; k < Ke; k += 256) idx[k] = k;
  __syncthreads();
  auto at = [&](int i, int j) -> double { return (i < K && j < K) ? S[(size_t)i * K + j] : 0.0; };
  for (int sweep = 0; sweep < 40; ++sweep) {
    double nrot = 0.0;
    for (int round = 0; round < Ke - 1; ++round) {
      for (int i = tid; i < np; i += 256) {
        int p = idx[i], q = idx[Ke - 1 - i];
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        if (q < K) {
          const double apq = at(p, q), app = at(p, p), aqq = at(q, q);
          if (fabs(apq) > 1e-300 && fabs(apq) > 1e-17 * sqrt(fabs(app) * fabs(aqq))) {
            const double tau = (aqq - app) / (2.0 * apq);
            const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
            c = 1.0 / sqrt(1.0 + t * t);
            s = t * c;
            nrot += 1.0;
          }
        }
        cs_c[i] = c;
        cs_s[i] = s;
      }
      __syncthreads();
      for (int e = tid; e < np * np; e += 256) {  // A <- J^T A J, one 2 x 2 pair block each
        const int bi = e / np, bj = e - bi * np;
        int p = idx[bi], q = idx[Ke - 1 - bi], r = idx[bj], t = idx[Ke - 1 - bj];
        if (p > q) { const int x = p; p = q; q = x; }
        if (r > t) { const int x = r; r = t; t = x; }
        const double ci = cs_c[bi], si = cs_s[bi], cj = cs_c[bj], sj = cs_s[bj];
        if (si == 0.0 && sj == 0.0) continue;
        const double b00 = at(p, r), b01 = at(p, t), b10 = at(q, r), b11 = at(q, t);
        const double x00 = ci * b00 - si * b10, x01 = ci * b01 - si * b11;
        const double x10 = si * b00 + ci * b10, x11 = si * b01 + ci * b11;
        double y00 = cj * x00 - sj * x01, y01 = sj * x00 + cj * x01;
        double y10 = cj * x10 - sj * x11, y11 = sj * x10 + cj * x11;
        if (bi == bj) { y01 = 0.0; y10 = 0.0; }
        if (p < K && r < K) S[(size_t)p * K + r] = y00;
        if (p < K && t < K) S[(size_t)p * K + t] = y01;
        if (q < K && r < K) S[(size_t)q * K + r] = y10;
        if (q < K && t < K) S[(size_t)q * K + t] = y11;
      }
      for (int e = tid; e < K * np; e += 256) {  // V <- V J
        const int r = e / np, i = e - r * np;
        const double c = cs_c[i], s = cs_s[i];
        if (s == 0.0) continue;
        int p = idx[i], q = idx[Ke - 1 - i];
        if (p > q) { const int x = p; p = q; q = x; }
        const double vp = Ub[(size_t)r * K + p], vq = Ub[(size_t)r * K + q];
        Ub[(size_t)r * K + p] = c * vp - s * vq;
        Ub[(size_t)r * K + q] = s * vp + c * vq;
      }
      __syncthreads();
      if (tid == 0) {  // round-robin: position 0 fixed, the others shift by one
        const int last = idx[Ke - 1];
        for (int k = Ke - 1; k > 1; --k) idx[k] = idx[k - 1];
        idx[1] = last;
      }
      __syncthreads();
    }
    if (block_total<4>(nrot, red, tid) == 0.0) break;
    __syncthreads();
  }
  // ---- eigenvalues descending, eigenvectors permuted to match (via the scratch) ----
  for (int k = tid; k < K; k += 256) {
    const double dk = S[(size_t)k * K + k];
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const double dj = S[(size_t)j * K + j];
      rank += (dj > dk) || (dj == dk && j < k);
    }
    idx[k] = rank;
    w[(size_t)b * K + rank] = dk;
  }
  __syncthreads();
  for (int e = tid; e < K * K; e += 256) {
    const int r = e / K, k = e - r * K;
    S[(size_t)r * K + idx[k]] = Ub[e];
  }
  __syncthreads();
  for (int e = tid; e < K * K; e += 256) Ub[e] = S[e];
  if (tid == 0 && fixed) fixed[b] = 1;
}

}  // namespace

// Wide factor sets: S[d][k] += sum over this call's M sims of v_m[d][k] for 2 < K <= 144 with the
// multi-wave solver (one workgroup of 2 / 3 waves per (date, sim) for K <= 96 / 144); ws: D*M*K
// doubles.  Invalid dates (dvalid[d] = 0) accumulate NaN.
// Batched eigendecomposition of symmetric [B][K][K] matrices, 64 < K <= 144 (two lanes per row,
// 3 / 5 waves for K <= 96 / 144): w [B][K] descending, U [B][K][K] with U[:, k] = eigenvector k
// (NaN for non-finite inputs); then eigh_wide_fix_kernel checks U^T U = I to `tol` and re-solves
// the matrices that fail with the Jacobi (ws: B*K*K doubles; fixed [B] nullable: 1 = re-solved,
// 2 = not re-solved: psd_tol >= 0 and an eigenvalue below -psd_tol lambda_max).
// Multisection rounds of the F0 eigh before its Laguerre loop (A/B knob; 0 = off).  F0 is not
// diagonally dominant (a Newey-West covariance), so the diagonal guesses are poorer than for
// the bias problems S C_z S.
int g_wide_eig_rounds = 0;
// 1 (default) = LAPACK's absolute eigenvalue accuracy eps ||T|| for the F0 eigh; 0 = resolve the
// smallest eigenvalues to 1e-22 ||T|| (round 4): K = 140 3.93 -> 1.24 ms, K = 80 2.31 -> 0.42 ms
// for the risk model's 112 / 172 Newey-West covariances, the same errors against LAPACK
// (profiles/r05/r05l)
int g_wide_eig_abstol = 1;
MFA_API int mfa_eigen_wide_set_eig_abstol(int on) {
  if (on != 0 && on != 1) return (int)hipErrorInvalidValue;
  g_wide_eig_abstol = on;
  return 0;
}
MFA_API int mfa_eigen_wide_set_eig_rounds(int r) {
  if (r < 0 || r > 7) return (int)hipErrorInvalidValue;
  g_wide_eig_rounds = r;
  return 0;
}

MFA_API int mfa_eigh_wide_fix_psd(const double* A, int B, int K, double tol, double psd_tol,
                                  double* w, double* U, double* ws, int* fixed, void* stream) {
  if (B <= 0) return 0;
  if (K <= 64 || K > 160 || ws == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (K > 144) {  // 144 < K <= 160: the same 5-wave pair layout at KP = 160 (LDS ~118 KB)
    const size_t lds = bias_wide2_lds(K, 160, 5);
    (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<160, 5, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((mc_bias_wide2_kernel<160, 5, true>), dim3(B), dim3(5 * 64), lds, s, A, K, 1,
                       (const double*)nullptr, (const int*)nullptr, w,
                       (g_wide_eig_rounds << 4) | (g_wide_eig_abstol << 8), U);
    hipLaunchKernelGGL(eigh_wide_fix_kernel<160>, dim3(B), dim3(256), 0, s, A, K, tol, psd_tol, w, U, ws,
                       fixed);
  } else if (K <= 96) {
    const size_t lds = bias_wide2_lds(K, 96, 3);
    (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<96, 3, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((mc_bias_wide2_kernel<96, 3, true>), dim3(B), dim3(3 * 64), lds, s, A, K, 1,
                       (const double*)nullptr, (const int*)nullptr, w,
                       (g_wide_eig_rounds << 4) | (g_wide_eig_abstol << 8), U);
    hipLaunchKernelGGL(eigh_wide_fix_kernel<96>, dim3(B), dim3(256), 0, s, A, K, tol, psd_tol, w, U, ws,
                       fixed);
  } else {
    const size_t lds = bias_wide2_lds(K, 144, 5);
    (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<144, 5, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((mc_bias_wide2_kernel<144, 5, true>), dim3(B), dim3(5 * 64), lds, s, A, K, 1,
                       (const double*)nullptr, (const int*)nullptr, w,
                       (g_wide_eig_rounds << 4) | (g_wide_eig_abstol << 8), U);
    hipLaunchKernelGGL(eigh_wide_fix_kernel<144>, dim3(B), dim3(256), 0, s, A, K, tol, psd_tol, w, U, ws,
                       fixed);
  }
  return (int)hipGetLastError();
}

// As mfa_eigh_wide_fix_psd with every failing matrix re-solved (psd_tol < 0).
MFA_API int mfa_eigh_wide_fix(const double* A, int B, int K, double tol, double* w, double* U,
                              double* ws, int* fixed, void* stream) {
  return mfa_eigh_wide_fix_psd(A, B, K, tol, -1.0, w, U, ws, fixed, stream);
}

// The tridiagonal EIG kernel alone (no check), 96 < K <= 144: A/B and tests.
MFA_API int mfa_eigh_wide(const double* A, int B, int K, double* w, double* U, void* stream) {
  if (B <= 0) return 0;
  if (K <= 96 || K > 160) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (K > 144) {
    const size_t lds = bias_wide2_lds(K, 160, 5);
    (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<160, 5, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((mc_bias_wide2_kernel<160, 5, true>), dim3(B), dim3(5 * 64), lds, s, A, K,
                       1, (const double*)nullptr, (const int*)nullptr, w, 0, U);
    return (int)hipGetLastError();
  }
  const size_t lds = bias_wide2_lds(K, 144, 5);
  (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<144, 5, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((mc_bias_wide2_kernel<144, 5, true>), dim3(B), dim3(5 * 64), lds, s, A, K, 1,
                     (const double*)nullptr, (const int*)nullptr, w, 0, U);
  return (int)hipGetLastError();
}

int g_wide_abl = 0;  // timing-only phase ablations (bits: 1 Laguerre, 2 eigenvectors, 4 Householder)
// 2 = two lanes per row at every K (default since round 6: K = 80 bias 10.1 -> 8.2 ms,
// profiles/r06/wide_householder/layout_ab.log), 1 = one lane per row for K <= 96 and two for
// K > 96 (round 5: 26.9 vs 28.3 ms at K = 140, 60 x 100 problems), 0 = one lane per row (A/B)
int g_wide_variant = 2;
MFA_API void mfa_eigen_wide_set_ablation(int abl) { g_wide_abl = abl; }
MFA_API int mfa_eigen_wide_set_variant(int v) {
  if (v < 0 || v > 2 || (!MFA_AB && v == 0)) return (int)hipErrorInvalidValue;  // 0: A/B builds
  g_wide_variant = v;
  return 0;
}

MFA_API int mfa_eigen_bias_accumulate_wide(const double* D0, const int* dvalid, int D, int K,
                                           int M, const double* Cz, double* ws, double* S,
                                           void* stream) {
  if (D <= 0 || M <= 0) return 0;
  if (K < 3 || K > 160) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if ((g_wide_variant == 1 && K > 96) || g_wide_variant == 2 || K > 144) {
    // two lanes per row: 5 waves per problem for K > 96 (KP = 160 above 144), 3 for K <= 96
    if (K > 144) {
      const size_t lds = bias_wide2_lds(K, 160, 5);
      (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<160, 5>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((mc_bias_wide2_kernel<160, 5>), dim3(D * M), dim3(5 * 64), lds, s, D0, K,
                         M, Cz, dvalid, ws, g_wide_abl);
    } else if (K > 96) {
      const size_t lds = bias_wide2_lds(K, 144, 5);
      (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<144, 5>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((mc_bias_wide2_kernel<144, 5>), dim3(D * M), dim3(5 * 64), lds, s, D0, K,
                         M, Cz, dvalid, ws, g_wide_abl);
    } else {
      const size_t lds = bias_wide2_lds(K, 96, 3);
      (void)hipFuncSetAttribute((const void*)mc_bias_wide2_kernel<96, 3>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((mc_bias_wide2_kernel<96, 3>), dim3(D * M), dim3(3 * 64), lds, s, D0, K,
                         M, Cz, dvalid, ws, g_wide_abl);
    }
    hipLaunchKernelGGL(wide_bias_sum_kernel, dim3(D), dim3(64), 0, s, ws, K, M, S);
    return (int)hipGetLastError();
  }
#define MFA_WIDE(KP_, NW_)                                                                     \
  if (K <= KP_) {                                                                            \
    const size_t lds = bias_wide_lds(K, KP_, NW_);                                           \
    (void)hipFuncSetAttribute((const void*)mc_bias_wide_kernel<KP_, NW_>,                    \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);         \
    hipLaunchKernelGGL((mc_bias_wide_kernel<KP_, NW_>), dim3(D * M), dim3(NW_ * 64), lds, s, \
                       D0, K, M, Cz, dvalid, ws, g_wide_abl);                                \
  } else
#if MFA_AB
  MFA_WIDE(96, 2) MFA_WIDE(144, 3) {}  // 144: one lane per row (A/B layout 0)
#else
  MFA_WIDE(96, 2) {}
#endif
#undef MFA_WIDE
  hipLaunchKernelGGL(wide_bias_sum_kernel, dim3(D), dim3(64), 0, s, ws, K, M, S);
  return (int)hipGetLastError();
}

