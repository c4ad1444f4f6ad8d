// Batched cross-sectional WLS factor-return regression (Barra CNE5/USE4 style) for gfx950.
//
// Reference semantics: Barra-master/mfm/CrossSection.py:12-20 (style z-score: cap-weighted mean,
// ONE pooled ddof-0 std) and :57-108 (sqrt-cap WLS, industry-neutral constraint
// sum_j s_j f_j = 0 via the K x (K-1) matrix R, pinv solve, f = Omega r, e = r - X f,
// unweighted R^2).  Nothing mirrors the reference's dense N x N weight matrix.
//
// Three kernels, each shaped for its own regime, all dates of a shard per launch:
//   K1 xs_moments   HBM streaming.  One 4-wave workgroup per date; [D][Q][N] fp32 styles,
//                   caps, returns and int16 industry ids stream through a 3-deep LDS ring filled
//                   by global_load_lds_dwordx4 (counted vmcnt + raw s_barrier, so two tiles stay
//                   in flight across barriers).  RAW fp64 moments accumulate in registers; the
//                   one-hot industry block is a segmented sum done with ds_add_f64 into 4 lane-
//                   interleaved replicas of a [P][Q+3] table (4x fewer same-address conflicts).
//                   z-scoring is folded in algebraically later, so the data is read once.
//   K2 xs_solve     latency-bound tiny algebra.  One wave per date: after eliminating the pivot
//                   industry the industry block is diag(W) + rho a a^T (Sherman-Morrison), and
//                   only the (1+Q) x (1+Q) Schur complement is Cholesky-factorised, row-per-lane
//                   in registers with shuffles.  Exactly-empty industries get f = 0 (pinv
//                   semantics); near-singular dates are flagged for the pinv fallback.
//   K3 xs_resid     HBM streaming, low VGPR count: specific returns + R^2.  Dates are visited in
//                   reverse order so the tail of K1's stream is still Infinity-Cache resident.
#include "common.h"

#include <utility>

namespace {

using namespace mfa;

enum XsStatus : int {
  XS_NO_ROWS = 1,        // no valid stock on the date
  XS_PIVOT_EMPTY = 2,    // constraint pivot industry has zero capital
  XS_NEAR_SINGULAR = 4,  // Schur Cholesky lost > 12 digits: host refines with pinv
  XS_ZERO_PIVOT = 8,     // exactly-zero pivots / empty industries (pinv semantics -> f = 0)
  XS_BAD_SIGMA = 16,     // pooled style std is zero / NaN
};
constexpr int XS_BAD = XS_NO_ROWS | XS_BAD_SIGMA | XS_PIVOT_EMPTY;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ bool finite_f(float v) { return __builtin_isfinite(v); }

__device__ __forceinline__ void lds_add(double* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ds_add_f64 from inline asm: hipcc's waitcnt pass emits vmcnt(0) (draining every in-flight
// LDS-DMA tile) before any compiler-visible LDS write while a global_load_lds is pending.  The
// segment tables never alias the DMA ring, so the atomic is hidden from that analysis.  LDS ops
// complete in order, so the compiler's own lgkmcnt waits stay correct; barriers drain these.
template <int OFF>
__device__ __forceinline__ void lds_add_nowait(unsigned lds_addr, double v) {
  asm volatile("ds_add_f64 %0, %1 offset:%2" ::"v"(lds_addr), "v"(v), "i"(OFF) : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}

// 4-byte async global -> LDS copy (one fp32 per lane: a 64-stock row per wave instruction).
__device__ __forceinline__ void glds4(const void* src, void* wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)wave_base, 4, 0, 0);
}

// 16-byte async global -> LDS copy; LDS destination = wave-uniform `wave_base` + lane * 16.
__device__ __forceinline__ void glds16(const void* src, void* wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)wave_base, 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define MFA_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MFA_W(1) MFA_W(2) MFA_W(3) MFA_W(4) MFA_W(5) MFA_W(6) MFA_W(7) MFA_W(8) MFA_W(9)
    MFA_W(10) MFA_W(11) MFA_W(12) MFA_W(13) MFA_W(14) MFA_W(15) MFA_W(16) MFA_W(17)
    MFA_W(18) MFA_W(19) MFA_W(20) MFA_W(21) MFA_W(22) MFA_W(23) MFA_W(24) MFA_W(25)
    MFA_W(26) MFA_W(27) MFA_W(28) MFA_W(29) MFA_W(30) MFA_W(31) MFA_W(32) MFA_W(33)
    MFA_W(34) MFA_W(35) MFA_W(36) MFA_W(37) MFA_W(38) MFA_W(39) MFA_W(40) MFA_W(41)
    MFA_W(42) MFA_W(43) MFA_W(44) MFA_W(45) MFA_W(46) MFA_W(47) MFA_W(48) MFA_W(49)
    MFA_W(50) MFA_W(51) MFA_W(52) MFA_W(53) MFA_W(54) MFA_W(55) MFA_W(56) MFA_W(57)
    MFA_W(58) MFA_W(59) MFA_W(60) MFA_W(61) MFA_W(62) MFA_W(63)
#undef MFA_W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Workgroup barrier that does NOT drain in-flight LDS-DMA (__syncthreads() would emit vmcnt(0)).
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// value of a compile-time register array at a runtime index, without scratch
template <int Q>
__device__ __forceinline__ double pick(const double (&a)[Q], int i) {
  double r = 0.0;
#pragma unroll
  for (int k = 0; k < Q; ++k) r = (k == i) ? a[k] : r;
  return r;
}

constexpr int kTile = 256;            // stocks per staged tile (K3)
constexpr int kRowBytes = kTile * 4;  // one fp32 field row of a tile
constexpr int kRep = 4;               // segment-table replicas (lane & 3)
constexpr int kWT = 64;               // stocks per wave tile (K1: one stock per lane)
constexpr int kWNB = 4;               // K1 per-wave ring depth

template <int Q>
struct Layout {
  static constexpr int NS = Q + 3;             // per-industry channels: W, A_q, B, s
  static constexpr int NG = Q * (Q + 1) / 2;   // packed symmetric raw Gram
  static constexpr int NACC = NG + 2 * Q + 4;  // Swxx | Swxr | Scx | Sc Sx Sxx n
  static constexpr int ND = Q + 1;             // dense block: country + styles
  static constexpr int BUF = (Q + 2) * kRowBytes + kTile * 2;  // one ring slot
  static constexpr int WSLOT = (Q + 2) * kWT * 4 + kWT * 2;    // K1 per-wave ring slot
  __host__ __device__ static constexpr int msize(int Pseg) { return NACC + Pseg * NS; }
};

// Reduce a compile-time register array across the workgroup into out[0..CNT) (LDS, zeroed by
// the caller) through a per-wave [8][65] fp64 tile: keeps the register footprint flat.
template <int CNT>
__device__ __forceinline__ void wg_reduce(const double (&v)[CNT], double* wbuf, double* out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int a = lane & 7, slice = lane >> 3;
#pragma unroll
  for (int c0 = 0; c0 < CNT; c0 += 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (c0 + i < CNT) wbuf[i * 65 + lane] = v[c0 + i];
    wave_sync_lds();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += wbuf[a * 65 + slice * 8 + i];
    t += __shfl_xor(t, 8, kWave);
    t += __shfl_xor(t, 16, kWave);
    t += __shfl_xor(t, 32, kWave);
    if (slice == 0 && c0 + a < CNT) lds_add(out + c0 + a, t);
    wave_sync_lds();
  }
}

// ------------------------------------------------------------------------------------------
// K1: raw moments.  mom[d] = [ Swxx(NG) | Swxr(Q) | Scx(Q) | Sc Sx Sxx n | seg[Pseg][NS] ]
// ------------------------------------------------------------------------------------------
template <int Q, int VAR>
__global__ __launch_bounds__(256) void xs_moments_kernel(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, double* __restrict__ mom) {
  using L = Layout<Q>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, BUF = L::BUF, NBUF = 3;
  // Per-wave DMA rings (own __shared__ object, separate from the atomics' dynamic LDS): each
  // wave streams its own 64-stock tiles (k = wid, wid + nw, ...) with no workgroup barrier until
  // the final reduction, so the 8 waves of a CU drift and overlap HBM, VALU and LDS phases.
  constexpr int WSLOT = L::WSLOT;
  constexpr int RINGW = kWNB * WSLOT > 8 * 65 * 8 ? kWNB * WSLOT : 8 * 65 * 8;
  __shared__ __attribute__((aligned(16))) char ring[4 * RINGW];
  extern __shared__ double dyn[];  // [kRep][Pseg*NS + 1] replicas | [NACC] totals
  const int d = blockIdx.x;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nthr >> 6;
  const int rstride = Pseg * NS + 1;  // odd stride spreads the replicas over banks
  const unsigned seg_a = lds_addr(dyn + (lane & (kRep - 1)) * rstride);
  double* acc = dyn + kRep * rstride;
  for (int i = tid; i < kRep * rstride + NACC; i += nthr) dyn[i] = 0.0;
  __syncthreads();

  const float* Xd = X + (size_t)d * Q * N;
  const float* cd = cap + (size_t)d * N;
  const float* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;

  double v[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) v[i] = 0.0;

  char* wring = ring + wid * RINGW;
  const int nrows = id ? Q + 3 : Q + 2;        // glds instructions per tile
  const int ntile_all = (N + kWT - 1) / kWT;
  const int ntile = ntile_all > wid ? (ntile_all - wid + nw - 1) / nw : 0;  // this wave's tiles
  auto issue = [&](int i) {
    char* slot = wring + (i % kWNB) * WSLOT;
    const int s0 = (wid + i * nw) * kWT;
    const bool in = s0 + lane < N;
    if (in) glds4(cd + s0 + lane, slot);
    if (in) glds4(rd + s0 + lane, slot + kWT * 4);
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (in) glds4(Xd + (size_t)q * N + s0 + lane, slot + (2 + q) * kWT * 4);
    if (id && lane < kWT / 2 && s0 + 2 * lane < N) glds4(id + s0 + 2 * lane, slot + (Q + 2) * kWT * 4);
  };
  for (int i = 0; i < kWNB - 1 && i < ntile; ++i) issue(i);
  for (int i = 0; i < ntile; ++i) {
    const bool tail = (i + kWNB - 1 >= ntile);
    wait_vmcnt(tail ? 0 : (kWNB - 2) * nrows);
    __builtin_amdgcn_wave_barrier();
    if (i + kWNB - 1 < ntile) issue(i + kWNB - 1);
    const char* slot = wring + (i % kWNB) * WSLOT;
    const float* bf = (const float*)slot;
    const int s = (wid + i * nw) * kWT + lane;
    const float cf = bf[lane], rf = bf[kWT + lane];
    const int j = id ? (int)((const int16_t*)(slot + (Q + 2) * kWT * 4))[lane] : 0;
    float xf[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) xf[q] = bf[(2 + q) * kWT + lane];
    bool ok = (s < N) && (j >= 0) && (j < Pseg) && finite_f(cf) && (cf >= 0.f) && finite_f(rf);
#pragma unroll
    for (int q = 0; q < Q; ++q) ok = ok && finite_f(xf[q]);
    if (ok) {
      const double c = cf, r = rf, w = sqrt(c);
      double x[Q], wx[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) { x[q] = xf[q]; wx[q] = w * x[q]; }
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int t = 0; t <= q; ++t) v[q * (q + 1) / 2 + t] = fma(wx[q], x[t], v[q * (q + 1) / 2 + t]);
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
      if (VAR & 1) {  // timing-only ablation: skip the segment atomics
        asm volatile("" ::"v"(w), "v"(r));
      } else {
        const unsigned a = seg_a + (unsigned)(j * NS * 8);
        lds_add_nowait<0>(a, w);
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (lds_add_nowait<8 * (1 + I)>(a, wx[I]), ...);
        }(std::make_integer_sequence<int, Q>{});
        lds_add_nowait<8 * (Q + 1)>(a, w * r);
        lds_add_nowait<8 * (Q + 2)>(a, c);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  wg_reduce<NACC>(v, (double*)wring, acc);
  __syncthreads();
  double* md = mom + (size_t)d * L::msize(Pseg);
  for (int i = tid; i < NACC; i += nthr) md[i] = acc[i];
  for (int i = tid; i < Pseg * NS; i += nthr) {
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < kRep; ++r) t += dyn[r * rstride + i];
    md[NACC + i] = t;
  }
}

// ------------------------------------------------------------------------------------------
// K2: structured constrained solve, one wave per date.
// coef[d] = [ beta_q (Q) | cst | f_ind (P) ]  for the residual pass (e = r - cst - f_j - b.x)
// ------------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(64) void xs_solve_kernel(const double* __restrict__ mom, int P,
                                                      int Pseg, int pivot_mode, double tol,
                                                      double* __restrict__ fout,
                                                      double* __restrict__ coef,
                                                      double* __restrict__ stats,
                                                      int* __restrict__ status) {
  using L = Layout<Q>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, ND = L::ND;
  extern __shared__ double sm[];
  const int d = blockIdx.x;
  const int lane = threadIdx.x;
  const int K = 1 + P + Q;
  const int MS = L::msize(Pseg);
  double* acc = sm;                   // [NACC]
  double* seg = sm + NACC;            // [Pseg][NS]   (A_q standardised in place)
  double* MID = seg + Pseg * NS;      // [Pseg][ND+1] M_ID | h_I
  double* S = MID + Pseg * (ND + 1);  // [ND][ND+1]   Schur complement | rhs
  double* fsh = S + ND * (ND + 1);    // [K]
  double* Yb = fsh + K;               // [Pseg][ND+1] M_II^{-1} [M_ID | h_I]
  const double* md = mom + (size_t)d * MS;
  for (int i0 = 0; i0 < MS; i0 += 8 * 64) {  // 8 independent loads in flight per lane
    double tmp[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 64 + lane;
      tmp[u] = i < MS ? md[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 64 + lane;
      if (i < MS) sm[i] = tmp[u];
    }
  }
  wave_sync_lds();

  const double Sc = acc[NG + 2 * Q + 0];
  const double nval = acc[NG + 2 * Q + 3];
  const double nq = nval * Q;
  const double mx = acc[NG + 2 * Q + 1] / nq;
  const double sigma = sqrt(fmax(acc[NG + 2 * Q + 2] / nq - mx * mx, 0.0));
  const double isig = 1.0 / sigma;
  int st = 0;
  if (!(nval > 0.0)) st |= XS_NO_ROWS;
  if (!(sigma > 0.0) || !__builtin_isfinite(sigma)) st |= XS_BAD_SIGMA;

  // industry totals (lane-strided partials + butterfly)
  double Sw = 0.0, Swr = 0.0, Swx[Q], mu[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) Swx[q] = 0.0;
  for (int j = lane; j < Pseg; j += 64) {
    const double* p = seg + j * NS;
    Sw += p[0];
    Swr += p[Q + 1];
#pragma unroll
    for (int q = 0; q < Q; ++q) Swx[q] += p[1 + q];
  }
  Sw = wave_sum(Sw);
  Swr = wave_sum(Swr);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    Swx[q] = wave_sum(Swx[q]);
    mu[q] = acc[NG + Q + q] / Sc;
  }
  // standardise the segmented style sums in place: A'_jq = (A_jq - mu_q W_j) / sigma
  for (int j = lane; j < Pseg; j += 64) {
    double* p = seg + j * NS;
#pragma unroll
    for (int q = 0; q < Q; ++q) p[1 + q] = (p[1 + q] - mu[q] * p[0]) * isig;
  }
  wave_sync_lds();

  // pivot industry (reference: always the last one, CrossSection.py:69)
  int jp = -1;
  if (P > 0) {
    if (pivot_mode == 1) {
      jp = P - 1;
    } else {
      for (int jb = 0; jb < P; jb += 64) {
        const int j = jb + lane;
        const unsigned long long m = __ballot(j < P && seg[j * NS + Q + 2] > 0.0);
        if (m) jp = jb + 63 - __builtin_clzll(m);
      }
      if (jp < 0) jp = P - 1;
    }
    if (!(seg[jp * NS + Q + 2] > 0.0)) st |= XS_PIVOT_EMPTY;
  }
  const double sp = P > 0 ? seg[jp * NS + Q + 2] : 1.0;
  const double rho = P > 0 ? seg[jp * NS] : 0.0;

  // M_ID rows (lane = industry): M_ID[j][u] = G[j][u] + a_j G[p][u], h_I = B_j + a_j B_p,
  // Y = M_II^{-1} [M_ID | h_I] with M_II = diag(W) + rho a a^T (Sherman-Morrison).
  double den = 0.0, at[ND + 1];
#pragma unroll
  for (int u = 0; u <= ND; ++u) at[u] = 0.0;
  for (int j = lane; j < P; j += 64) {
    const double* p = seg + j * NS;
    const double* pp = seg + jp * NS;
    const double W = p[0];
    const bool act = (j != jp) && (W > 0.0);
    const double aj = act ? -p[Q + 2] / sp : 0.0;
    const double iW = act ? 1.0 / W : 0.0;
    double* row = MID + j * (ND + 1);
    double m[ND + 1];
    m[0] = act ? W + aj * pp[0] : 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) m[1 + q] = act ? p[1 + q] + aj * pp[1 + q] : 0.0;
    m[ND] = act ? p[Q + 1] + aj * pp[Q + 1] : 0.0;
#pragma unroll
    for (int u = 0; u <= ND; ++u) {
      row[u] = m[u];
      at[u] = fma(aj, m[u] * iW, at[u]);
    }
    den = fma(aj * rho, aj * iW, den);
  }
  den = wave_sum(den);
#pragma unroll
  for (int u = 0; u <= ND; ++u) at[u] = wave_sum(at[u]);
  const double kappa = rho / (1.0 + den);
  wave_sync_lds();
  for (int j = lane; j < P; j += 64) {
    const double* p = seg + j * NS;
    const double W = p[0];
    const bool act = (j != jp) && (W > 0.0);
    const double aj = act ? -p[Q + 2] / sp : 0.0;
    const double iW = act ? 1.0 / W : 0.0;
    const double* row = MID + j * (ND + 1);
    double* y = Yb + j * (ND + 1);
#pragma unroll
    for (int u = 0; u <= ND; ++u) y[u] = act ? (row[u] - kappa * at[u] * aj) * iW : 0.0;
  }
  wave_sync_lds();

  // dense block (country + z-scored styles) and Schur complement:
  //   S[u][w] = M_DD[u][w] - sum_j M_ID[j][u] Y[j][w]   (w = ND is the rhs column)
  for (int e = lane; e < ND * (ND + 1); e += 64) {
    const int u = e / (ND + 1), w = e % (ND + 1);
    double m;
    if (w == ND) {
      m = u == 0 ? Swr : (acc[NG + u - 1] - pick<Q>(mu, u - 1) * Swr) * isig;
    } else if (u == 0 && w == 0) {
      m = Sw;
    } else if (u == 0 || w == 0) {
      const int q = (u == 0 ? w : u) - 1;
      m = (pick<Q>(Swx, q) - pick<Q>(mu, q) * Sw) * isig;
    } else {
      const int q = u - 1, s = w - 1;
      const int hi = q > s ? q : s, lo = q > s ? s : q;
      const double muq = pick<Q>(mu, q), mus = pick<Q>(mu, s);
      m = (acc[hi * (hi + 1) / 2 + lo] - muq * pick<Q>(Swx, s) - mus * pick<Q>(Swx, q) +
           muq * mus * Sw) * isig * isig;
    }
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
    int j = 0;
    for (; j + 4 <= P; j += 4) {
      t0 = fma(MID[(j + 0) * (ND + 1) + u], Yb[(j + 0) * (ND + 1) + w], t0);
      t1 = fma(MID[(j + 1) * (ND + 1) + u], Yb[(j + 1) * (ND + 1) + w], t1);
      t2 = fma(MID[(j + 2) * (ND + 1) + u], Yb[(j + 2) * (ND + 1) + w], t2);
      t3 = fma(MID[(j + 3) * (ND + 1) + u], Yb[(j + 3) * (ND + 1) + w], t3);
    }
    for (; j < P; ++j) t0 = fma(MID[j * (ND + 1) + u], Yb[j * (ND + 1) + w], t0);
    S[e] = m - ((t0 + t1) + (t2 + t3));
  }
  wave_sync_lds();

  // Cholesky of the ND x ND Schur complement: lane i holds row i in registers
  double row[ND], Lkk[ND];
#pragma unroll
  for (int w = 0; w < ND; ++w) row[w] = lane < ND ? S[lane * (ND + 1) + w] : 0.0;
  double yv = lane < ND ? S[lane * (ND + 1) + ND] : 0.0;
  double dmax = 0.0;
#pragma unroll
  for (int k = 0; k < ND; ++k) dmax = fmax(dmax, fabs(S[k * (ND + 1) + k]));
  const double ztol = tol * dmax;
  unsigned skip = 0u;
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const double dk = __shfl(row[k], k, 64);  // current pivot
    const double dorig = S[k * (ND + 1) + k];
    if (!(dk > ztol)) {  // pinv semantics: drop the direction (exactly singular block)
      skip |= 1u << k;
      st |= (dorig > ztol) ? XS_NEAR_SINGULAR : XS_ZERO_PIVOT;
      Lkk[k] = 0.0;
      if (lane >= k) row[k] = 0.0;
    } else {
      if (dk < 1e-12 * dorig) st |= XS_NEAR_SINGULAR;
      const double l = sqrt(dk);
      Lkk[k] = l;
      if (lane > k) row[k] /= l;
      if (lane == k) row[k] = l;
#pragma unroll
      for (int w = k + 1; w < ND; ++w) {  // row_i[w] -= L_ik L_wk   (k < w <= i)
        const double lwk = __shfl(row[k], w, 64);
        if (lane >= w) row[w] = fma(-row[k], lwk, row[w]);
      }
    }
  }
  // forward L y = b, backward L^T g = y  (lane k holds entry k)
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const double yk = ((skip >> k) & 1u) ? 0.0 : __shfl(yv, k, 64) / Lkk[k];
    if (lane == k) yv = yk;
    if (lane > k) yv = fma(-row[k], yk, yv);
  }
  double gv = yv;
#pragma unroll
  for (int k = ND - 1; k >= 0; --k) {
    const double gk = ((skip >> k) & 1u) ? 0.0 : __shfl(gv, k, 64) / Lkk[k];
    if (lane == k) gv = gk;
#pragma unroll
    for (int i = 0; i < k; ++i) {  // g_i -= L_ki g_k ; L_ki is lane k's row[i]
      const double lki = __shfl(row[i], k, 64);
      if (lane == i) gv = fma(-lki, gk, gv);
    }
  }
  double gD[ND];
#pragma unroll
  for (int u = 0; u < ND; ++u) gD[u] = __shfl(gv, u, 64);
  // industries: g_j = Y[j][ND] - sum_u Y[j][u] g_u ; the pivot from the constraint
  double piv = 0.0;
  for (int j = lane; j < P; j += 64) {
    const double* y = Yb + j * (ND + 1);
    double g = y[ND];
#pragma unroll
    for (int u = 0; u < ND; ++u) g = fma(-y[u], gD[u], g);
    if (j != jp) piv = fma(-seg[j * NS + Q + 2] / sp, g, piv);
    fsh[1 + j] = g;
  }
  piv = wave_sum(piv);
  wave_sync_lds();
  if (lane == 0) {
    fsh[0] = gD[0];
    if (P > 0) fsh[1 + jp] = piv;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (lane == q) fsh[1 + P + q] = gD[1 + q];
  wave_sync_lds();

  const bool bad = (st & XS_BAD) != 0;
  double* fo = fout + (size_t)d * K;
  double* co = coef + (size_t)d * (Q + 1 + P);
  for (int i = lane; i < K; i += 64) fo[i] = bad ? qnan() : fsh[i];
  // residual coefficients on RAW styles: e = r - cst - f_j - sum_q beta_q x_q
  if (lane < Q) co[lane] = bad ? qnan() : fsh[1 + P + lane] * isig;
  if (lane == 0) {
    double cst = fsh[0];
#pragma unroll
    for (int q = 0; q < Q; ++q) cst -= gD[1 + q] * isig * mu[q];
    co[Q] = bad ? qnan() : cst;
    status[d] = st;
  }
  for (int j = lane; j < P; j += 64) co[Q + 1 + j] = bad ? qnan() : fsh[1 + j];
  if (stats) {
    double* sd = stats + (size_t)d * (Q + 2);
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (lane == q) sd[q] = mu[q];
    if (lane == Q) sd[Q] = sigma;
    if (lane == Q + 1) sd[Q + 1] = nval;
  }
}

// ------------------------------------------------------------------------------------------
// K3: specific returns and R^2 (dates visited in reverse: MALL-resident tail of K1 first)
// ------------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(256) void xs_resid_kernel(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int D, int N, int P, const double* __restrict__ coef,
    const int* __restrict__ status, float* __restrict__ eout, double* __restrict__ r2out) {
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red[4][5];
  const int d = D - 1 - blockIdx.x;
  const int tid = threadIdx.x;
  const int Pseg = P > 0 ? P : 1;
  const double* co = coef + (size_t)d * (Q + 1 + P);
  for (int i = tid; i < Q + 1 + P; i += blockDim.x) cf_s[i] = co[i];
  __syncthreads();
  double beta[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) beta[q] = cf_s[q];
  const double cst = cf_s[Q];
  const double* fI = cf_s + Q + 1;
  const float* Xd = X + (size_t)d * Q * N;
  const float* cd = cap + (size_t)d * N;
  const float* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;
  float* ed = eout ? eout + (size_t)d * N : nullptr;
  double se = 0.0, see = 0.0, sr = 0.0, srr = 0.0, nn = 0.0;
  for (int n = tid; n < N; n += blockDim.x) {
    const float c = cd[n], r = rd[n];
    const int j = id ? (int)id[n] : 0;
    float xf[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) xf[q] = Xd[(size_t)q * N + n];
    bool ok = (j >= 0) && (j < Pseg) && finite_f(c) && (c >= 0.f) && finite_f(r);
    double e = (double)r - cst;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      ok = ok && finite_f(xf[q]);
      e = fma(-beta[q], (double)xf[q], e);
    }
    float eo = qnanf();
    if (ok) {
      if (P > 0) e -= fI[j];
      se += e;
      see = fma(e, e, see);
      sr += r;
      srr = fma((double)r, (double)r, srr);
      nn += 1.0;
      eo = (float)e;
    }
    if (ed) ed[n] = eo;
  }
  se = wave_sum(se); see = wave_sum(see); sr = wave_sum(sr); srr = wave_sum(srr); nn = wave_sum(nn);
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    red[w][0] = se; red[w][1] = see; red[w][2] = sr; red[w][3] = srr; red[w][4] = nn;
  }
  __syncthreads();
  if (tid == 0) {
    double a = 0, b = 0, c = 0, e2 = 0, n = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      a += red[i][0]; b += red[i][1]; c += red[i][2]; e2 += red[i][3]; n += red[i][4];
    }
    const double ve = b / n - (a / n) * (a / n);
    const double vr = e2 / n - (c / n) * (c / n);
    r2out[d] = (status[d] & XS_BAD) ? qnan() : 1.0 - ve / vr;
  }
}

template <int Q, int VAR = 0>
hipError_t launch_q(const float* X, const float* cap, const float* ret, const int16_t* ind,
                    int D, int N, int P, int pivot_mode, double tol, double* f, float* e,
                    double* r2, double* stats, int* status, double* ws, hipStream_t s) {
  using L = Layout<Q>;
  const int Pseg = P > 0 ? P : 1;
  const int K = 1 + P + Q;
  double* mom = ws;
  double* coef = ws + (size_t)D * L::msize(Pseg);
  const size_t lds1 = ((size_t)kRep * (Pseg * L::NS + 1) + L::NACC) * sizeof(double);
  const size_t lds2 = ((size_t)L::msize(Pseg) + (size_t)Pseg * (L::ND + 1) * 2 +
                       L::ND * (L::ND + 1) + K) * sizeof(double);
  if (lds1 + 4 * (size_t)kWNB * L::WSLOT + 16640 > 160 * 1024 || lds2 > 64 * 1024)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((xs_moments_kernel<Q, VAR>), dim3(D), dim3(256), lds1, s, X, cap, ret,
                     P > 0 ? ind : nullptr, N, Pseg, mom);
  hipLaunchKernelGGL(xs_solve_kernel<Q>, dim3(D), dim3(64), lds2, s, mom, P, Pseg, pivot_mode,
                     tol, f, coef, stats, status);
  if (!(VAR & 4))
    hipLaunchKernelGGL(xs_resid_kernel<Q>, dim3(D), dim3(256), 0, s, X, cap, ret,
                       P > 0 ? ind : nullptr, D, N, P, coef, status, e, r2);
  return hipGetLastError();
}

}  // namespace

// Workspace bytes needed by mfa_xs_wls: D * (msize + Q + 1 + P) doubles.
MFA_API size_t mfa_xs_wls_workspace(int D, int P, int Q) {
  const int Pseg = P > 0 ? P : 1;
  const size_t ms = (size_t)Q * (Q + 1) / 2 + 2 * Q + 4 + (size_t)Pseg * (Q + 3);
  return (size_t)D * (ms + Q + 1 + P) * sizeof(double);
}

// X: [D][Q][N] fp32 styles, cap/ret: [D][N] fp32, ind: [D][N] int16 industry id (<0 = absent;
// may be null when P == 0).  N must be a multiple of 8 (16-byte aligned rows; pad with absent
// stocks).  Outputs: f [D][1+P+Q] fp64 (country, industries, styles), e [D][N] fp32 specific
// returns (nullable), r2 [D] fp64, stats [D][Q+2] fp64 = (mu_q, sigma, n_valid) (nullable),
// status [D] int32 XsStatus bits.  pivot_mode: 0 = last non-empty industry, 1 = reference.
MFA_API int mfa_xs_wls(const float* X, const float* cap, const float* ret, const int16_t* ind,
                       int D, int N, int P, int Q, int pivot_mode, double tol, double* f,
                       float* e, double* r2, double* stats, int* status, void* ws,
                       void* stream) {
  if (D <= 0) return 0;
  if (Q < 1 || Q > 16 || P < 0 || P > 128 || N <= 0 || (N % 8) != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  double* w = (double*)ws;
  switch (Q) {
#define MFA_Q(qq)                                                                              \
  case qq:                                                                                     \
    return (int)launch_q<qq>(X, cap, ret, ind, D, N, P, pivot_mode, tol, f, e, r2, stats,      \
                             status, w, s);
    MFA_Q(1) MFA_Q(2) MFA_Q(3) MFA_Q(4) MFA_Q(5) MFA_Q(6) MFA_Q(7) MFA_Q(8)
    MFA_Q(9) MFA_Q(10) MFA_Q(11) MFA_Q(12) MFA_Q(13) MFA_Q(14) MFA_Q(15) MFA_Q(16)
#undef MFA_Q
  }
  return (int)hipErrorInvalidValue;
}

// Timing-only ablation entry (Q = 10): bit 1 = no segment atomics, bit 4 = no residual pass.
MFA_API int mfa_xs_wls_variant(const float* X, const float* cap, const float* ret,
                               const int16_t* ind, int D, int N, int P, int variant, double* f,
                               float* e, double* r2, double* stats, int* status, void* ws,
                               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  double* w = (double*)ws;
  switch (variant) {
#define MFA_V(vv)                                                                              \
  case vv:                                                                                     \
    return (int)launch_q<10, vv>(X, cap, ret, ind, D, N, P, 0, 1e-14, f, e, r2, stats,        \
                                 status, w, s);
    MFA_V(0) MFA_V(1) MFA_V(4) MFA_V(5)
#undef MFA_V
  }
  return (int)hipErrorInvalidValue;
}
