// Batched cross-sectional WLS factor-return regression (Barra CNE5/USE4 style) for gfx950.
//
// Reference semantics: Barra-master/mfm/CrossSection.py:12-20 (style z-score: cap-weighted mean,
// ONE pooled ddof-0 std) and :57-108 (sqrt-cap WLS, industry-neutral constraint
// sum_j s_j f_j = 0 via the K x (K-1) matrix R, pinv solve, f = Omega r, e = r - X f,
// unweighted R^2).  Nothing mirrors the reference's dense N x N weight matrix.
//
// Three kernels, each shaped for its own regime, all dates of a shard per launch:
//   K1 xs_moments   HBM streaming.  One 4-wave workgroup per date; every wave streams its own
//                   64-stock tiles of the [D][Q][N] fp32 styles, caps, returns and int16
//                   industry ids through a private 4-slot LDS ring filled by
//                   global_load_lds_dword (counted vmcnt, no workgroup barrier until the date's
//                   final reduction).  RAW fp64 moments accumulate in registers; the one-hot
//                   industry block is a segmented sum done with ds_add_f64 into an 8-way
//                   replicated [P][Q+3] table laid out so one issue group is <= 2-way conflicted.
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

#ifndef MFA_XS_RING
#define MFA_XS_RING 4
#endif
#ifndef MFA_XS_REP
#define MFA_XS_REP 8
#endif
constexpr int kTile = 256;            // stocks per staged tile (K3)
constexpr int kRowBytes = kTile * 4;  // one fp32 field row of a tile
// Segment-table replicas: entry (j, ch) owns R consecutive doubles and lane l adds into slot
// l & (R-1).  With R = 8 the 16 lanes of a ds_add_f64 issue group land on bank pairs
// (l & 7) + 8 * ((j*NS + ch) & 1): at most 2-way conflicts whatever the industry mix (4
// lane-strided replicas measured 8.3 conflict cycles per instruction).
constexpr int kRepMax = MFA_XS_REP;
constexpr int kSegLdsBudget = 48 * 1024;  // R = 8 only while the table leaves 2 WGs / CU
constexpr int kWT = 64;               // stocks per wave tile (K1: one stock per lane)
constexpr int kWNB = MFA_XS_RING;     // K1 per-wave ring depth

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
// DET: `out` is this wave's own partial row (plain stores, summed in wave order by the caller)
// instead of the shared total (LDS atomics: order-dependent rounding).
template <int CNT, bool DET = false>
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
    if (slice == 0 && c0 + a < CNT) {
      if constexpr (DET) out[c0 + a] = t;
      else lds_add(out + c0 + a, t);
    }
    wave_sync_lds();
  }
}

// ------------------------------------------------------------------------------------------
// K1: raw moments.  mom[d] = [ Swxx(NG) | Swxr(Q) | Scx(Q) | Sc Sx Sxx n | seg[Pseg][NS] ]
// ------------------------------------------------------------------------------------------
template <int Q>
struct Ring {
  // Per-wave DMA rings (own __shared__ object, separate from the atomics' dynamic LDS): each
  // wave streams its own 64-stock tiles (k = wid, wid + nw, ...) with no workgroup barrier until
  // the final reduction, so the 8 waves of a CU drift and overlap HBM, VALU and LDS phases.
  static constexpr int WSLOT = Layout<Q>::WSLOT;
  // >= the reduction tile [8][65] fp64 + one partial row (deterministic wg_reduce)
  static constexpr int RED = (8 * 65 + Layout<Q>::NACC) * 8;
  static constexpr int RINGW = kWNB * WSLOT > RED ? kWNB * WSLOT : RED;
  static constexpr int BYTES = 4 * RINGW;
};

// Moments of date d.  `ring` = Ring<Q>::BYTES of LDS, `dyn` = [Pseg*NS][R] replicated segment
// sums | [NACC] totals (LDS), `md` = msize(Pseg) doubles out (global memory or LDS that does
// not alias `dyn`; may alias `ring`).  Ends with a workgroup barrier.
//
// VAR & 32 = bitwise-deterministic mode (4-wave workgroups): every segment replica is owned by
// ONE wave (R/4 per wave), so its atomics land in that wave's program order, and the per-lane
// totals are reduced through per-wave partial rows summed in wave order.  The default mode
// shares replicas across waves (fewer bank conflicts) and is reproducible to rounding only.
template <int Q, int VAR, int R>
__device__ __forceinline__ void moments_body(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, int d, char* ring, double* dyn,
    double* md) {
  using L = Layout<Q>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC;
  constexpr int WSLOT = Ring<Q>::WSLOT, RINGW = Ring<Q>::RINGW;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nthr >> 6;
  constexpr bool DET = (VAR & 32) != 0;
  static_assert(!DET || (R % 4 == 0 && NACC <= 256), "deterministic mode: 4 waves, R/4 replicas each");
  const int rep = DET ? wid * (R / 4) + (lane & (R / 4 - 1)) : (lane & (R - 1));
  const unsigned seg_a = lds_addr(dyn + rep);
  double* acc = dyn + R * Pseg * NS;
  for (int i = tid; i < R * Pseg * NS + NACC; i += nthr) dyn[i] = 0.0;
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
      if constexpr ((VAR & 2) != 0) {  // timing-only ablation: skip the moment FMAs
#pragma unroll
        for (int q = 0; q < Q; ++q) asm volatile("" ::"v"(wx[q]));
      } else {
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int t = 0; t <= q; ++t) v[q * (q + 1) / 2 + t] = fma(wx[q], x[t], v[q * (q + 1) / 2 + t]);
      }
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
        const unsigned a = seg_a + (unsigned)(j * NS * R * 8);
        lds_add_nowait<0>(a, w);
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (lds_add_nowait<8 * R * (1 + I)>(a, wx[I]), ...);
        }(std::make_integer_sequence<int, Q>{});
        lds_add_nowait<8 * R * (Q + 1)>(a, w * r);
        lds_add_nowait<8 * R * (Q + 2)>(a, c);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (DET) {
    static_assert(Ring<Q>::RINGW >= 8 * 65 * 8 + NACC * 8, "partial row must fit the wave ring");
    wg_reduce<NACC, true>(v, (double*)wring, (double*)(wring + 8 * 65 * 8));
    __syncthreads();
    double t = 0.0;
    if (tid < NACC)
      for (int w = 0; w < nw; ++w) t += ((const double*)(ring + w * RINGW + 8 * 65 * 8))[tid];
    __syncthreads();  // md may alias the ring
    if (tid < NACC) md[tid] = t;
  } else {
    wg_reduce<NACC>(v, (double*)wring, acc);
    __syncthreads();
    for (int i = tid; i < NACC; i += nthr) md[i] = acc[i];
  }
  for (int i = tid; i < Pseg * NS; i += nthr) {
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) t += dyn[i * R + r];
    md[NACC + i] = t;
  }
  __syncthreads();
}

template <int Q, int VAR, int R>
__global__ __launch_bounds__(256) void xs_moments_kernel(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, double* __restrict__ mom) {
  __shared__ __attribute__((aligned(16))) char ring[Ring<Q>::BYTES];
  extern __shared__ double dyn[];
  const int d = blockIdx.x;
  moments_body<Q, VAR, R>(X, cap, ret, ind, N, Pseg, d, ring, dyn,
                          mom + (size_t)d * Layout<Q>::msize(Pseg));
}

// ------------------------------------------------------------------------------------------
// K2: structured constrained solve, one wave per date.
// coef[d] = [ beta_q (Q) | cst | f_ind (P) ]  for the residual pass (e = r - cst - f_j - b.x)
//
// Algebra (CrossSection.py:57-106 with the constraint substituted): with g_j the standardised
// industry row [W_j, (A_jq - mu_q W_j)/sigma, B_j], pivot p, a_j = -s_j/s_p and
// m_j = g_j + a_j g_p for the active industries, the industry block is diag(W) + rho a a^T and
//   S   = M_DD - G + kappa at at^T,    G = sum_j m_j m_j^T / W_j,   at = sum_j a_j m_j / W_j,
//   kappa = rho / (1 + rho c0),        c0 = sum_j a_j^2 / W_j,
//   f_j = (m_j . h - kappa a_j z) / W_j,  f_p = z (1 - kappa c0),  h = [-g_D, 1],  z = at . h.
// G, at, c0 and the industry totals are ONE weighted Gram over industries with augmented
// channels [m | a | 1], computed by v_mfma_f64_16x16x4f64 straight from the moments in LDS
// (A[i][k] from lane i + 16k, B[k][j] from lane j + 16k, D[(l>>4) + 4r][l&15] in register r
// -- layout probed in tools/probes/mfma64_probe.hip).  Only the (1+Q)^2 Cholesky is serial; it
// runs redundantly in every lane's registers.  All dates are resident at once, so the kernel
// time is one date's critical path.
// ------------------------------------------------------------------------------------------
typedef double v4d __attribute__((ext_vector_type(4)));

template <int Q>
constexpr size_t solve_lds_doubles(int Pseg) {
  using L = Layout<Q>;
  return (size_t)L::msize(Pseg) + (size_t)(Q + 4) * (Q + 4) + (size_t)L::ND * (L::ND + 1) +
         (Q + 2) + Q + 2 * (((size_t)Pseg + 3) & ~(size_t)3);
}

// Constrained solve of date d by ONE wave (threadIdx.x < 64).  `sm` (LDS, solve_lds_doubles)
// holds the date's moments in [0, msize(Pseg)) on entry.  Writes f (global), the residual
// coefficients `co` [Q+1+P] (global or LDS), stats/status (global) and, if non-null, the
// status word to `st_lds`.
template <int Q>
__device__ __forceinline__ void solve_body(double* sm, int d, int P, int Pseg, int pivot_mode,
                                           double tol, double* __restrict__ fout,
                                           double* co, double* __restrict__ stats,
                                           int* __restrict__ status, int* st_lds,
                                           long long* __restrict__ stamps) {
  using L = Layout<Q>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, ND = L::ND;
  constexpr int NC = ND + 1;              // standardised industry row incl. the rhs
  constexpr int CH = NC + 2;              // Gram channels: m (NC) | a | 1
  constexpr int TT = (CH + 15) / 16;      // MFMA tiles per dimension
  static_assert(TT <= 2, "Q <= 28");
  // optional phase timestamps (s_memtime, core clocks) for latency attribution
  auto stamp = [&](int k) {
    if (stamps && threadIdx.x == 0) stamps[(size_t)d * 8 + k] = __builtin_amdgcn_s_memtime();
  };
  const int lane = threadIdx.x;
  const int K = 1 + P + Q;
  const int MS = L::msize(Pseg);
  const int P4 = (Pseg + 3) & ~3;         // industries padded to the MFMA k-step
  double* acc = sm;                       // [NACC]
  double* seg = sm + NACC;                // [Pseg][NS]  W, A_q, B, s
  double* Gs = sm + MS;                   // [CH][CH]    Gram over industries
  double* S = Gs + CH * CH;               // [ND][NC]    Schur complement | rhs
  double* gpv = S + ND * NC;              // [NC]        standardised pivot row
  double* muv = gpv + NC;                 // [Q]
  double* ajv = muv + Q;                  // [P4]        a_j
  double* iwv = ajv + P4;                 // [P4]        1 / W_j
  stamp(1);

  const double Sc = acc[NG + 2 * Q + 0];
  const double nval = acc[NG + 2 * Q + 3];
  const double nq = nval * Q;
  const double mx = acc[NG + 2 * Q + 1] / nq;
  const double sigma = sqrt(fmax(acc[NG + 2 * Q + 2] / nq - mx * mx, 0.0));
  const double isig = 1.0 / sigma;
  const double iSc = 1.0 / Sc;
  int st = 0;
  if (!(nval > 0.0)) st |= XS_NO_ROWS;
  if (!(sigma > 0.0) || !__builtin_isfinite(sigma)) st |= XS_BAD_SIGMA;

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
  const int rp = P > 0 ? jp : 0;          // P == 0: the single segment holds the totals
  const double sp = P > 0 ? seg[rp * NS + Q + 2] : 1.0;
  const double rho = P > 0 ? seg[rp * NS] : 0.0;
  const double isp = 1.0 / sp;

  // this lane's Gram channels c = t*16 + (lane & 15): mean and pivot-row value
  const int li = lane & 15, lk = lane >> 4;
  double muc[TT], gpc[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int c = t * 16 + li;
    muc[t] = (c >= 1 && c <= Q) ? acc[NG + Q + c - 1] * iSc : 0.0;
    const double W = seg[rp * NS];
    const double raw = c < NC ? seg[rp * NS + c] : 0.0;
    gpc[t] = (c >= 1 && c <= Q) ? (raw - muc[t] * W) * isig : raw;
    if (lk == 0 && c < NC) gpv[c] = gpc[t];
    if (lk == 0 && c >= 1 && c <= Q) muv[c - 1] = muc[t];
  }

  // per-industry scalars once, lane-parallel: a_j and 1/W_j (0 for pivot / empty / padding)
  for (int j = lane; j < P4; j += 64) {
    const double W = j < P ? seg[j * NS] : 0.0;
    const bool act = (j < P) && (j != jp) && (W > 0.0);
    ajv[j] = act ? -seg[j * NS + Q + 2] * isp : 0.0;
    iwv[j] = act ? 1.0 / W : 0.0;
  }
  wave_sync_lds();

  // Gram over active industries: A = [m/W | a/W | 1], B = [m | a | 0]
  v4d G[TT][TT];
#pragma unroll
  for (int ti = 0; ti < TT; ++ti)
#pragma unroll
    for (int tj = 0; tj < TT; ++tj) G[ti][tj] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < P4; k0 += 4) {
    const int j = k0 + lk;
    const double* p = seg + (j < P ? j : 0) * NS;
    const double W = p[0];
    const double aj = ajv[j], iW = iwv[j];
    const bool act = iW != 0.0;
    double av[TT], bv[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      const int c = t * 16 + li;
      const double raw = c < NC ? p[c] : 0.0;
      const double g = (c >= 1 && c <= Q) ? (raw - muc[t] * W) * isig : raw;
      const double m = g + aj * gpc[t];
      const double v = c < NC ? m : (c == NC ? aj : 0.0);
      bv[t] = act ? v : 0.0;
      av[t] = act ? (c == NC + 1 ? 1.0 : v * iW) : 0.0;
    }
#pragma unroll
    for (int ti = 0; ti < TT; ++ti)
#pragma unroll
      for (int tj = 0; tj < TT; ++tj)
        G[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ti], bv[tj], G[ti][tj], 0, 0, 0);
  }
#pragma unroll
  for (int ti = 0; ti < TT; ++ti)
#pragma unroll
    for (int tj = 0; tj < TT; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ti * 16 + lk + 4 * r, w = tj * 16 + li;
        if (i < CH && w < CH) Gs[i * CH + w] = G[ti][tj][r];
      }
  wave_sync_lds();
  stamp(2);

  // uniform scalars; S = M_DD - G + kappa at at^T in the MFMA output layout
  const double c0 = Gs[NC * CH + NC];
  const double kappa = rho / (1.0 + rho * c0);
  const double sa = Gs[(NC + 1) * CH + NC];  // sum of a_j over active industries
  // industry totals of the standardised rows: sum_active m + (1 - sum a) g_p
  auto tot = [&](int w) { return Gs[(NC + 1) * CH + w] + (1.0 - sa) * gpv[w]; };
  const double Sw = tot(0);
#pragma unroll
  for (int ti = 0; ti < TT; ++ti)
#pragma unroll
    for (int tj = 0; tj < TT; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int u = ti * 16 + lk + 4 * r, w = tj * 16 + li;
        if (u >= ND || w >= NC) continue;
        double m;
        if (u == 0) {
          m = tot(w);
        } else if (w == 0) {
          m = tot(u);
        } else if (w == ND) {
          m = acc[NG + u - 1] * isig - muv[u - 1] * isig * tot(ND);
        } else {
          const int q = u - 1, s2 = w - 1;
          const int hi = q > s2 ? q : s2, lo = q > s2 ? s2 : q;
          const double muq = muv[q], mus = muv[s2];
          m = (acc[hi * (hi + 1) / 2 + lo] - muq * mus * Sw) * isig * isig -
              (muq * tot(w) + mus * tot(u)) * isig;
        }
        S[u * NC + w] = m - G[ti][tj][r] + kappa * Gs[NC * CH + u] * Gs[NC * CH + w];
      }
  wave_sync_lds();
  stamp(3);

  // Cholesky of the ND x ND Schur complement, right-looking (one dependent step per column),
  // in registers, redundantly in every lane; 1/sqrt from v_rsq_f64 + two Newton steps.
  double Lm[ND * (ND + 1) / 2], b[ND], dorig[ND], il[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
#pragma unroll
    for (int k = 0; k <= i; ++k) Lm[i * (i + 1) / 2 + k] = S[i * NC + k];
    b[i] = S[i * NC + ND];
    dorig[i] = Lm[i * (i + 1) / 2 + i];
  }
  double dmax = 0.0;
#pragma unroll
  for (int k = 0; k < ND; ++k) dmax = fmax(dmax, fabs(dorig[k]));
  const double ztol = tol * dmax;
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const double dk = Lm[k * (k + 1) / 2 + k];
    if (!(dk > ztol)) {  // pinv semantics: drop the direction (exactly singular block)
      st |= (dorig[k] > ztol) ? XS_NEAR_SINGULAR : XS_ZERO_PIVOT;
      il[k] = 0.0;
#pragma unroll
      for (int i = k; i < ND; ++i) Lm[i * (i + 1) / 2 + k] = 0.0;
      continue;
    }
    if (dk < 1e-12 * dorig[k]) st |= XS_NEAR_SINGULAR;
    double y = __builtin_amdgcn_rsq(dk);
    y = fma(0.5 * y, fma(-dk * y, y, 1.0), y);
    y = fma(0.5 * y, fma(-dk * y, y, 1.0), y);
    il[k] = y;
    Lm[k * (k + 1) / 2 + k] = dk * y;
#pragma unroll
    for (int i = k + 1; i < ND; ++i) Lm[i * (i + 1) / 2 + k] *= y;
#pragma unroll
    for (int i = k + 1; i < ND; ++i)
#pragma unroll
      for (int c = k + 1; c <= i; ++c)
        Lm[i * (i + 1) / 2 + c] = fma(-Lm[i * (i + 1) / 2 + k], Lm[c * (c + 1) / 2 + k],
                                      Lm[i * (i + 1) / 2 + c]);
  }
#pragma unroll
  for (int k = 0; k < ND; ++k) {  // L y = b, column-oriented (il = 0 zeroes dropped directions)
    b[k] *= il[k];
#pragma unroll
    for (int i = k + 1; i < ND; ++i) b[i] = fma(-Lm[i * (i + 1) / 2 + k], b[k], b[i]);
  }
#pragma unroll
  for (int k = ND - 1; k >= 0; --k) {  // L^T g = y
    b[k] *= il[k];
#pragma unroll
    for (int i = 0; i < k; ++i) b[i] = fma(-Lm[k * (k + 1) / 2 + i], b[k], b[i]);
  }
  stamp(4);

  // industries: f_j = (m_j . h - kappa a_j z) / W_j with h = [-g_D, 1]; pivot f_p = z (1 - kappa c0)
  double z = Gs[NC * CH + ND], gph = gpv[ND];
#pragma unroll
  for (int u = 0; u < ND; ++u) {
    z = fma(-Gs[NC * CH + u], b[u], z);
    gph = fma(-gpv[u], b[u], gph);
  }
  const bool bad = (st & XS_BAD) != 0;
  double* fo = fout + (size_t)d * K;
  for (int j = lane; j < P; j += 64) {
    const double* p = seg + j * NS;
    const double W = p[0];
    double fj = 0.0;
    if (j == jp) {
      fj = z * (1.0 - kappa * c0);
    } else if (W > 0.0) {
      const double aj = -p[Q + 2] * isp;
      double mh = p[ND];  // g_j . h  (g_j[ND] = B_j, h[ND] = 1)
      mh = fma(-W, b[0], mh);
#pragma unroll
      for (int q = 0; q < Q; ++q) mh = fma(-(p[1 + q] - muv[q] * W) * isig, b[1 + q], mh);
      fj = (mh + aj * gph - kappa * aj * z) * iwv[j];
    }
    fo[1 + j] = bad ? qnan() : fj;
    co[Q + 1 + j] = bad ? qnan() : fj;
  }
  if (lane == 0) fo[0] = bad ? qnan() : b[0];
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (lane == q) {
      fo[1 + P + q] = bad ? qnan() : b[1 + q];
      co[q] = bad ? qnan() : b[1 + q] * isig;  // residual coefficients on RAW styles
    }
  if (lane == 0) {
    double cst = b[0];
#pragma unroll
    for (int q = 0; q < Q; ++q) cst -= b[1 + q] * isig * muv[q];
    co[Q] = bad ? qnan() : cst;
    status[d] = st;
    if (st_lds) *st_lds = st;
  }
  if (stats) {
    double* sd = stats + (size_t)d * (Q + 2);
    if (lane < Q) sd[lane] = muv[lane];
    if (lane == Q) sd[Q] = sigma;
    if (lane == Q + 1) sd[Q + 1] = nval;
  }
  stamp(5);
}

template <int Q>
__global__ __launch_bounds__(64) void xs_solve_kernel(const double* __restrict__ mom, int P,
                                                      int Pseg, int pivot_mode, double tol,
                                                      double* __restrict__ fout,
                                                      double* __restrict__ coef,
                                                      double* __restrict__ stats,
                                                      int* __restrict__ status,
                                                      long long* __restrict__ stamps) {
  extern __shared__ double sm[];
  const int d = blockIdx.x;
  const int lane = threadIdx.x;
  if (stamps && lane == 0) stamps[(size_t)d * 8] = __builtin_amdgcn_s_memtime();
  const int MS = Layout<Q>::msize(Pseg);
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
  solve_body<Q>(sm, d, P, Pseg, pivot_mode, tol, fout, coef + (size_t)d * (Q + 1 + P), stats,
                status, nullptr, stamps);
}

// ------------------------------------------------------------------------------------------
// K3: specific returns and R^2 (dates visited in reverse: MALL-resident tail of K1 first)
// ------------------------------------------------------------------------------------------
// Specific returns + R^2 of date d from the coefficients `cf_s` [Q+1+P] (LDS) by the whole
// workgroup (<= 16 waves); `red` = 16 x 5 doubles of LDS.
// Residual-pass data of 4 consecutive stocks x UP iterations, loaded by waves 1..3 while wave 0
// solves (fused kernel, `kPre`): the pass then starts with 1536 stocks already in registers.
#ifndef MFA_XS_PREU
#define MFA_XS_PREU 2
#endif
constexpr int kPreU = MFA_XS_PREU;
constexpr int kPreStocks = 3 * 64 * 4 * kPreU;
template <int Q>
struct ResidPre {
  float4 c4[kPreU], r4[kPreU], x4[kPreU][Q];
  uint2 j4[kPreU];
};

template <int Q>
__device__ __forceinline__ void resid_prefetch(const float* __restrict__ X,
                                               const float* __restrict__ cap,
                                               const float* __restrict__ ret,
                                               const int16_t* __restrict__ ind, int d, int N,
                                               ResidPre<Q>& pr) {
  const int nlo = N > kPreStocks ? N - kPreStocks : 0;
  const int t = threadIdx.x - 64;  // waves 1..3
  const float* Xd = X + (size_t)d * Q * N;
#pragma unroll
  for (int u = 0; u < kPreU; ++u) {
    const int n = nlo + t * 4 + u * 768;
    if (n < N) {
      pr.c4[u] = *(const float4*)(cap + (size_t)d * N + n);
      pr.r4[u] = *(const float4*)(ret + (size_t)d * N + n);
#pragma unroll
      for (int q = 0; q < Q; ++q) pr.x4[u][q] = *(const float4*)(Xd + (size_t)q * N + n);
      pr.j4[u] = ind ? *(const uint2*)(ind + (size_t)d * N + n) : make_uint2(0u, 0u);
    }
  }
}

// pre != nullptr: waves 1..3 hold the last kPreStocks stocks in `pre` (resid_prefetch) and the
// main loop covers [0, N - kPreStocks) only.
template <int Q, bool PRE = false>
__device__ __forceinline__ void resid_body(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int d, int N, int P, const double* cf_s, bool bad,
    float* __restrict__ eout, double* __restrict__ r2out, double (*red)[5],
    const ResidPre<Q>& pre = ResidPre<Q>{}, double* __restrict__ sums_out = nullptr) {
  const int tid = threadIdx.x;
  const int Pseg = P > 0 ? P : 1;
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
  // Four consecutive stocks per thread (16-byte loads; N % 8 == 0 keeps rows aligned) and U
  // iterations' loads issued before any is consumed: the pass is latency-bound otherwise.
  constexpr int U = 3;
  const int step = blockDim.x * 4;
  auto one = [&](float c, float r, int j, const float (&xf)[Q]) -> float {
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
    return eo;
  };
  auto consume4 = [&](const float4& c4, const float4& r4, const float4 (&x4)[Q], uint2 j4, int n) {
    const int js[4] = {(int)(short)(j4.x & 0xFFFF), (int)(short)(j4.x >> 16),
                       (int)(short)(j4.y & 0xFFFF), (int)(short)(j4.y >> 16)};
    const float cs[4] = {c4.x, c4.y, c4.z, c4.w};
    const float rs[4] = {r4.x, r4.y, r4.z, r4.w};
    float eo[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float xf[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) xf[q] = ((const float*)&x4[q])[k];
      eo[k] = one(cs[k], rs[k], js[k], xf);
    }
    if (ed) *(float4*)(ed + n) = make_float4(eo[0], eo[1], eo[2], eo[3]);
  };
  int Nmain = N;
  if constexpr (PRE) {
    const int nlo = N > kPreStocks ? N - kPreStocks : 0;
    Nmain = nlo;
    if (tid >= 64) {
#pragma unroll
      for (int u = 0; u < kPreU; ++u) {
        const int n = nlo + (tid - 64) * 4 + u * 768;
        if (n < N) consume4(pre.c4[u], pre.r4[u], pre.x4[u], pre.j4[u], n);
      }
    }
  }
  // Blocks of U*step stocks walked from the END of the date: the moments pass streamed the
  // tail last, so the re-read starts with the lines most likely still in the Infinity Cache.
  const int nblk = (Nmain + U * step - 1) / (U * step);
  for (int b = nblk - 1; b >= 0; --b) {
    const int n0 = b * U * step + tid * 4;
    float4 c4[U], r4[U], x4[U][Q];
    uint2 j4[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n0 + u * step;
      if (n < Nmain) {
        c4[u] = *(const float4*)(cd + n);
        r4[u] = *(const float4*)(rd + n);
#pragma unroll
        for (int q = 0; q < Q; ++q) x4[u][q] = *(const float4*)(Xd + (size_t)q * N + n);
        j4[u] = id ? *(const uint2*)(id + n) : make_uint2(0u, 0u);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n0 + u * step;
      if (n < Nmain) consume4(c4[u], r4[u], x4[u], j4[u], n);
    }
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
    if (sums_out) {  // stock-sharded regression: the caller all-reduces, then forms R^2
      double* so = sums_out + (size_t)d * 5;
      so[0] = a; so[1] = b; so[2] = c; so[3] = e2; so[4] = n;
    } else {
      const double ve = b / n - (a / n) * (a / n);
      const double vr = e2 / n - (c / n) * (c / n);
      r2out[d] = bad ? qnan() : 1.0 - ve / vr;
    }
  }
}

template <int Q>
__global__ __launch_bounds__(256) void xs_resid_kernel(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int D, int N, int P, const double* __restrict__ coef,
    const int* __restrict__ status, float* __restrict__ eout, double* __restrict__ r2out,
    double* __restrict__ sums_out = nullptr) {
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red[16][5];
  const int d = D - 1 - blockIdx.x;
  const double* co = coef + (size_t)d * (Q + 1 + P);
  for (int i = threadIdx.x; i < Q + 1 + P; i += blockDim.x) cf_s[i] = co[i];
  __syncthreads();
  resid_body<Q>(X, cap, ret, ind, d, N, P, cf_s, (status[d] & XS_BAD) != 0, eout, r2out, red,
                ResidPre<Q>{}, sums_out);
}

// ------------------------------------------------------------------------------------------
// Fused K1 -> K2 -> K3: one 4-wave workgroup per date streams the date's panel slice once
// from HBM (moments), solves it in wave 0, then re-reads the slice for the residual pass.
// Two workgroups fit per CU, so ~512 dates (~128 MB of panel) are in flight: the re-read is
// served by the 256 MB Infinity Cache instead of HBM, and the single-wave solve of one date
// overlaps the other workgroup's streaming.  HBM traffic drops from ~2x to ~1x the panel.
// ------------------------------------------------------------------------------------------
template <int Q, int NW>
constexpr int fused_ring_bytes() {
  constexpr int a = NW * Ring<Q>::RINGW;
  constexpr int b = (int)(solve_lds_doubles<Q>(128) * 8);
  return a > b ? a : b;
}

// NW = waves per workgroup: 4 (two workgroups per CU) or 2 (four per CU: more dates in flight,
// so a date's solve / residual phase overlaps three streaming dates instead of one).
template <int Q, int R, int VAR = 0, int NW = 4, bool PRE = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void xs_fused_kernel(
    const float* __restrict__ X, const float* __restrict__ cap, const float* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int P, int Pseg, int pivot_mode, double tol,
    double* __restrict__ fout, float* __restrict__ eout, double* __restrict__ r2out,
    double* __restrict__ stats, int* __restrict__ status, long long* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) char ring[fused_ring_bytes<Q, NW>()];
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red[4][5];
  __shared__ int st_s;
  extern __shared__ double dyn[];
  const int d = blockIdx.x;
  // optional per-date phase stamps (s_memtime) + hardware ids for occupancy analysis
  auto stamp = [&](int k) {
    if (stamps && threadIdx.x == 0) stamps[(size_t)d * 8 + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  double* sm = (double*)ring;  // moments, then the solve's scratch (ring is idle by then)
  moments_body<Q, VAR & 35, R>(X, cap, ret, ind, N, Pseg, d, ring, dyn, sm);
  stamp(1);
  if constexpr ((VAR & 8) != 0) {  // timing-only ablation: no solve
    for (int i = threadIdx.x; i < Q + 1 + P; i += blockDim.x) cf_s[i] = sm[i] * 1e-30;
    if (threadIdx.x == 0) st_s = 0;
  } else if (threadIdx.x < 64) {
    // solve-internal phase stamps go to the second [D][8] block of the stamp buffer
    long long* ss = stamps ? stamps + (size_t)gridDim.x * 8 : nullptr;
    if (ss && threadIdx.x == 0) ss[(size_t)d * 8] = __builtin_amdgcn_s_memtime();
    solve_body<Q>(sm, d, P, Pseg, pivot_mode, tol, fout, cf_s, stats, status, &st_s, ss);
  }
  ResidPre<Q> pre;
  if constexpr (PRE && NW == 4) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0)
      resid_prefetch<Q>(X, cap, ret, ind, d, N, pre);
  }
  __syncthreads();
  stamp(2);
  if constexpr ((VAR & 4) == 0)
    resid_body<Q, PRE && NW == 4>(X, cap, ret, ind, d, N, P, cf_s, (st_s & XS_BAD) != 0, eout,
                                  r2out, red, pre);
  if constexpr ((VAR & 16) != 0) {  // timing-only: a second residual pass (cache-hit cost)
    __syncthreads();
    resid_body<Q>(X, cap, ret, ind, d, N, P, cf_s, (st_s & XS_BAD) != 0, eout, r2out, red);
  }
  stamp(3);
  if (stamps && threadIdx.x == 0) {
    stamps[(size_t)d * 8 + 4] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    stamps[(size_t)d * 8 + 5] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
}

constexpr int kXsDeterministic = 0x100;  // pivot_mode flag: bitwise-deterministic kernel
long long* g_stamps = nullptr;  // debug: per-date K2 phase stamps [D][8]
int g_xs_mode = 0;              // 0 = fused single kernel, 1 = three kernels (ablation)

template <int Q, int VAR = 0>
hipError_t launch_q(const float* X, const float* cap, const float* ret, const int16_t* ind,
                    int D, int N, int P, int pivot_mode, double tol, double* f, float* e,
                    double* r2, double* stats, int* status, double* ws, hipStream_t s) {
  using L = Layout<Q>;
  const int Pseg = P > 0 ? P : 1;
  const int K = 1 + P + Q;
  const int MS = L::msize(Pseg);
  double* mom = ws;
  double* coef = ws + (size_t)D * MS;
  const size_t ring = Ring<Q>::BYTES;
  const size_t seg8 = (size_t)kRepMax * Pseg * L::NS * sizeof(double);
  const bool rep8 = seg8 <= kSegLdsBudget;
  const size_t lds1 = ((rep8 ? (size_t)kRepMax : 1) * Pseg * L::NS + L::NACC) * sizeof(double);
  constexpr int CH = Q + 4;
  const size_t P4 = ((size_t)Pseg + 3) & ~(size_t)3;
  const size_t lds2 = ((size_t)L::msize(Pseg) + CH * CH + L::ND * (L::ND + 1) + (Q + 2) + Q +
                       2 * P4) * sizeof(double);
  if (lds1 + ring > 160 * 1024 || lds2 > 64 * 1024) return hipErrorInvalidValue;
  const int16_t* indp = P > 0 ? ind : nullptr;
  if (pivot_mode & kXsDeterministic) {  // bitwise-reproducible variant of the default path
    if (!rep8) return hipErrorNotSupported;
    hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32, 4, true>), dim3(D), dim3(256), lds1,
                       s, X, cap, ret, indp, N, P, Pseg, pivot_mode & 0xff, tol, f, e, r2, stats,
                       status, nullptr);
    return hipGetLastError();
  }
  if (g_xs_mode == 3 || g_xs_mode == 4) {  // 2-wave workgroups, 2 segment replicas
    long long* st = g_xs_mode == 4 ? g_stamps : nullptr;
    const size_t lds2w = ((size_t)2 * Pseg * L::NS + L::NACC) * sizeof(double);
    if (lds2w + fused_ring_bytes<Q, 2>() + 2048 <= 40 * 1024) {
      hipLaunchKernelGGL((xs_fused_kernel<Q, 2, VAR, 2>), dim3(D), dim3(128), lds2w, s, X, cap, ret,
                         indp, N, P, Pseg, pivot_mode, tol, f, e, r2, stats, status, st);
      return hipGetLastError();
    }
  }
  // default: residual prefetch by waves 1..3 during the wave-0 solve (mode 0 / 5; 6 = stamps)
  if (g_xs_mode == 0 || g_xs_mode == 5 || g_xs_mode == 6) {
    long long* st = g_xs_mode == 6 ? g_stamps : nullptr;
    if (rep8) {
      hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR, 4, true>), dim3(D), dim3(256), lds1, s,
                         X, cap, ret, indp, N, P, Pseg, pivot_mode, tol, f, e, r2, stats, status, st);
      return hipGetLastError();
    }
  }
  if (g_xs_mode == 0 || g_xs_mode == 2 || g_xs_mode == 3 || g_xs_mode == 4 || g_xs_mode >= 5) {
    // (mode 7: fused without the residual prefetch; also the fallback for large P)
    long long* st = (g_xs_mode == 2 || g_xs_mode == 4) ? g_stamps : nullptr;
    if (rep8)
      hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR>), dim3(D), dim3(256), lds1, s, X, cap, ret,
                         indp, N, P, Pseg, pivot_mode, tol, f, e, r2, stats, status, st);
    else
      hipLaunchKernelGGL((xs_fused_kernel<Q, 1>), dim3(D), dim3(256), lds1, s, X, cap, ret, indp,
                         N, P, Pseg, pivot_mode, tol, f, e, r2, stats, status, st);
    return hipGetLastError();
  }
  if (rep8)
    hipLaunchKernelGGL((xs_moments_kernel<Q, VAR, kRepMax>), dim3(D), dim3(256), lds1, s, X, cap,
                       ret, indp, N, Pseg, mom);
  else
    hipLaunchKernelGGL((xs_moments_kernel<Q, VAR, 1>), dim3(D), dim3(256), lds1, s, X, cap, ret,
                       indp, N, Pseg, mom);
  hipLaunchKernelGGL(xs_solve_kernel<Q>, dim3(D), dim3(64), lds2, s, mom, P, Pseg, pivot_mode, tol,
                     f, coef, stats, status, g_stamps);
  if (!(VAR & 4))
    hipLaunchKernelGGL(xs_resid_kernel<Q>, dim3(D), dim3(256), 0, s, X, cap, ret, indp, D, N, P,
                       coef, status, e, r2);
  return hipGetLastError();
}

}  // namespace

// Debug: record K2 phase timestamps (s_memtime) into buf[D][8] on the next calls (null = off).
MFA_API void mfa_xs_set_stamps(long long* buf) { g_stamps = buf; }

// Ablation: 0 = fused single-kernel path with the residual prefetch during the solve (default),
// 1 = three separate kernels, 2 = fused (no prefetch) with per-date phase stamps into the
// mfa_xs_set_stamps buffer, 3 / 4 = fused with 2-wave workgroups (without / with stamps),
// 5 / 6 = default path (without / with stamps), 7 = fused without the prefetch.
MFA_API void mfa_xs_set_mode(int mode) { g_xs_mode = mode; }

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
// status [D] int32 XsStatus bits.  pivot_mode: 0 = last non-empty industry, 1 = reference;
// | 0x100 = bitwise-deterministic kernel (needs the 8-replica segment table: P <= 59 at Q = 10).
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

// Timing-only ablation entry (Q = 10): bit 1 = no segment atomics, bit 2 = no style-Gram FMAs,
// bit 4 = no residual pass, bit 8 = no solve (fused mode only).
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
    MFA_V(0) MFA_V(1) MFA_V(2) MFA_V(3) MFA_V(4) MFA_V(5) MFA_V(6) MFA_V(7) MFA_V(8)
    MFA_V(12) MFA_V(15) MFA_V(16) MFA_V(20)
#undef MFA_V
  }
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------
// Stock-sharded (TP) regression pieces, SURVEY.md §2.5: every rank streams ITS stocks of every
// date into raw moments (additive: the caller all-reduces them), solves redundantly from the
// summed moments, and forms its stocks' specific returns plus the five R^2 sums
// [sum e, sum e^2, sum r, sum r^2, n] per date (all-reduced again by the caller).
// ------------------------------------------------------------------------------------------
namespace {
template <int Q>
hipError_t split_q(int what, const float* X, const float* cap, const float* ret,
                   const int16_t* ind, int D, int N, int P, int pivot_mode, double tol,
                   double* mom, double* f, double* coef, double* stats, int* status, float* e,
                   double* sums, hipStream_t s) {
  using L = Layout<Q>;
  const int Pseg = P > 0 ? P : 1;
  const int16_t* indp = P > 0 ? ind : nullptr;
  if (what == 0) {
    const size_t seg8 = (size_t)kRepMax * Pseg * L::NS * sizeof(double);
    const bool rep8 = seg8 <= kSegLdsBudget;
    const size_t lds1 = ((rep8 ? (size_t)kRepMax : 1) * Pseg * L::NS + L::NACC) * sizeof(double);
    if (lds1 + Ring<Q>::BYTES > 160 * 1024) return hipErrorInvalidValue;
    if (rep8)
      hipLaunchKernelGGL((xs_moments_kernel<Q, 0, kRepMax>), dim3(D), dim3(256), lds1, s, X, cap,
                         ret, indp, N, Pseg, mom);
    else
      hipLaunchKernelGGL((xs_moments_kernel<Q, 0, 1>), dim3(D), dim3(256), lds1, s, X, cap, ret,
                         indp, N, Pseg, mom);
  } else if (what == 1) {
    constexpr int CH = Q + 4;
    const size_t P4 = ((size_t)Pseg + 3) & ~(size_t)3;
    const size_t lds2 = ((size_t)L::msize(Pseg) + CH * CH + L::ND * (L::ND + 1) + (Q + 2) + Q +
                         2 * P4) * sizeof(double);
    if (lds2 > 64 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xs_solve_kernel<Q>, dim3(D), dim3(64), lds2, s, mom, P, Pseg, pivot_mode,
                       tol, f, coef, stats, status, (long long*)nullptr);
  } else {
    hipLaunchKernelGGL(xs_resid_kernel<Q>, dim3(D), dim3(256), 0, s, X, cap, ret, indp, D, N, P,
                       coef, status, e, (double*)nullptr, sums);
  }
  return hipGetLastError();
}

int split_dispatch(int what, const float* X, const float* cap, const float* ret,
                   const int16_t* ind, int D, int N, int P, int Q, int pivot_mode, double tol,
                   double* mom, double* f, double* coef, double* stats, int* status, float* e,
                   double* sums, void* stream) {
  if (D <= 0) return 0;
  if (Q < 1 || Q > 16 || P < 0 || P > 128 || N < 0 || (N % 8) != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  switch (Q) {
#define MFA_Q(qq)                                                                              \
  case qq:                                                                                     \
    return (int)split_q<qq>(what, X, cap, ret, ind, D, N, P, pivot_mode, tol, mom, f, coef,     \
                            stats, status, e, sums, s);
    MFA_Q(1) MFA_Q(2) MFA_Q(3) MFA_Q(4) MFA_Q(5) MFA_Q(6) MFA_Q(7) MFA_Q(8)
    MFA_Q(9) MFA_Q(10) MFA_Q(11) MFA_Q(12) MFA_Q(13) MFA_Q(14) MFA_Q(15) MFA_Q(16)
#undef MFA_Q
  }
  return (int)hipErrorInvalidValue;
}
}  // namespace

// Raw moments [D][msize] of this rank's stocks (layout: Layout<Q>, see K1 above).
MFA_API int mfa_xs_moments(const float* X, const float* cap, const float* ret, const int16_t* ind,
                           int D, int N, int P, int Q, double* mom, void* stream) {
  return split_dispatch(0, X, cap, ret, ind, D, N, P, Q, 0, 0.0, mom, nullptr, nullptr, nullptr,
                        nullptr, nullptr, nullptr, stream);
}

// Constrained solve from (summed) moments: f [D][1+P+Q], coef [D][Q+1+P], stats, status.
MFA_API int mfa_xs_solve(const double* mom, int D, int P, int Q, int pivot_mode, double tol,
                         double* f, double* coef, double* stats, int* status, void* stream) {
  return split_dispatch(1, nullptr, nullptr, nullptr, nullptr, D, 0, P, Q, pivot_mode, tol,
                        (double*)mom, f, coef, stats, status, nullptr, nullptr, stream);
}

// Specific returns of this rank's stocks (e nullable) + per-date R^2 sums [D][5].
MFA_API int mfa_xs_resid_sums(const float* X, const float* cap, const float* ret,
                              const int16_t* ind, int D, int N, int P, int Q, const double* coef,
                              const int* status, float* e, double* sums, void* stream) {
  return split_dispatch(2, X, cap, ret, ind, D, N, P, Q, 0, 0.0, nullptr, nullptr,
                        (double*)coef, nullptr, (int*)status, e, sums, stream);
}

// Bytes per date of the raw-moment layout (msize doubles).
MFA_API size_t mfa_xs_moments_bytes(int P, int Q) {
  const int Pseg = P > 0 ? P : 1;
  return ((size_t)Q * (Q + 1) / 2 + 2 * Q + 4 + (size_t)Pseg * (Q + 3)) * sizeof(double);
}
