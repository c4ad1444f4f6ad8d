// Batched cross-sectional WLS factor-return regression (Barra CNE5/USE4 style) for gfx950,
// templated on the panel's storage type T (float or double).  Included by xs_wls.hip (fp32
// panels) and xs_wls_f64.hip (fp64 panels: the reference reads float64 CSV exposures,
// Barra-master/demo.py:21-35, and regresses them in float64, mfm/CrossSection.py:57-108).
//
// Reference semantics: Barra-master/mfm/CrossSection.py:12-20 (style z-score: cap-weighted mean,
// ONE pooled ddof-0 std) and :57-108 (sqrt-cap WLS, industry-neutral constraint
// sum_j s_j f_j = 0 via the K x (K-1) matrix R, pinv solve, f = Omega r, e = r - X f,
// unweighted R^2).  Nothing mirrors the reference's dense N x N weight matrix.
//
// Three phases, all dates of a shard per launch (fused into one kernel by default):
//   K1 moments   HBM streaming.  Every wave streams its own 64-stock tiles of the [D][Q][N]
//                styles, caps, returns and int16 industry ids through a private LDS ring
//                filled by global_load_lds (4 B per lane for fp32 rows; 16 B per lane, two
//                512-B fp64 rows per instruction, for fp64), with counted vmcnt and no workgroup
//                barrier until the date's final reduction.  RAW fp64 moments accumulate in
//                registers; the one-hot industry block is a segmented sum done with ds_add_f64
//                into an R-way replicated [P][Q+3] table laid out so one issue group is <= 2-way
//                conflicted.  z-scoring is folded in algebraically later: the data is read once.
//   K2 solve     latency-bound tiny algebra.  One wave per date: after eliminating the pivot
//                industry the industry block is diag(W) + rho a a^T (Sherman-Morrison), and
//                only the (1+Q) x (1+Q) Schur complement is Cholesky-factorised, row-per-lane
//                in registers.  Exactly-empty industries get f = 0 (pinv semantics); near-
//                singular dates are flagged for the pseudo-inverse refinement pass.
//   K3 resid     HBM / Infinity-Cache streaming, low VGPR count: specific returns (stored in T)
//                + R^2.  16-byte vector loads (4 fp32 / 2 fp64 stocks per lane).
#pragma once
#include "common.h"
#include "jacobi.h"

#include <utility>

// CS-WLS execution mode shared by the fp32 and fp64 translation units (mfa_xs_set_mode):
// 0 = fused single kernel (with the residual prefetch during the solve: fp32 panels, and fp64
// panels on the LDS-DMA moments path), 1 = three separate kernels (ablation / large-P
// fallback), 7 = fused without the prefetch, 23 / 24 = prefetch forced on the plain-load /
// LDS-DMA path (A/B), 30 = resident fused kernel (fp64, Q = 10; xs_resident_kernel), 31 = the
// deterministic LDS-DMA fused kernel whatever the default.
extern int g_mfa_xs_mode;
// Stock chunks per date: 0 = automatic (chunked below kXsChunkMinD dates), > 0 forced, < 0 never.
extern int g_mfa_xs_chunks;
// Team (pipelined) CS-WLS kernel: 0 = off, > 0 = forced chunks per date, < 0 = automatic.
extern int g_mfa_xs_coop;
// Pipelined team kernel: residual pass `lag` tickets behind the moments (1..kPipeMaxLag), and
// the persistent grid's workgroups per CU (0 = the occupancy limit).
extern int g_mfa_xs_lag;
extern int g_mfa_xs_pipe_wpc;
// Phase timestamps of the resident kernel ([D][6] u64: wall clock at start / moments / reduction /
// solve / end, hardware id), null = off (mfa_xs_set_prof, timing tools only).
extern unsigned long long* g_mfa_xs_prof;

namespace mfa_xs {

using namespace mfa;

enum XsStatus : int {
  XS_NO_ROWS = 1,        // no valid stock on the date
  XS_PIVOT_EMPTY = 2,    // constraint pivot industry has zero capital
  XS_NEAR_SINGULAR = 4,  // Schur Cholesky lost > 12 digits: refined with the pseudo-inverse
  XS_ZERO_PIVOT = 8,     // exactly-zero pivots / empty industries (pinv semantics -> f = 0)
  XS_BAD_SIGMA = 16,     // pooled style std is zero / NaN
  XS_REFINED = 32,       // re-solved on the device with the eigen pseudo-inverse (pinv)
  XS_PINV_CUT = 128,     // that pinv dropped an eigen-direction below 1e-15 lambda_max (a
                         // numerically rank-deficient system, not necessarily an exactly
                         // singular one: np.linalg.inv would not raise on it)
};
constexpr int XS_BAD = XS_NO_ROWS | XS_BAD_SIGMA | XS_PIVOT_EMPTY;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

template <typename T>
__device__ __forceinline__ bool finite_v(T v) { return __builtin_isfinite(v); }

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

// LDS reads of an LDS-DMA ring slot from inline asm: a compiler-visible LDS read while any
// global_load_lds is in flight gets a vmcnt(0) from hipcc's waitcnt pass (it cannot tell the
// slots apart), which drained the prefetched tiles before every tile's compute.  The caller
// waits with lgkmcnt(0) before using the values.
template <int OFF>
__device__ __forceinline__ double lds_ld(unsigned a, double) {
  double v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ float lds_ld(unsigned a, float) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return v;
}
template <typename V>
__device__ __forceinline__ void reg_fence(V& v) {
  asm volatile("" : "+v"(v));
}
__device__ __forceinline__ int lds_ld_i16(unsigned a) {
  int v;
  asm volatile("ds_read_i16 %0, %1" : "=v"(v) : "v"(a));
  return v;
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

#ifndef MFA_XS_NT_AUX
#define MFA_XS_NT_AUX 0
#endif
// Stores of auxiliary per-date outputs (moment export, validity masks): non-temporal when
// MFA_XS_NT_AUX, so they do not take Infinity-Cache space from panel lines awaiting re-read.
template <typename V>
__device__ __forceinline__ void aux_store(V* p, V v) {
  if constexpr (MFA_XS_NT_AUX) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef MFA_XS_REP
#define MFA_XS_REP 8
#endif
// Segment-table replicas: entry (j, ch) owns R consecutive doubles and lane l adds into slot
// l & (R-1).  With R = 8 the 16 lanes of a ds_add_f64 issue group land on bank pairs
// (l & 7) + 8 * ((j*NS + ch) & 1): at most 2-way conflicts whatever the industry mix (4
// lane-strided replicas measured 8.3 conflict cycles per instruction).
constexpr int kRepMax = MFA_XS_REP;
constexpr int kXsSegPad = 2;  // doubles of padding per industry segment (LDS bank spread)
constexpr int kSegLdsBudget = 48 * 1024;  // R = 8 only while the table leaves 2 WGs / CU
// Industries of the split path (moments -> solve -> refine -> residual kernels): the fused
// kernel's in-kernel solve is sized for P <= 128 (its ring doubles as the solve's LDS); wider
// industry sets (K > 145 risk models) take the split kernels, whose per-date solve LDS stays
// within 64 KB and structured pinv within 160 KB up to 256 industries at Q = 16.
constexpr int kXsSplitMaxP = 256;
constexpr int kWT = 64;                   // stocks per wave tile (K1: one stock per lane)

// Per-type streaming parameters.  fp32: 4-slot ring of 3.2 KB tiles; fp64: 2-slot ring of
// 6.3 KB tiles (4 waves x 2 x 6.3 KB + the segment table keeps 2 workgroups per CU).
template <typename T> struct Stream;
template <> struct Stream<float> {
  static constexpr int RING = 4;
  static constexpr int VEC = 4;  // residual pass: stocks per 16-byte load
  static constexpr int U = 3;    // residual iterations in flight
};
#ifndef MFA_XS_U64
#define MFA_XS_U64 2
#endif
template <> struct Stream<double> {
  static constexpr int RING = 2;
  static constexpr int VEC = 2;
  static constexpr int U = MFA_XS_U64;
};

template <int Q, typename T>
struct Layout {
  static constexpr int NS = Q + 3;             // per-industry channels: W, A_q, B, s
  static constexpr int NG = Q * (Q + 1) / 2;   // packed symmetric raw Gram
  static constexpr int NACC = NG + 2 * Q + 4;  // Swxx | Swxr | Scx | Sc Sx Sxx n
  static constexpr int ND = Q + 1;             // dense block: country + styles
  static constexpr int ROWB = kWT * (int)sizeof(T);            // one field row of a wave tile
  static constexpr int WSLOT = (Q + 2) * ROWB + kWT * 2;       // K1 per-wave ring slot
  __host__ __device__ static constexpr int msize(int Pseg) { return NACC + Pseg * NS; }
  // replicated segment table [Pseg][NS][R] + SEGPAD doubles per segment: without the pad every
  // segment starts at the same LDS bank (NS * R * 8 B = 0 mod 128 B), so lanes of one
  // ds_add_f64 that own the same replica pile onto 2 banks whatever their industries (8-way
  // conflicts in the 2-replicas-per-wave deterministic mode)
  static constexpr int SEGPAD = kXsSegPad;
  __host__ __device__ static constexpr int seg_stride(int R) { return NS * R + SEGPAD; }
  __host__ __device__ static constexpr int seg_doubles(int R, int Pseg) { return Pseg * seg_stride(R); }
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
template <int Q, typename T>
struct Ring {
  // Per-wave DMA rings (own __shared__ object, separate from the atomics' dynamic LDS): each
  // wave streams its own 64-stock tiles (k = wid, wid + nw, ...) with no workgroup barrier until
  // the final reduction, so the 8 waves of a CU drift and overlap HBM, VALU and LDS phases.
  static constexpr int WSLOT = Layout<Q, T>::WSLOT;
  static constexpr int NB = Stream<T>::RING;
  // >= the reduction tile [8][65] fp64 + one partial row (deterministic wg_reduce)
  static constexpr int RED = (8 * 65 + Layout<Q, T>::NACC) * 8;
  static constexpr int RINGW = NB * WSLOT > RED ? NB * WSLOT : RED;
  static constexpr int BYTES = 4 * RINGW;
};

// A/B knob (fp64 panels): the cap row, which the residual pass never re-reads (it uses the
// moments pass's validity bits), gets its own non-temporal DMA instruction so it does not take
// Infinity-Cache space from rows awaiting re-read (one extra DMA instruction per tile).
#ifndef MFA_XS_CAP_NT
#define MFA_XS_CAP_NT 0
#endif
// LDS-DMA instructions one wave issues per tile (the vmcnt unit of the ring).
template <int Q, typename T>
__device__ __forceinline__ constexpr int dma_per_tile(bool has_ind) {
  return (sizeof(T) == 4 ? (Q + 5) / 4 : (MFA_XS_CAP_NT ? 1 + (Q + 2) / 2 : (Q + 3) / 2)) +
         (has_ind ? 1 : 0);
}

// Moments of stocks [nb, ne) of date d (a chunk, or the whole date with nb = 0, ne = N; nb is
// a multiple of 64).  `ring` = Ring<Q,T>::BYTES of LDS, `dyn` = [Pseg*NS][R] replicated
// segment sums | [NACC] totals (LDS), `md` = msize(Pseg) doubles out (global memory or LDS that
// does not alias `dyn`; may alias `ring`).  Ends with a workgroup barrier.
//
// VAR & 32 = bitwise-deterministic mode (4-wave workgroups): every segment replica is owned by
// ONE wave (R/4 per wave), so its atomics land in that wave's program order, and the per-lane
// totals are reduced through per-wave partial rows summed in wave order.  The default mode
// shares replicas across waves (fewer bank conflicts) and is reproducible to rounding only.
// VAR & 1 / & 2: timing-only ablations (no segment atomics / no style-Gram FMAs).
template <int Q, int VAR, int R, typename T>
__device__ __forceinline__ void moments_body(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, int d, char* ring, double* dyn,
    double* md, int nb = 0, int ne = -1, double* __restrict__ gout = nullptr,
    unsigned long long* __restrict__ okm = nullptr) {
  using L = Layout<Q, T>;
  if (ne < 0) ne = N;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC;
  constexpr int WSLOT = Ring<Q, T>::WSLOT, RINGW = Ring<Q, T>::RINGW, NB = Ring<Q, T>::NB;
  constexpr int ROWB = L::ROWB;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nthr >> 6;
  constexpr bool DET = (VAR & 32) != 0;
  constexpr bool PLAIN = (VAR & 64) != 0;
  static_assert(!DET || (R % 4 == 0 && NACC <= 256), "deterministic mode: 4 waves, R/4 replicas each");
  const int rep = DET ? wid * (R / 4) + (lane & (R / 4 - 1)) : (lane & (R - 1));
  const unsigned seg_a = lds_addr(dyn + rep);
  constexpr int SJ = L::seg_stride(R);
  double* acc = dyn + Pseg * SJ;
  for (int i = tid; i < Pseg * SJ + NACC; i += nthr) dyn[i] = 0.0;
  __syncthreads();

  const T* Xd = X + (size_t)d * Q * N;
  const T* cd = cap + (size_t)d * N;
  const T* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;

  double v[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) v[i] = 0.0;

  char* wring = ring + wid * RINGW;
  const int nrows = dma_per_tile<Q, T>(id != nullptr);  // DMA instructions per tile
  const int ntile_all = (ne - nb + kWT - 1) / kWT;
  const int ntile = ntile_all > wid ? (ntile_all - wid + nw - 1) / nw : 0;  // this wave's tiles
  auto issue = [&](int i) {
    char* slot = wring + (i % NB) * WSLOT;
    const int s0 = nb + (wid + i * nw) * kWT;
    if constexpr (sizeof(T) == 4) {
      // four 256-B fp32 rows per instruction: lane l -> row rr + l / 16, stocks 4 (l % 16) + 0..3
      // (16-B pieces: a third of the 4-B DMA instructions for the same image)
      const int sub = lane >> 4, s = s0 + 4 * (lane & 15);
      const bool in = s < ne;  // ne is a multiple of 4: all four stocks of the piece exist
#pragma unroll
      for (int rr = 0; rr < Q + 2; rr += 4) {
        const int row = rr + sub;
        const T* src = row == 0 ? cd : (row == 1 ? rd : Xd + (size_t)(row - 2) * N);
        if (in && row < Q + 2) glds16(src + s, slot + rr * ROWB);
      }
    } else {
      // two 512-B fp64 rows per instruction: lanes 0-31 -> row rr, lanes 32-63 -> row rr + 1
      const int half = lane >> 5, s = s0 + 2 * (lane & 31);
      const bool in = s < ne;  // ne is even: both stocks of the pair exist
      constexpr int R0 = MFA_XS_CAP_NT ? 1 : 0;
      if constexpr (MFA_XS_CAP_NT) {  // cap row alone (lanes 0-31), non-temporal
        if (in && half == 0)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(cd + s), (lds_void_t*)slot, 16, 0, 2);
      }
#pragma unroll
      for (int rr = R0; rr < Q + 2; rr += 2) {
        const int row = rr + half;
        const T* src = row == 0 ? cd : (row == 1 ? rd : Xd + (size_t)(row - 2) * N);
        if (in && row < Q + 2) glds16(src + s, slot + rr * ROWB);
      }
    }
    if (id && lane < kWT / 2 && s0 + 2 * lane < ne) glds4(id + s0 + 2 * lane, slot + (Q + 2) * ROWB);
  };
  // the per-stock accumulation of one loaded tile (shared by the LDS-DMA ring and the
  // plain-load paths): s = this lane's stock, okm bits, moments FMAs, segment atomics
  auto consume = [&](int s, T cf, T rf, int j, const T (&xf)[Q]) {
      bool ok = (s < ne) && (j >= 0) && (j < Pseg) && finite_v(cf) && (cf >= T(0)) && finite_v(rf);
  #pragma unroll
      for (int q = 0; q < Q; ++q) ok = ok && finite_v(xf[q]);
      if (okm) {  // validity bits of this 64-stock tile for the residual pass (no cap re-read)
        const unsigned long long m = __ballot(ok);
        if (lane == 0) aux_store(okm + ((s - lane) >> 6), m);
      }
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
          const unsigned a = seg_a + (unsigned)(j * SJ * 8);
          const double wr = w * r;
          lds_add_nowait<0>(a, w);
          [&]<int... I>(std::integer_sequence<int, I...>) {
            (lds_add_nowait<8 * R * (1 + I)>(a, wx[I]), ...);
          }(std::make_integer_sequence<int, Q>{});
          lds_add_nowait<8 * R * (Q + 1)>(a, wr);
          lds_add_nowait<8 * R * (Q + 2)>(a, c);
        }
      }
  };
  if constexpr (PLAIN) {
    // VAR & 64: plain vector loads straight into registers (one stock per lane, each field row
    // a coalesced 64-lane load), the next tile's loads in flight while this one is consumed --
    // no LDS-DMA ring (whose per-CU issue path caps a lone workgroup near 25 GB/s)
    // VAR & 128: two tiles in flight (fp32 panels have the registers for it)
    constexpr bool DEEP = (VAR & 128) != 0;
    struct Tile {
      T c, r, x[Q];
      int j;
    };
    Tile n1{}, n2{};
    auto ldt = [&](int i, Tile& t) {
      const int s = nb + (wid + i * nw) * kWT + lane;
      const bool in = s < ne;
      t.c = in ? cd[s] : T(0);
      t.r = in ? rd[s] : T(0);
#pragma unroll
      for (int q = 0; q < Q; ++q) t.x[q] = in ? Xd[(size_t)q * N + s] : T(0);
      t.j = (in && id) ? (int)id[s] : 0;
    };
    if (ntile > 0) ldt(0, n1);
    if (DEEP && ntile > 1) ldt(1, n2);
    for (int i = 0; i < ntile; ++i) {
      const int s = nb + (wid + i * nw) * kWT + lane;
      const Tile cur = n1;
      if constexpr (DEEP) {
        n1 = n2;
        if (i + 2 < ntile) ldt(i + 2, n2);
      } else {
        if (i + 1 < ntile) ldt(i + 1, n1);
      }
      consume(s, cur.c, cur.r, cur.j, cur.x);
    }
  } else {
  for (int i = 0; i < NB - 1 && i < ntile; ++i) issue(i);
  for (int i = 0; i < ntile; ++i) {
    // The slot of tile i - 1 is free (its reads completed last iteration): refill it with tile
    // i + NB - 1 BEFORE waiting for tile i, so NB - 1 tiles stay in flight across the wait.
    if (i + NB - 1 < ntile) issue(i + NB - 1);
    const int ahead = ntile - 1 - i < NB - 1 ? ntile - 1 - i : NB - 1;  // tiles issued after i
    // + the validity-mask stores issued after tile i's DMA (iterations i-NB+1 .. i-1): vmcnt
    // counts stores too, in issue order
    const int younger = ahead * nrows + (okm ? (i < NB - 1 ? i : NB - 1) : 0);
    wait_vmcnt(__builtin_amdgcn_readfirstlane(younger));  // wave-uniform: scalar switch
    __builtin_amdgcn_wave_barrier();
    const char* slot = wring + (i % NB) * WSLOT;
    const int s = nb + (wid + i * nw) * kWT + lane;
    const unsigned la = lds_addr(slot) + lane * (unsigned)sizeof(T);
    T cf = lds_ld<0>(la, T()), rf = lds_ld<ROWB>(la, T());
    int j = id ? lds_ld_i16(lds_addr(slot) + (Q + 2) * ROWB + lane * 2) : 0;
    T xf[Q];
    [&]<int... I>(std::integer_sequence<int, I...>) {
      ((xf[I] = lds_ld<(2 + I) * ROWB>(la, T())), ...);
    }(std::make_integer_sequence<int, Q>{});
    // the wait, then empty asm that "redefines" every loaded register: no consumer of a value
    // can be scheduled between its read and the wait
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(cf), "+v"(rf), "+v"(j));
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (reg_fence(xf[I]), ...);
    }(std::make_integer_sequence<int, Q>{});
    consume(s, cf, rf, j, xf);
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (DET) {
    static_assert(RINGW >= 8 * 65 * 8 + NACC * 8, "partial row must fit the wave ring");
    wg_reduce<NACC, true>(v, (double*)wring, (double*)(wring + 8 * 65 * 8));
    __syncthreads();
    double t = 0.0;
    if (tid < NACC)
      for (int w = 0; w < nw; ++w) t += ((const double*)(ring + w * RINGW + 8 * 65 * 8))[tid];
    __syncthreads();  // md may alias the ring
    if (tid < NACC) md[tid] = t;
    if (gout && tid < NACC) aux_store(gout + tid, t);
  } else {
    wg_reduce<NACC>(v, (double*)wring, acc);
    __syncthreads();
    for (int i = tid; i < NACC; i += nthr) {
      const double t = acc[i];
      md[i] = t;
      if (gout) aux_store(gout + i, t);
    }
  }
  for (int i = tid; i < Pseg * NS; i += nthr) {
    const double* row = dyn + (i / NS) * SJ + (i % NS) * R;
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) t += row[r];
    md[NACC + i] = t;
    if (gout) aux_store(gout + NACC + i, t);
  }
  __syncthreads();
}

// Grid D * S: workgroup b handles stock chunk s = b % S ([s*C, min(N, s*C + C))) of date
// d = b / S and writes its partial moments to mom[b] (S = 1: the whole date).
template <int Q, int VAR, int R, typename T>
__global__ __launch_bounds__(256) void xs_moments_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, int S, int C, double* __restrict__ mom) {
  __shared__ __attribute__((aligned(16))) char ring[Ring<Q, T>::BYTES];
  extern __shared__ double dyn[];
  const int b = blockIdx.x, d = b / S, sc = b - d * S;
  const int nb = sc * C, ne = min(N, nb + C);
  moments_body<Q, VAR, R, T>(X, cap, ret, ind, N, Pseg, d, ring, dyn,
                             mom + (size_t)b * Layout<Q, T>::msize(Pseg), nb, ne);
}

// ------------------------------------------------------------------------------------------
// K2: structured constrained solve, one wave per date (storage-type independent).
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
  using L = Layout<Q, double>;
  return (size_t)L::msize(Pseg) + (size_t)(Q + 4) * (Q + 4) + (size_t)L::ND * (L::ND + 1) +
         (Q + 2) + Q + 2 * (((size_t)Pseg + 3) & ~(size_t)3);
}

// Constrained solve of date d by ONE wave (threadIdx.x < 64).  `sm` (LDS, solve_lds_doubles)
// holds the date's moments in [0, msize(Pseg)) on entry.  Writes f (global), the residual
// coefficients `co` [Q+1+P] (global or LDS), stats/status (global) and, if non-null, the
// status word to `st_lds`.
template <int Q, bool ROWL = false>
__device__ __forceinline__ void solve_body(double* sm, int d, int P, int Pseg, int pivot_mode,
                                           double tol, double* __restrict__ fout,
                                           double* co, double* __restrict__ stats,
                                           int* __restrict__ status, int* st_lds) {
  using L = Layout<Q, double>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, ND = L::ND;
  constexpr int NC = ND + 1;              // standardised industry row incl. the rhs
  constexpr int CH = NC + 2;              // Gram channels: m (NC) | a | 1
  constexpr int TT = (CH + 15) / 16;      // MFMA tiles per dimension
  static_assert(TT <= 2, "Q <= 28");
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

  // Cholesky of the ND x ND Schur complement, right-looking (one dependent step per column).
  // Default: in registers, redundantly in every lane (shortest chain); ROWL: row per lane with
  // readlane broadcasts (one row of registers instead of the triangle, for the low-VGPR
  // MFMA-moments kernel).  1/sqrt from v_rsq_f64 + two Newton steps.
  double b[ND];
  if constexpr (!ROWL) {
  double Lm[ND * (ND + 1) / 2], dorig[ND], il[ND];
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
  } else {
  // Cholesky of the ND x ND Schur complement, right-looking, ROW PER LANE: lane i < ND keeps
  // row i of L (ND doubles) and the pivot column is broadcast by readlane, so the register
  // footprint is one row, not the whole triangle (which set the kernel's VGPR count).  L is
  // staged in LDS (over S, already consumed) for the column-oriented back substitution.
  double Li[ND], bi = 0.0, dori = 0.0;
#pragma unroll
  for (int k = 0; k < ND; ++k) Li[k] = (lane < ND && k <= lane) ? S[lane * NC + k] : 0.0;
  if (lane < ND) {
    bi = S[lane * NC + ND];
    dori = S[lane * NC + lane];
  }
  double dmax = 0.0;
#pragma unroll
  for (int k = 0; k < ND; ++k) dmax = fmax(dmax, fabs(readlane(dori, k)));
  const double ztol = tol * dmax;
  double il[ND];
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const double dk = readlane(Li[k], k);
    const double dok = readlane(dori, k);
    if (!(dk > ztol)) {  // pinv semantics: drop the direction (exactly singular block)
      st |= (dok > ztol) ? XS_NEAR_SINGULAR : XS_ZERO_PIVOT;
      il[k] = 0.0;
      if (lane >= k) Li[k] = 0.0;
      continue;
    }
    if (dk < 1e-12 * dok) st |= XS_NEAR_SINGULAR;
    double y = __builtin_amdgcn_rsq(dk);
    y = fma(0.5 * y, fma(-dk * y, y, 1.0), y);
    y = fma(0.5 * y, fma(-dk * y, y, 1.0), y);
    il[k] = y;
    if (lane == k) Li[k] = dk * y;
    else if (lane > k) Li[k] *= y;
#pragma unroll
    for (int c = k + 1; c < ND; ++c) {
      const double lck = readlane(Li[k], c);
      if (lane >= c) Li[c] = fma(-Li[k], lck, Li[c]);
    }
  }
  // L y = b (column oriented; il = 0 zeroes dropped directions): lane i holds b_i / y_i
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const double yk = readlane(bi, k) * il[k];
    if (lane == k) bi = yk;
    else if (lane > k) bi = fma(-Li[k], yk, bi);
  }
  wave_sync_lds();
  double* Ls = S;  // [ND][ND] row-major L (S is consumed)
  if (lane < ND) {
#pragma unroll
    for (int k = 0; k < ND; ++k) Ls[lane * ND + k] = Li[k];
  }
  wave_sync_lds();
  // L^T g = y: g_k = (y_k - sum_{i>k} L[i][k] g_i) il_k ; lane i keeps its running value
#pragma unroll
  for (int k = ND - 1; k >= 0; --k) {
    const double gk = readlane(bi, k) * il[k];
    if (lane == k) bi = gk;
    else if (lane < k) bi = fma(-Ls[k * ND + lane], gk, bi);
  }
#pragma unroll
  for (int k = 0; k < ND; ++k) b[k] = readlane(bi, k);  // the solution, wave-uniform
  }

  // industries: f_j = (m_j . h - kappa a_j z) / W_j with h = [-g_D, 1]; pivot f_p = z (1 - kappa c0)
  double z = Gs[NC * CH + ND], gph = gpv[ND];
#pragma unroll
  for (int u = 0; u < ND; ++u) {
    z = fma(-Gs[NC * CH + u], b[u], z);
    gph = fma(-gpv[u], b[u], gph);
  }
  const bool bad = (st & XS_BAD) != 0;
  double* fo = fout ? fout + (size_t)d * K : nullptr;  // null: coefficients only
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
    if (fout) fo[1 + j] = bad ? qnan() : fj;
    co[Q + 1 + j] = bad ? qnan() : fj;
  }
  if (fout && lane == 0) fo[0] = bad ? qnan() : b[0];
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (lane == q) {
      if (fout) fo[1 + P + q] = bad ? qnan() : b[1 + q];
      co[q] = bad ? qnan() : b[1 + q] * isig;  // residual coefficients on RAW styles
    }
  if (lane == 0) {
    double cst = b[0];
#pragma unroll
    for (int q = 0; q < Q; ++q) cst -= b[1 + q] * isig * muv[q];
    co[Q] = bad ? qnan() : cst;
    if (status) status[d] = st;
    if (st_lds) *st_lds = st;
  }
  if (stats) {
    double* sd = stats + (size_t)d * (Q + 2);
    if (lane < Q) sd[lane] = muv[lane];
    if (lane == Q) sd[Q] = sigma;
    if (lane == Q + 1) sd[Q + 1] = nval;
  }
}

// Sum of the S partial-moment rows of date d in chunk order (deterministic) into LDS `sm`.
template <int Q>
__device__ __forceinline__ void load_moments(const double* __restrict__ mom, int d, int S,
                                             int Pseg, double* sm) {
  const int MS = Layout<Q, double>::msize(Pseg);
  const double* md = mom + (size_t)d * S * MS;
  for (int i0 = (int)threadIdx.x; i0 < MS; i0 += 4 * (int)blockDim.x) {
    double tmp[4] = {0.0, 0.0, 0.0, 0.0};  // 4 independent load chains per lane
    for (int sc = 0; sc < S; ++sc)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * (int)blockDim.x;
        if (i < MS) tmp[u] += md[(size_t)sc * MS + i];
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      if (i < MS) sm[i] = tmp[u];
    }
  }
}

template <int Q>
__global__ __launch_bounds__(64) void xs_solve_kernel(const double* __restrict__ mom, int S, int P,
                                                      int Pseg, int pivot_mode, double tol,
                                                      double* __restrict__ fout,
                                                      double* __restrict__ coef,
                                                      double* __restrict__ stats,
                                                      int* __restrict__ status) {
  extern __shared__ double sm[];
  const int d = blockIdx.x;
  load_moments<Q>(mom, d, S, Pseg, sm);
  wave_sync_lds();
  solve_body<Q>(sm, d, P, Pseg, pivot_mode, tol, fout, coef + (size_t)d * (Q + 1 + P), stats,
                status, nullptr);
}

// ------------------------------------------------------------------------------------------
// K3: specific returns and R^2.
// ------------------------------------------------------------------------------------------
// Residual-pass vector types: HIP's float4 / double2 (16-byte rows) and packed int16 ids.
// (With clang ext_vector types instead, hipcc scheduled a full vmcnt(0) drain at the top of
// every residual iteration: +30 us on the fp32 step.)
// Infinity-Cache (MALL) hygiene of the residual pass (profiles/r02_xs_nt_store_ab.md): the
// specific returns are stored non-temporally (write-once output: fp64 step 421 -> 412 us), and
// the fp64 re-read of the panel slice, the last use of those lines, is loaded non-temporally
// so it does not refresh dead lines over those other dates still have to re-read (412 ->
// 387 us).  fp32 panels: neutral for the stores, slower at small D for the loads (plain loads).
#ifndef MFA_XS_NT_E
#define MFA_XS_NT_E 1
#endif
#ifndef MFA_XS_NT_LD64
#define MFA_XS_NT_LD64 1
#endif
template <typename T> struct RVec;
template <> struct RVec<float> {
  typedef float4 vec;
  typedef uint2 ivec;
  static __device__ __forceinline__ void unpack(const vec& v, float (&a)[4]) {
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
  }
  static __device__ __forceinline__ void unpack(const ivec& v, int (&a)[4]) {
    a[0] = (int)(short)(v.x & 0xFFFF); a[1] = (int)(short)(v.x >> 16);
    a[2] = (int)(short)(v.y & 0xFFFF); a[3] = (int)(short)(v.y >> 16);
  }
  static __device__ __forceinline__ vec pack(const float (&a)[4]) {
    return make_float4(a[0], a[1], a[2], a[3]);
  }
  static __device__ __forceinline__ vec load(const float* p) { return *(const vec*)p; }
  static __device__ __forceinline__ void store(float* p, const vec& v) {
    if constexpr (MFA_XS_NT_E) {
      __builtin_nontemporal_store(v.x, p); __builtin_nontemporal_store(v.y, p + 1);
      __builtin_nontemporal_store(v.z, p + 2); __builtin_nontemporal_store(v.w, p + 3);
    } else {
      *(vec*)p = v;
    }
  }
  static __device__ __forceinline__ ivec izero() { return make_uint2(0u, 0u); }
};
template <> struct RVec<double> {
  typedef double2 vec;
  typedef unsigned ivec;
  static __device__ __forceinline__ void unpack(const vec& v, double (&a)[2]) { a[0] = v.x; a[1] = v.y; }
  static __device__ __forceinline__ void unpack(const ivec& v, int (&a)[2]) {
    a[0] = (int)(short)(v & 0xFFFF); a[1] = (int)(short)(v >> 16);
  }
  static __device__ __forceinline__ vec pack(const double (&a)[2]) { return make_double2(a[0], a[1]); }
  static __device__ __forceinline__ vec load(const double* p) {
    if constexpr (MFA_XS_NT_LD64) {
      typedef double d2 __attribute__((ext_vector_type(2)));
      const d2 t = __builtin_nontemporal_load((const d2*)p);
      return make_double2(t.x, t.y);
    } else {
      return *(const vec*)p;
    }
  }
  static __device__ __forceinline__ void store(double* p, const vec& v) {
    if constexpr (MFA_XS_NT_E) {
      __builtin_nontemporal_store(v.x, p); __builtin_nontemporal_store(v.y, p + 1);
    } else {
      *(vec*)p = v;
    }
  }
  static __device__ __forceinline__ ivec izero() { return 0u; }
};

// Residual-pass data of the last stocks, loaded by waves 1..3 while wave 0 solves (fused kernel,
// PRE): the pass then starts with 3 x 64 x VEC x kPreU stocks already in registers (1536 fp32 /
// 768 fp64 stocks).  The cap row is not loaded when the moments pass left validity bits (okm).
#ifndef MFA_XS_PREU
#define MFA_XS_PREU 2
#endif
constexpr int kPreU = MFA_XS_PREU;
template <typename T>
constexpr int pre_stocks() { return 3 * 64 * Stream<T>::VEC * kPreU; }
template <int Q, typename T>
struct ResidPre {
  typename RVec<T>::vec c4[kPreU], r4[kPreU], x4[kPreU][Q];
  typename RVec<T>::ivec j4[kPreU];
};

template <int Q, typename T>
__device__ __forceinline__ void resid_prefetch(const T* __restrict__ X, const T* __restrict__ cap,
                                               const T* __restrict__ ret,
                                               const int16_t* __restrict__ ind, int d, int N,
                                               bool need_cap, ResidPre<Q, T>& pr) {
  using RV = RVec<T>;
  constexpr int V = Stream<T>::VEC;
  const int nlo = N > pre_stocks<T>() ? N - pre_stocks<T>() : 0;
  const int t = threadIdx.x - 64;  // waves 1..3
  const T* Xd = X + (size_t)d * Q * N;
#pragma unroll
  for (int u = 0; u < kPreU; ++u) {
    const int n = nlo + t * V + u * 192 * V;
    if (n < N) {
      if (need_cap) pr.c4[u] = RV::load(cap + (size_t)d * N + n);
      pr.r4[u] = RV::load(ret + (size_t)d * N + n);
#pragma unroll
      for (int q = 0; q < Q; ++q) pr.x4[u][q] = RV::load(Xd + (size_t)q * N + n);
      pr.j4[u] = ind ? *(const typename RV::ivec*)(ind + (size_t)d * N + n) : RV::izero();
    }
  }
}

// Specific returns + R^2 of date d from the coefficients `cf_s` [Q+1+P] (LDS) by the whole
// workgroup (<= 16 waves); `red` = 16 x 5 doubles of LDS.
// PRE: waves 1..3 hold the last pre_stocks<T>() stocks in `pre` (resid_prefetch) and the main
// loop covers [0, N - pre_stocks<T>()) only.
// sums_out != nullptr: stock-sharded regression: write the 5 R^2 sums instead of R^2.
template <int Q, typename T, bool PRE = false, int UU = 0>
__device__ __forceinline__ void resid_body(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int d, int N, int P, const double* cf_s, bool bad,
    T* __restrict__ eout, double* __restrict__ r2out, double (*red)[5],
    const ResidPre<Q, T>& pre = ResidPre<Q, T>{}, double* __restrict__ sums_out = nullptr, int nb = 0,
    int ne = -1, const unsigned long long* __restrict__ okm = nullptr) {
  if (ne < 0) ne = N;
  constexpr int V = Stream<T>::VEC, U = UU > 0 ? UU : Stream<T>::U;
  using RV = RVec<T>;
  typedef typename RV::vec vec;
  typedef typename RV::ivec ivec;
  const int tid = threadIdx.x;
  const int Pseg = P > 0 ? P : 1;
  double beta[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) beta[q] = cf_s[q];
  const double cst = cf_s[Q];
  const double* fI = cf_s + Q + 1;
  const T* Xd = X + (size_t)d * Q * N;
  const T* cd = cap + (size_t)d * N;
  const T* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;
  T* ed = eout ? eout + (size_t)d * N : nullptr;
  double se = 0.0, see = 0.0, sr = 0.0, srr = 0.0, nn = 0.0;
  // V consecutive stocks per thread (16-byte loads; N % 8 == 0 keeps rows aligned) and U
  // iterations' loads issued before any is consumed: the pass is latency-bound otherwise.
  const int step = blockDim.x * V;
  // vbit: the moments pass's validity bit of the stock (okm given) or -1 (check here)
  auto one = [&](T c, T r, int j, const T (&xf)[Q], int vbit) -> T {
    bool ok;
    if (vbit >= 0) {
      ok = vbit != 0;
    } else {
      ok = (j >= 0) && (j < Pseg) && finite_v(c) && (c >= T(0)) && finite_v(r);
#pragma unroll
      for (int q = 0; q < Q; ++q) ok = ok && finite_v(xf[q]);
    }
    double e = (double)r - cst;
#pragma unroll
    for (int q = 0; q < Q; ++q) e = fma(-beta[q], (double)xf[q], e);
    T eo = (T)qnan();
    if (ok) {
      if (P > 0) e -= fI[j];
      se += e;
      see = fma(e, e, see);
      sr += (double)r;
      srr = fma((double)r, (double)r, srr);
      nn += 1.0;
      eo = (T)e;
    }
    return eo;
  };
  // okw: validity bits of the V stocks (okm given: cv is not loaded) or -1
  auto compute = [&](const vec& cv, const vec& rv, const vec (&xv)[Q], ivec jv, int okw) -> vec {
    T cs[V], rs[V], xs[Q][V], eo[V];
    int js[V];
    if (okw < 0) RV::unpack(cv, cs);
    RV::unpack(rv, rs);
    RV::unpack(jv, js);
#pragma unroll
    for (int q = 0; q < Q; ++q) RV::unpack(xv[q], xs[q]);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      T xf[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) xf[q] = xs[q][k];
      eo[k] = one(okw < 0 ? cs[k] : T(0), rs[k], js[k], xf, okw < 0 ? -1 : ((okw >> k) & 1));
    }
    return RV::pack(eo);
  };
  const unsigned long long* okd = okm;  // this date's tile masks (or null)
  auto okbits = [&](int n) -> int {
    return okd ? (int)((okd[n >> 6] >> (n & 63)) & ((1u << V) - 1)) : -1;
  };
  int Nmain = ne;
  if constexpr (PRE) {
    const int nlo = N > pre_stocks<T>() ? N - pre_stocks<T>() : 0;
    Nmain = nlo;
    if (tid >= 64) {
#pragma unroll
      for (int u = 0; u < kPreU; ++u) {
        const int n = nlo + (tid - 64) * V + u * 192 * V;
        if (n < N) {
          const vec eo = compute(pre.c4[u], pre.r4[u], pre.x4[u], pre.j4[u], okbits(n));
          if (ed) RV::store(ed + n, eo);
        }
      }
    }
  }
  // Blocks of U*step stocks walked from the END of the date: the moments pass streamed the
  // tail last, so the re-read starts with the lines most likely still in the Infinity Cache.
  // Software-pipelined: block b-1's loads are issued before block b's specific returns are
  // stored, and the store data lives in its own registers, so no iteration waits for the
  // previous one's stores to drain (register reuse of store data made hipcc insert
  // vmcnt(1..2) waits at the top of every iteration: +30 us on the fp32 step).
  const int nblk = (Nmain - nb + U * step - 1) / (U * step);
  vec cv[U], rv[U], xv[U][Q];
  ivec jv[U];
  auto load_blk = [&](int b) {
    const int n0 = nb + b * U * step + tid * V;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n0 + u * step;
      if (n < Nmain) {
        if (!okd) cv[u] = RV::load(cd + n);
        rv[u] = RV::load(rd + n);
#pragma unroll
        for (int q = 0; q < Q; ++q) xv[u][q] = RV::load(Xd + (size_t)q * N + n);
        jv[u] = id ? *(const ivec*)(id + n) : RV::izero();
      }
    }
  };
  if (nblk > 0) load_blk(nblk - 1);
  for (int b = nblk - 1; b >= 0; --b) {
    const int n0 = nb + b * U * step + tid * V;
    vec eo[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n0 + u * step;
      if (n < Nmain) eo[u] = compute(cv[u], rv[u], xv[u], jv[u], okbits(n));
    }
    if (b > 0) load_blk(b - 1);
    if (ed) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int n = n0 + u * step;
        if (n < Nmain) RV::store(ed + n, eo[u]);
      }
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
    if (sums_out) {  // chunk / stock-shard partial sums: R^2 is formed after the combine
      double* so = sums_out;
      so[0] = a; so[1] = b; so[2] = c; so[3] = e2; so[4] = n;
    } else {
      const double ve = b / n - (a / n) * (a / n);
      const double vr = e2 / n - (c / n) * (c / n);
      r2out[d] = bad ? qnan() : 1.0 - ve / vr;
    }
  }
}

// Grid D * S (dates in reverse: the MALL-resident tail of K1's stream first).  S = 1 and no
// sums_out: R^2 per date; otherwise the five R^2 sums of chunk s go to sums_out[d * S + s].
template <int Q, typename T>
__global__ __launch_bounds__(256) void xs_resid_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int D, int N, int P, int S, int C,
    const double* __restrict__ coef, const int* __restrict__ status, T* __restrict__ eout,
    double* __restrict__ r2out, double* __restrict__ sums_out = nullptr) {
  __shared__ double cf_s[Q + 1 + kXsSplitMaxP];
  __shared__ double red[16][5];
  const int b = (int)(gridDim.x - 1 - blockIdx.x), d = b / S, sc = b - d * S;
  const int nb = sc * C, ne = min(N, nb + C);
  const double* co = coef + (size_t)d * (Q + 1 + P);
  for (int i = threadIdx.x; i < Q + 1 + P; i += blockDim.x) cf_s[i] = co[i];
  __syncthreads();
  resid_body<Q, T>(X, cap, ret, ind, d, N, P, cf_s, (status[d] & XS_BAD) != 0, eout, r2out, red,
                   ResidPre<Q, T>{}, sums_out ? sums_out + (size_t)b * 5 : nullptr, nb, ne);
}

// R^2 of every date from its S chunk sums [sum e, sum e^2, sum r, sum r^2, n], in chunk order.
template <int = 0>
__global__ __launch_bounds__(256) void xs_r2_combine_kernel(const double* __restrict__ sums, int D,
                                                            int S, const int* __restrict__ status,
                                                            double* __restrict__ r2out) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  double a = 0, b = 0, c = 0, e2 = 0, n = 0;
  for (int sc = 0; sc < S; ++sc) {
    const double* p = sums + ((size_t)d * S + sc) * 5;
    a += p[0]; b += p[1]; c += p[2]; e2 += p[3]; n += p[4];
  }
  const double ve = b / n - (a / n) * (a / n);
  const double vr = e2 / n - (c / n) * (c / n);
  r2out[d] = (status[d] & XS_BAD) ? qnan() : 1.0 - ve / vr;
}

#if MFA_AB
#include "ab/xs_mfma_moments.h"
#endif

// ------------------------------------------------------------------------------------------
// Fused K1 -> K2 -> K3: one 4-wave workgroup per date streams the date's panel slice once
// from HBM (moments), solves it in wave 0, then re-reads the slice for the residual pass.
// Two workgroups fit per CU, so ~512 dates are in flight: the re-read is served mostly by the
// 256 MB Infinity Cache instead of HBM, and the single-wave solve of one date overlaps the
// other workgroup's streaming.
// ------------------------------------------------------------------------------------------
template <int Q, typename T>
constexpr int fused_ring_bytes() {
  constexpr int a = Ring<Q, T>::BYTES;
  constexpr int b = (int)(solve_lds_doubles<Q>(128) * 8);
  return a > b ? a : b;
}

template <int Q, int R, int VAR, bool PRE, typename T>
#ifndef MFA_XS_WPE_BIGQ
#define MFA_XS_WPE_BIGQ 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(Q <= 10 ? 2 : MFA_XS_WPE_BIGQ, Q <= 10 ? 2 : MFA_XS_WPE_BIGQ))) void xs_fused_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int P, int Pseg, int pivot_mode, double tol,
    double* __restrict__ fout, T* __restrict__ eout, double* __restrict__ r2out,
    double* __restrict__ stats, int* __restrict__ status, double* __restrict__ mom_out,
    unsigned long long* __restrict__ okm) {
  __shared__ __attribute__((aligned(16))) char ring[fused_ring_bytes<Q, T>()];
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red[4][5];
  __shared__ int st_s;
  extern __shared__ double dyn[];
  const int d = blockIdx.x;
  double* sm = (double*)ring;  // moments, then the solve's scratch (ring is idle by then)
  // per-tile validity bits written by the moments pass and read by the residual pass of the same
  // workgroup: the residual re-read skips the cap row (8 of 98 bytes per fp64 stock)
  unsigned long long* okd = okm + (size_t)d * ((N + kWT - 1) / kWT);
  // every date's moments also go to mom_out (from registers, ~9.7 MB per 2520 dates): the
  // device pseudo-inverse pass reads them for near-singular dates.  (Exporting only flagged
  // dates from LDS after the solve cost ~30 us per 2520-date step: the extra LDS read of the
  // DMA ring region made hipcc add conservative vmcnt drains.)
  moments_body<Q, VAR & 227, R, T>(X, cap, ret, ind, N, Pseg, d, ring, dyn, sm, 0, -1,
                                  mom_out ? mom_out + (size_t)d * Layout<Q, T>::msize(Pseg)
                                          : nullptr,
                                  okd);
  if constexpr ((VAR & 8) != 0) {  // timing-only ablation: no solve
    for (int i = threadIdx.x; i < Q + 1 + P; i += blockDim.x) cf_s[i] = sm[i] * 1e-30;
    if (threadIdx.x == 0) st_s = 0;
  } else if (threadIdx.x < 64) {
    solve_body<Q>(sm, d, P, Pseg, pivot_mode, tol, fout, cf_s, stats, status, &st_s);
  }
  ResidPre<Q, T> pre;
  if constexpr (PRE) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0)
      resid_prefetch<Q, T>(X, cap, ret, ind, d, N, okd == nullptr, pre);
  }
  __syncthreads();
  if constexpr ((VAR & 4) == 0)
    resid_body<Q, T, PRE>(X, cap, ret, ind, d, N, P, cf_s, (st_s & XS_BAD) != 0, eout, r2out,
                          red, pre, nullptr, 0, -1, okd);
  if constexpr ((VAR & 16) != 0) {  // timing-only: a second residual pass (cache-hit cost)
    __syncthreads();
    resid_body<Q, T>(X, cap, ret, ind, d, N, P, cf_s, (st_s & XS_BAD) != 0, eout, r2out, red);
  }
}

#if MFA_AB
#include "ab/xs_resident.h"
#endif

constexpr int XS_COOP_TIMEOUT = 64;  // status bit: a team wait gave up (results invalid)
constexpr int kCoopSpin = 1 << 21;   // poll iterations (s_sleep 4 each, ~0.2 s) before giving up
constexpr int kCoopMaxC = 16;        // chunks per date at most
constexpr int kPipeGroups = 8;       // ticket groups: blockIdx & 7 (the blocks sharing an XCD)
constexpr int kPipeMaxLag = 3;       // residual pass at most 3 tickets behind the moments
constexpr int kReadyBit = 1 << 30;   // ready flag = status | kReadyBit

#if MFA_AB
#include "ab/xs_team.h"
#endif

// ------------------------------------------------------------------------------------------
// Device pseudo-inverse refinement (pinv semantics of CrossSection.py:76,98) for dates the
// Cholesky flagged near-singular (e.g. an exactly collinear style pair).  Grid D; a workgroup
// whose date is not flagged exits at once, so the pass rides in the same stream / HIP graph as
// the regression with no host synchronisation.  A flagged date rebuilds the reference's
// constrained normal matrix A = R^T X^T W X R (Kr x Kr, Kr = K - 1 with industries) and rhs
// from its exported raw moments, eigen-decomposes A with the one-wave Jacobi (jacobi.h), and
// applies pinv(A) = V diag(1/lambda) V^T over |lambda| > 1e-15 max|lambda| (numpy's pinv rcond
// on the singular values |lambda|).  f = R g, then the whole workgroup redoes the date's
// specific returns and R^2.
// ------------------------------------------------------------------------------------------
constexpr int kXsRefineMaxK = 64;   // full-matrix Jacobi pinv up to here; structured above

template <int Q>
__host__ __device__ constexpr size_t refine_lds_doubles(int P) {
  const int Pseg = P > 0 ? P : 1;
  const int K = 1 + P + Q, Kr = P > 0 ? K - 1 : K;
  return (size_t)Layout<Q, double>::msize(Pseg) + 2 * (size_t)Kr * (Kr + 1) + 4 * 64 +
         4 * (size_t)Kr + (Q + 4);
}

// ------------------------------------------------------------------------------------------
// Structured pseudo-inverse for ANY K (industries up to 128): pinv semantics of
// CrossSection.py:76,98 without forming the Kr x Kr matrix.  After the constraint the normal
// matrix is M = [[A_I, B], [B^T, C]] with the industry block A_I = diag(W) + rho a a^T over the
// active non-pivot industries (positive definite; exactly-empty industries are zero rows/cols
// and get f = 0, as pinv gives them), B[j][u] = m_j[u] and the dense block C over
// [country | z-styles] (ND = Q + 1 columns).  The normal equations are consistent (rhs in
// range(M)), so every near-null direction of M lies in the dense block's Schur complement S:
//   null(M) = { [-A_I^{-1} B n ; n] : n in null(S) }.
// The wave eigen-decomposes S (ND x ND, Jacobi), keeps eigenpair (mu_k, v_k) unless its
// Rayleigh quotient on M, mu_k / (1 + |A_I^{-1} B v_k|^2), is <= 1e-15 lambda_max(M) (numpy's
// pinv rcond; lambda_max by power iteration on the structured M), solves the kept part
// (x2 = sum v v^T b~ / mu, x1 = A_I^{-1}(b1 - B x2)) and projects the result orthogonally to
// the cut null directions: the minimum-norm solution pinv(M) b.  O(P ND^2) work in one wave.
// ------------------------------------------------------------------------------------------
template <int Q>
__host__ __device__ constexpr size_t refine_struct_lds_doubles(int P) {
  constexpr int ND = Q + 1, NC = ND + 1;
  const int Pseg = P > 0 ? P : 1;
  const int P4 = (Pseg + 63) & ~63;
  return (size_t)Layout<Q, double>::msize(Pseg) + (size_t)P4 * NC   // moments | m_j rows
         + 3 * (size_t)P4                                           // a_j/W_j, 1/W_j, x1 / tmp
         + (size_t)ND * P4                                          // z1_k of cut directions
         + 2 * (size_t)ND * (ND + 1) + (size_t)ND * NC              // S (Jacobi), V, S | rhs
         + 4 * 64 + 4 * (size_t)NC + 2 * (size_t)ND * ND + 64;      // rot, vectors, H, misc
}

// One wave (threadIdx.x < 64).  `md` = the date's raw moments (LDS), `ws` = scratch after them
// (refine_struct_lds_doubles - msize doubles).  Writes f (global row fo, K entries), the
// residual coefficients co[Q+1+P] (LDS or global) and returns the status bits to OR in.
template <int Q>
__device__ int struct_pinv_wave(const double* md, double* ws, int P, int pivot_mode,
                                double* __restrict__ fo, double* co) {
  using L = Layout<Q, double>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, ND = L::ND, NC = ND + 1;
  const int lane = threadIdx.x & 63;
  const int Pseg = P > 0 ? P : 1;
  const int P4 = (Pseg + 63) & ~63;
  const double* acc = md;
  const double* seg = md + NACC;
  double* mrow = ws;                 // [P4][NC]  m_j (0 for inactive)
  double* aw = mrow + P4 * NC;       // [P4]      a_j / W_j
  double* iw = aw + P4;              // [P4]      1 / W_j (0 = inactive)
  double* x1 = iw + P4;              // [P4]      industry unknowns / scratch
  double* z1 = x1 + P4;              // [ND][P4]  -A_I^{-1} B v_k
  double* Aj = z1 + ND * P4;         // [ND][ND+1] Jacobi matrix -> eigenvalues
  double* Vj = Aj + ND * (ND + 1);   // [ND][ND+1] eigenvectors (columns)
  double* Sx = Vj + ND * (ND + 1);   // [ND][NC]   Schur complement | reduced rhs
  double* rot = Sx + ND * NC;        // [4*64]
  double* gp = rot + 4 * 64;         // [NC] standardised pivot row
  double* at = gp + NC;              // [NC] sum a m / W
  double* totv = at + NC;            // [NC] column totals
  double* x2 = totv + NC;            // [NC] dense unknowns
  double* H = x2 + NC;               // [ND][ND] Gram of the cut null directions
  double* vk = H + ND * ND;          // [ND][ND] scratch
  double* misc = vk + ND * ND;       // [64]

  const double Sc = acc[NG + 2 * Q + 0];
  const double nval = acc[NG + 2 * Q + 3];
  const double nq = nval * Q;
  const double mx = acc[NG + 2 * Q + 1] / nq;
  const double sigma = sqrt(fmax(acc[NG + 2 * Q + 2] / nq - mx * mx, 0.0));
  const double isig = 1.0 / sigma;
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
  }
  const int rp = P > 0 ? jp : 0;
  const double sp = P > 0 ? seg[rp * NS + Q + 2] : 1.0;
  const double rho = P > 0 ? seg[rp * NS] : 0.0;
  auto muq = [&](int q) { return acc[NG + Q + q] / Sc; };
  auto stdz = [&](const double* row, int c) {  // standardised industry channel c of `row`
    const double raw = row[c];
    return (c >= 1 && c <= Q) ? (raw - muq(c - 1) * row[0]) * isig : raw;
  };
  if (lane < NC) gp[lane] = P > 0 ? stdz(seg + rp * NS, lane) : 0.0;
  for (int j = lane; j < P4; j += 64) {
    const double W = j < P ? seg[j * NS] : 0.0;
    const bool act = (j < P) && (j != jp) && (W > 0.0);
    const double a = act ? -seg[j * NS + Q + 2] / sp : 0.0;
    iw[j] = act ? 1.0 / W : 0.0;
    aw[j] = act ? a / W : 0.0;
    x1[j] = a;  // a_j, consumed below
  }
  wsync();
  for (int e = lane; e < P4 * NC; e += 64) {
    const int j = e / NC, c = e - (e / NC) * NC;
    mrow[e] = iw[j] != 0.0 ? stdz(seg + j * NS, c) + x1[j] * gp[c] : 0.0;
  }
  // c0 = sum a^2 / W, sa = sum a (active)
  double c0 = 0.0, sa = 0.0;
  for (int j = lane; j < P4; j += 64) { c0 = fma(x1[j], aw[j], c0); sa += x1[j]; }
  c0 = wave_total(c0);
  sa = wave_total(sa);
  const double kappa = P > 0 ? rho / (1.0 + rho * c0) : 0.0;
  wsync();
  // column totals and at
  if (lane < NC) {
    double t = 0.0, u = 0.0;
    for (int j = 0; j < P4; ++j) { t += mrow[j * NC + lane]; u = fma(aw[j], mrow[j * NC + lane], u); }
    // P == 0: the single segment holds the totals
    totv[lane] = P > 0 ? t + (1.0 - sa) * gp[lane] : stdz(seg, lane);
    at[lane] = u;
  }
  wsync();
  const double Sw = totv[0];
  // S = C - B^T A_I^{-1} B (+ rhs column) = M_DD - G + kappa at at^T
  for (int e = lane; e < ND * NC; e += 64) {
    const int u = e / NC, w = e - (e / NC) * NC;
    double m;
    if (u == 0) m = totv[w];
    else if (w == 0) m = totv[u];
    else if (w == ND) m = acc[NG + u - 1] * isig - muq(u - 1) * isig * totv[ND];
    else {
      const int q = u - 1, s2 = w - 1;
      const int hi = q > s2 ? q : s2, lo = q > s2 ? s2 : q;
      m = (acc[hi * (hi + 1) / 2 + lo] - muq(q) * muq(s2) * Sw) * isig * isig -
          (muq(q) * totv[w] + muq(s2) * totv[u]) * isig;
    }
    double g = 0.0;
    for (int j = 0; j < P4; ++j) g = fma(mrow[j * NC + u] * iw[j], mrow[j * NC + w], g);
    Sx[e] = m - g + kappa * at[u] * at[w];
    if (w < ND) H[u * ND + w] = m;  // the dense block C itself, for the power iteration
  }
  wsync();
  for (int e = lane; e < ND * ND; e += 64) {
    const int u = e / ND, w = e - (e / ND) * ND;
    Aj[u * (ND + 1) + w] = Sx[u * NC + w];
  }
  wsync();
  jacobi_wave(Aj, Vj, ND, ND + 1, rot, 60, 1e-17);

  // A_I^{-1} y = y / W - kappa (a/W) ((a/W)^T y), in place on a [P4] LDS vector
  auto ainv = [&](double* y) {
    double t = 0.0;
    for (int j = lane; j < P4; j += 64) t = fma(aw[j], y[j], t);
    t = wave_total(t);
    wsync();
    for (int j = lane; j < P4; j += 64) y[j] = y[j] * iw[j] - kappa * aw[j] * t;
    wsync();
  };
  // lambda_max(M) by power iteration on [x1; x2] (x1 in z1 row 0 as scratch, x2 in misc)
  double* p1 = z1;  // reused: the cut directions are formed after this
  for (int j = lane; j < P4; j += 64) p1[j] = iw[j] != 0.0 ? 1.0 : 0.0;
  if (lane < ND) misc[lane] = 1.0;
  wsync();
  double lmax = 0.0;
  for (int it = 0; it < 60; ++it) {
    // y1 = W x1 + rho a (a^T x1) + B x2 ; y2 = B^T x1 + C x2  (C = M_DD = S + G - kappa at at^T)
    double ax = 0.0;
    for (int j = lane; j < P4; j += 64) ax = fma(aw[j] * (iw[j] != 0.0 ? 1.0 / iw[j] : 0.0), p1[j], ax);
    ax = wave_total(ax);
    double y1[2] = {0.0, 0.0};
    for (int jj = 0; jj < 2; ++jj) {
      const int j = lane + 64 * jj;
      if (j < P4 && iw[j] != 0.0) {
        const double W = 1.0 / iw[j], a = aw[j] * W;
        double t = W * p1[j] + rho * a * ax;
        for (int u = 0; u < ND; ++u) t = fma(mrow[j * NC + u], misc[u], t);
        y1[jj] = t;
      }
    }
    double y2 = 0.0;
    if (lane < ND) {
      const int u = lane;
      for (int j = 0; j < P4; ++j) y2 = fma(mrow[j * NC + u], p1[j], y2);
      for (int w = 0; w < ND; ++w) y2 = fma(H[u * ND + w], misc[w], y2);
    }
    double nn = y1[0] * y1[0] + y1[1] * y1[1] + (lane < ND ? y2 * y2 : 0.0);
    nn = wave_total(nn);
    const double nrm = sqrt(nn);
    lmax = nrm;  // |M x| with |x| = 1 after the first step
    const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
    wsync();
    for (int jj = 0; jj < 2; ++jj) {
      const int j = lane + 64 * jj;
      if (j < P4) p1[j] = y1[jj] * inv;
    }
    if (lane < ND) misc[lane] = y2 * inv;
    wsync();
  }
  const double cut = 1e-15 * lmax;
  // eigenpairs of S: z1_k = -A_I^{-1} B v_k, Rayleigh quotient on M, keep / cut
  int ncut = 0;
  unsigned keep_mask = 0;
  for (int k = 0; k < ND; ++k) {
    double* zk = z1 + ncut * P4;
    for (int j = lane; j < P4; j += 64) {
      double t = 0.0;
      for (int u = 0; u < ND; ++u) t = fma(mrow[j * NC + u], Vj[u * (ND + 1) + k], t);
      zk[j] = -t;
    }
    wsync();
    ainv(zk);
    double zz = 0.0;
    for (int j = lane; j < P4; j += 64) zz = fma(zk[j], zk[j], zz);
    zz = wave_total(zz);
    const double muk = Aj[k * (ND + 1) + k];
    if (fabs(muk) / (1.0 + zz) > cut) {
      keep_mask |= 1u << k;
    } else {
      if (lane < ND) vk[ncut * ND + lane] = Vj[lane * (ND + 1) + k];
      ++ncut;  // zk stays: a cut direction
    }
    wsync();
  }
  // x2 = sum_kept v v^T b~ / mu
  if (lane < ND) {
    double t = 0.0;
    for (int k = 0; k < ND; ++k) {
      if (!(keep_mask & (1u << k))) continue;
      double vb = 0.0;
      for (int u = 0; u < ND; ++u) vb = fma(Vj[u * (ND + 1) + k], Sx[u * NC + ND], vb);
      t = fma(Vj[lane * (ND + 1) + k], vb / Aj[k * (ND + 1) + k], t);
    }
    x2[lane] = t;
  }
  wsync();
  // x1 = A_I^{-1} (b1 - B x2),  b1_j = m_j[ND]
  for (int j = lane; j < P4; j += 64) {
    double t = mrow[j * NC + ND];
    for (int u = 0; u < ND; ++u) t = fma(-mrow[j * NC + u], x2[u], t);
    x1[j] = iw[j] != 0.0 ? t : 0.0;
  }
  wsync();
  ainv(x1);
  // minimum norm: x -= Z (Z^T Z)^{-1} Z^T x over the cut directions Z_k = [z1_k ; v_k]
  if (ncut > 0) {
    for (int e = 0; e < ncut * ncut; ++e) {
      const int k = e / ncut, l = e - (e / ncut) * ncut;
      double t = 0.0;
      for (int j = lane; j < P4; j += 64) t = fma(z1[k * P4 + j], z1[l * P4 + j], t);
      t = wave_total(t);
      double vv = 0.0;
      for (int u = 0; u < ND; ++u) vv = fma(vk[k * ND + u], vk[l * ND + u], vv);
      if (lane == 0) H[k * ND + l] = t + vv;
    }
    for (int k = 0; k < ncut; ++k) {
      double t = 0.0;
      for (int j = lane; j < P4; j += 64) t = fma(z1[k * P4 + j], x1[j], t);
      t = wave_total(t);
      double vx = 0.0;
      for (int u = 0; u < ND; ++u) vx = fma(vk[k * ND + u], x2[u], vx);
      if (lane == 0) misc[k] = t + vx;
    }
    wsync();
    if (lane == 0) {  // Cholesky solve of the ncut x ncut SPD Gram (ncut <= 17)
      for (int k = 0; k < ncut; ++k) {
        double dk = H[k * ND + k];
        for (int i = 0; i < k; ++i) dk -= H[k * ND + i] * H[k * ND + i];
        dk = sqrt(fmax(dk, 1e-300));
        H[k * ND + k] = dk;
        for (int i = k + 1; i < ncut; ++i) {
          double t = H[i * ND + k];
          for (int l = 0; l < k; ++l) t -= H[i * ND + l] * H[k * ND + l];
          H[i * ND + k] = t / dk;
        }
      }
      for (int k = 0; k < ncut; ++k) {
        double t = misc[k];
        for (int l = 0; l < k; ++l) t -= H[k * ND + l] * misc[l];
        misc[k] = t / H[k * ND + k];
      }
      for (int k = ncut - 1; k >= 0; --k) {
        double t = misc[k];
        for (int l = k + 1; l < ncut; ++l) t -= H[l * ND + k] * misc[l];
        misc[k] = t / H[k * ND + k];
      }
    }
    wsync();
    for (int j = lane; j < P4; j += 64) {
      double t = x1[j];
      for (int k = 0; k < ncut; ++k) t = fma(-misc[k], z1[k * P4 + j], t);
      x1[j] = t;
    }
    if (lane < ND) {
      double t = x2[lane];
      for (int k = 0; k < ncut; ++k) t = fma(-misc[k], vk[k * ND + lane], t);
      x2[lane] = t;
    }
    wsync();
  }
  // outputs: f in the original order, residual coefficients on RAW styles
  double fpv = 0.0;
  for (int j = lane; j < P4; j += 64) fpv = fma(aw[j] * (iw[j] != 0.0 ? 1.0 / iw[j] : 0.0), x1[j], fpv);
  fpv = wave_total(fpv);
  for (int j = lane; j < P; j += 64) {
    const double fj = j == jp ? fpv : x1[j];
    fo[1 + j] = fj;
    co[Q + 1 + j] = fj;
  }
  if (lane == 0) fo[0] = x2[0];
  if (lane < Q) {
    fo[1 + P + lane] = x2[1 + lane];
    co[lane] = x2[1 + lane] * isig;
  }
  if (lane == 0) {
    double cst = x2[0];
    for (int q = 0; q < Q; ++q) cst -= x2[1 + q] * isig * muq(q);
    co[Q] = cst;
  }
  wsync();
  return ncut > 0 ? XS_REFINED | XS_PINV_CUT : XS_REFINED;
}

// Full-matrix Jacobi pinv of the constrained normal matrix, K <= kXsRefineMaxK (the reference's
// own algebra: eigen-decompose A = R^T X^T W X R, drop |lambda| <= 1e-15 max|lambda|).  The
// whole workgroup builds A in LDS, wave 0 solves.  Writes f (row fo), co[Q+1+P] and returns
// the status bits to OR in (threadIdx.x < 64).
template <int Q>
__device__ int jacobi_pinv_block(const double* md, double* ws, int P, int pivot_mode,
                                 double* __restrict__ fo, double* co, double* sc, int* piv_s) {
  using L = Layout<Q, double>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int Pseg = P > 0 ? P : 1;
  const int K = 1 + P + Q, Kr = P > 0 ? K - 1 : K, lda = Kr + 1;
  double* A = ws;                  // [Kr][lda]
  double* V = A + Kr * lda;        // [Kr][lda]
  double* rot = V + Kr * lda;      // [4*64]
  double* rhs = rot + 4 * 64;      // [Kr]
  double* alp = rhs + Kr;          // [Kr]  constraint weights alpha_u
  double* g = alp + Kr;            // [Kr]  eigen-space coefficients
  double* mu = g + Kr;             // [Q]   cap-weighted style means
  const double* acc = md;
  const double* seg = md + NACC;
  if (tid == 0) {
    double Wt = 0.0, Bt = 0.0;
    for (int j = 0; j < Pseg; ++j) { Wt += seg[j * NS]; Bt += seg[j * NS + Q + 1]; }
    const double nq = acc[NG + 2 * Q + 3] * Q;
    const double mx = acc[NG + 2 * Q + 1] / nq;
    sc[0] = Wt; sc[1] = Bt;
    sc[2] = sqrt(fmax(acc[NG + 2 * Q + 2] / nq - mx * mx, 0.0));
    int jp = -1;
    if (P > 0) {
      if (pivot_mode == 1) jp = P - 1;
      else for (int j = 0; j < P; ++j) if (seg[j * NS + Q + 2] > 0.0) jp = j;
      if (jp < 0) jp = P - 1;
    }
    *piv_s = jp;
    sc[3] = P > 0 ? seg[jp * NS + Q + 2] : 1.0;
  }
  if (tid < Q) mu[tid] = acc[NG + Q + tid] / acc[NG + 2 * Q];
  __syncthreads();
  const double Wt = sc[0], Bt = sc[1], sig = sc[2], isig = 1.0 / sig, sp = sc[3];
  const int jp = *piv_s;
  // Aq_tot[q] = sum_j A_jq
  auto aqt = [&](int q) {
    double t = 0.0;
    for (int j = 0; j < Pseg; ++j) t += seg[j * NS + 1 + q];
    return t;
  };
  // entries of the full X^T W X over the ORIGINAL columns [country | industries | z-styles]
  auto mfull = [&](int i, int j) -> double {
    if (i > j) { const int t = i; i = j; j = t; }
    const int s0 = 1 + P;
    if (j < s0) {  // country / industry block
      if (i == 0) return j == 0 ? Wt : seg[(j - 1) * NS];
      return i == j ? seg[(i - 1) * NS] : 0.0;
    }
    const int qj = j - s0;
    if (i == 0) return (aqt(qj) - mu[qj] * Wt) * isig;
    if (i < s0) return (seg[(i - 1) * NS + 1 + qj] - mu[qj] * seg[(i - 1) * NS]) * isig;
    const int qi = i - s0;
    const int hi = qi > qj ? qi : qj, lo = qi > qj ? qj : qi;
    return (acc[hi * (hi + 1) / 2 + lo] - mu[qi] * aqt(qj) - mu[qj] * aqt(qi) +
            mu[qi] * mu[qj] * Wt) * isig * isig;
  };
  auto bfull = [&](int i) -> double {
    const int s0 = 1 + P;
    if (i == 0) return Bt;
    if (i < s0) return seg[(i - 1) * NS + Q + 1];
    const int q = i - s0;
    return (acc[NG + q] - mu[q] * Bt) * isig;
  };
  const int pc = 1 + jp;  // pivot column (P > 0)
  auto orig = [&](int u) { return (P > 0 && u >= pc) ? u + 1 : u; };
  for (int u = tid; u < Kr; u += blockDim.x) {
    const int ou = orig(u);
    alp[u] = (P > 0 && ou >= 1 && ou <= P) ? -seg[(ou - 1) * NS + Q + 2] / sp : 0.0;
  }
  __syncthreads();
  for (int e = tid; e < Kr * Kr; e += blockDim.x) {
    const int u = e / Kr, v = e % Kr;
    if (v < u) continue;
    const int ou = orig(u), ov = orig(v);
    double a = mfull(ou, ov);
    if (P > 0) {
      const double au = alp[u], av = alp[v];
      a += au * mfull(pc, ov) + av * mfull(ou, pc) + au * av * mfull(pc, pc);
    }
    A[u * lda + v] = a;
    A[v * lda + u] = a;
  }
  for (int u = tid; u < Kr; u += blockDim.x)
    rhs[u] = bfull(orig(u)) + (P > 0 ? alp[u] * bfull(pc) : 0.0);
  __syncthreads();
  if (tid >= 64) return 0;
  jacobi_wave(A, V, Kr, lda, rot, 40, 1e-17);
  double lmax = 0.0;
  for (int k = lane; k < Kr; k += 64) lmax = fmax(lmax, fabs(A[k * lda + k]));
  lmax = wave_max(lmax);
  const double cut = 1e-15 * lmax;
  // c_k = (v_k . rhs) / lambda_k over the kept spectrum
  double ncut = 0.0;
  for (int k = lane; k < Kr; k += 64) {
    const double lk = A[k * lda + k];
    double t = 0.0;
    for (int i = 0; i < Kr; ++i) t = fma(V[i * lda + k], rhs[i], t);
    g[k] = fabs(lk) > cut ? t / lk : 0.0;
    ncut += fabs(lk) > cut ? 0.0 : 1.0;
  }
  ncut = wave_sum(ncut);
  wsync();
  for (int i = lane; i < Kr; i += 64) {  // g <- V c
    double t = 0.0;
    for (int k = 0; k < Kr; ++k) t = fma(V[i * lda + k], g[k], t);
    rot[i < 256 ? i : 0] = t;  // rot is free again: stage V c (Kr <= 64)
  }
  wsync();
  // f in original order: f[orig(u)] = g[u], f[pivot] = sum_u alpha_u g[u]
  double fp = 0.0;
  for (int u = lane; u < Kr; u += 64) fp = fma(alp[u], rot[u], fp);
  fp = wave_sum(fp);
  for (int u = lane; u < Kr; u += 64) {
    const int ou = orig(u);
    fo[ou] = rot[u];
    if (ou >= 1 && ou <= P) co[Q + ou] = rot[u];          // industry f_j at Q + 1 + j
    if (ou > P) co[ou - 1 - P] = rot[u] * isig;           // raw-style coefficient
  }
  if (P > 0 && lane == 0) { fo[pc] = fp; co[Q + pc] = fp; }
  wsync();
  if (lane == 0) {
    double cst = rot[0];  // country (column 0 is never the pivot)
    for (int q = 0; q < Q; ++q) cst -= co[q] * mu[q];
    co[Q] = cst;
  }
  wsync();
  // same status semantics as the structured pinv (K > 64): PINV_CUT iff a direction was cut
  return ncut > 0.0 ? XS_REFINED | XS_PINV_CUT : XS_REFINED;
}

template <int Q>
__host__ __device__ constexpr size_t refine_any_lds_doubles(int P) {
  return 1 + Q + P > kXsRefineMaxK ? refine_struct_lds_doubles<Q>(P) : refine_lds_doubles<Q>(P);
}

// ------------------------------------------------------------------------------------------
// Device pseudo-inverse refinement (pinv semantics of CrossSection.py:76,98) for dates the
// Cholesky flagged near-singular (e.g. an exactly collinear style pair).  Grid D; a workgroup
// whose date is not flagged exits at once, so the pass rides in the same stream / HIP graph as
// the regression with no host synchronisation.  K <= 64: the reference's own algebra (the
// constrained normal matrix A = R^T X^T W X R in LDS, one-wave Jacobi, pinv(A) = V diag(1 /
// lambda) V^T over |lambda| > 1e-15 max|lambda|); larger K (SW-L2-sized industry sets): the
// structured pinv above.  RESID: the whole workgroup then redoes the date's specific returns
// and R^2; otherwise (stock-sharded path) only f and the residual coefficients coef[d] are
// rewritten, for the caller's residual pass.
// ------------------------------------------------------------------------------------------
template <int Q, typename T, bool RESID>
__global__ __launch_bounds__(256) void xs_refine_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int P, int pivot_mode, int S,
    const double* __restrict__ mom, double* __restrict__ fout, T* __restrict__ eout,
    double* __restrict__ r2out, int* __restrict__ status, double* __restrict__ coef) {
  using L = Layout<Q, double>;
  const int d = blockIdx.x;
  const int st0 = status[d];
  if (!(st0 & XS_NEAR_SINGULAR) || (st0 & XS_BAD)) return;  // uniform: whole workgroup exits
  extern __shared__ double sm[];
  __shared__ double cf_s[Q + 1 + kXsSplitMaxP];
  __shared__ double red[4][5];
  __shared__ double sc[4];   // W_tot, B_tot, sigma, s_pivot
  __shared__ int piv_s;
  __shared__ int st_s;
  const int tid = threadIdx.x;
  const int Pseg = P > 0 ? P : 1;
  const int MS = L::msize(Pseg);
  const int K = 1 + P + Q;
  double* md = sm;                 // [MS] raw moments
  load_moments<Q>(mom, d, S, Pseg, md);
  __syncthreads();
  double* fo = fout ? fout + (size_t)d * K : nullptr;  // null: coefficients only
  double* co = RESID ? cf_s : coef + (size_t)d * (Q + 1 + P);
  int bits;
  if (K > kXsRefineMaxK) {
    bits = tid < 64 ? struct_pinv_wave<Q>(md, md + MS, P, pivot_mode, fo, co) : 0;
  } else {
    bits = jacobi_pinv_block<Q>(md, md + MS, P, pivot_mode, fo, co, sc, &piv_s);
  }
  if (tid == 0) {
    st_s = st0 | bits;
    status[d] = st0 | bits;
  }
  if constexpr (RESID) {
    __syncthreads();
    resid_body<Q, T>(X, cap, ret, ind, d, N, P, cf_s, false, eout, r2out, red);
  }
}

constexpr int kXsDeterministic = 0x100;  // pivot_mode flag: bitwise-deterministic kernel
constexpr int kXsRefine = 0x200;         // pivot_mode flag: device pinv pass for flagged dates

template <int Q, typename T>
size_t solve_lds_bytes(int Pseg) {
  return solve_lds_doubles<Q>(Pseg) * sizeof(double);
}

// ------------------------------------------------------------------------------------------
// Path selection.  Default: the fused kernel, one workgroup per date, ~512 dates in flight.
// Chunked path (mfa_xs_set_chunks(S > 0), or automatic below kXsChunkMinD dates): each date is
// cut into S stock chunks of C stocks, for shards too small to fill the chip:
//   moments (D*S WGs, partial moments) -> solve (D waves, partials summed in chunk order)
//   -> residuals (D*S WGs, partial R^2 sums) -> R^2 combine (chunk order).
// Chunk sums are combined in a fixed order, so the chunked path is as deterministic as the
// per-workgroup reductions it is built from.
// ------------------------------------------------------------------------------------------
constexpr int kXsChunkMinD = 0;      // automatic chunking off: measured slower than the fused
                                     // kernel at every D in 315..2520 (profiles/r02_xs_paths.md)
constexpr int kXsChunkTargetWG = 2048;
constexpr int kXsMinChunk = 256;     // stocks

inline int xs_chunk_size(int N, int S) { return ((N + S - 1) / S + kWT - 1) / kWT * kWT; }

inline int xs_chunks(int D, int N) {
  const int maxS = N / kXsMinChunk > 1 ? N / kXsMinChunk : 1;
  int S;
  if (g_mfa_xs_chunks > 0) S = g_mfa_xs_chunks;
  else if (g_mfa_xs_chunks < 0 || D >= kXsChunkMinD) S = 1;
  else S = (kXsChunkTargetWG + D - 1) / D;
  S = S < 1 ? 1 : (S > maxS ? maxS : S);
  const int C = xs_chunk_size(N, S);
  return (N + C - 1) / C;  // no empty trailing chunk after rounding C up to 64
}

// Team (pipelined) path: chunks per date (g_mfa_xs_coop: 0 = off, > 0 = forced, < 0 = auto).
// Auto: enough chunks for ~kCoopTargetChunks chunks, at least kCoopMinChunk stocks per chunk.
constexpr int kCoopTargetChunks = 8192;
constexpr int kCoopMinChunk = 512;
inline int xs_coop_chunks(int D, int N) {
  const int g = g_mfa_xs_coop;
  if (g == 0 || g_mfa_xs_mode != 0) return 1;
  int C = g > 0 ? g : (kCoopTargetChunks + D - 1) / D;
  const int minChunk = g > 0 ? kWT : kCoopMinChunk;  // forced counts: one tile per chunk at least
  const int maxC = N / minChunk > 1 ? N / minChunk : 1;
  C = C < 1 ? 1 : (C > maxC ? maxC : C);
  C = C > kCoopMaxC ? kCoopMaxC : C;
  if (C <= 1) return 1;
  const int Cs = xs_chunk_size(N, C);
  return (N + Cs - 1) / Cs;
}
inline int xs_pipe_lag() {
  const int l = g_mfa_xs_lag;
  return l < 1 ? 1 : (l > kPipeMaxLag ? kPipeMaxLag : l);
}

// Workspace: partial moments [D][S][msize] | coef [D][Q+1+P] | partial R^2 sums [D][S][5] |
// per-tile validity bits [D][ceil(N/64)] u64 (fused kernel) | team counters (8 + 3 D) ints.
// S = max(chunked-path chunks, team chunks).
inline size_t xs_workspace_bytes(int D, int N, int P, int Q) {
  const int Pseg = P > 0 ? P : 1;
  const size_t ms = (size_t)Q * (Q + 1) / 2 + 2 * Q + 4 + (size_t)Pseg * (Q + 3);
  const size_t S1 = (size_t)xs_chunks(D, N), S2 = (size_t)xs_coop_chunks(D, N);
  const size_t S = S1 > S2 ? S1 : S2;
  return (size_t)D * (S * ms + Q + 1 + P + S * 5 + (N + kWT - 1) / kWT) * sizeof(double) +
         (kPipeGroups + 3 * (size_t)D) * sizeof(int);
}

// Persistent grid of the pipelined team kernel: resident workgroups (occupancy query, cached per
// kernel), a multiple of the 8 ticket groups, no more than the busiest group's tickets need.
template <typename K>
int pipe_grid(K kern, size_t lds, int D, int C) {
  // (kernel, LDS bytes) -> resident workgroups per CU; kernels of one signature share a type,
  // so the cache is keyed by the kernel's address
  static const void* keys[64];
  static size_t klds[64];
  static int vals[64], nkeys = 0, cus = 0;
  int per = -1;
  for (int i = 0; i < nkeys; ++i)
    if (keys[i] == (const void*)kern && klds[i] == lds) per = vals[i];
  if (per < 0) {
    int dev = 0;
    if (cus <= 0 && (hipGetDevice(&dev) != hipSuccess ||
                     hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess))
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 256, lds) != hipSuccess || per < 1) per = 1;
    if (nkeys < 64) {
      keys[nkeys] = (const void*)kern;
      klds[nkeys] = lds;
      vals[nkeys++] = per;
    }
  }
  int w = g_mfa_xs_pipe_wpc > 0 && g_mfa_xs_pipe_wpc < per ? g_mfa_xs_pipe_wpc : per;
  int G = w * cus;
  G -= G % kPipeGroups;
  const int need = kPipeGroups * ((D + kPipeGroups - 1) / kPipeGroups) * C;
  G = G < need ? G : need;
  return G < kPipeGroups ? kPipeGroups : G;
}

// Moments source of the fused kernel: plain vector loads straight into registers, or the
// LDS-DMA ring.  Measured (tools/xs_mode_time.py, profiles/r03_xs_plain_loads.jsonl): plain loads
// win for fp32 panels at every D (2520 dates: 298 -> 273 us) and for fp64 shards up to ~2
// dates per CU (315: 72 -> 66 us; a lone workgroup's LDS-DMA issue path caps near 25 GB/s per
// CU), the ring for larger fp64 steps (2520: 386 vs 395 us).  Bitwise-identical results.
constexpr int kXsPlainMaxD64 = 512;
#ifndef MFA_XS_RESIDENT_DEFAULT
#define MFA_XS_RESIDENT_DEFAULT 0
#endif
template <typename T>
inline bool xs_plain_moments(int D) {
  return sizeof(T) == 4 || D <= kXsPlainMaxD64;
}

#if MFA_AB
#include "ab/xs_resident_lds.h"
#endif

template <int Q, int VAR, typename T>
hipError_t launch_q(const T* X, const T* cap, const T* ret, const int16_t* ind, int D, int N,
                    int P, int pivot_mode, double tol, double* f, T* e, double* r2, double* stats,
                    int* status, double* ws, hipStream_t s) {
  using L = Layout<Q, T>;
  const int Pseg = P > 0 ? P : 1;
  const int MS = L::msize(Pseg);
  const bool det = (pivot_mode & kXsDeterministic) != 0;
  const bool refine = (pivot_mode & kXsRefine) != 0;
  const int pm = pivot_mode & 0xff;
  const int mode = g_mfa_xs_mode;
  const int Sc = xs_chunks(D, N), Ct = xs_coop_chunks(D, N);
  const bool team = Ct > 1 && Sc == 1;
  const int S = team ? Ct : Sc;  // partial-moment rows per date (read by the refine pass)
  const int Sw = Sc > Ct ? Sc : Ct;  // workspace layout stride (xs_workspace_bytes)
  const int C = xs_chunk_size(N, S);
  const bool chunked = !team && (S > 1 || mode == 1);
  double* mom = ws;
  double* coef = ws + (size_t)D * Sw * MS;
  double* sums = coef + (size_t)D * (Q + 1 + P);
  unsigned long long* okm = (unsigned long long*)(sums + (size_t)D * Sw * 5);
  int* sync = (int*)(okm + (size_t)D * ((N + kWT - 1) / kWT));
  const size_t seg8 = (size_t)L::seg_doubles(kRepMax, Pseg) * sizeof(double);
  const bool rep8 = seg8 <= kSegLdsBudget;
  const size_t lds1 = ((size_t)L::seg_doubles(rep8 ? kRepMax : 1, Pseg) + L::NACC) * sizeof(double);
  const size_t lds2 = solve_lds_bytes<Q, T>(Pseg);
  if (lds1 + fused_ring_bytes<Q, T>() > 160 * 1024 || lds2 > 64 * 1024) return hipErrorInvalidValue;
  if (refine && refine_any_lds_doubles<Q>(P) * sizeof(double) > 160 * 1024) return hipErrorInvalidValue;
  if (det && !rep8) return hipErrorNotSupported;
  const int16_t* indp = P > 0 ? ind : nullptr;
  constexpr bool PRE = sizeof(T) == 4;
#if MFA_AB
  const size_t res_lds = (!team && !chunked) ? xs_resident_lds<Q, T>(mode, det, D, N, P) : 0;
#else
  (void)team; (void)chunked; (void)C; (void)sums; (void)sync; (void)mode;
#endif
#if MFA_AB  // team (pipelined) and chunked paths, MFMA / resident / forced-variant A/B modes
  if (team) {
    if (hipError_t err = hipMemsetAsync(sync, 0, (kPipeGroups + 3 * (size_t)D) * sizeof(int), s)) return err;
    const int lag = xs_pipe_lag();
#define MFA_XS_PIPE(RR, VV)                                                                     \
  {                                                                                             \
    auto kern = xs_pipe_kernel<Q, RR, VV, T>;                                                   \
    const int G = pipe_grid(kern, lds1, D, S);                                                  \
    hipLaunchKernelGGL(kern, dim3(G), dim3(256), lds1, s, X, cap, ret, indp, D, N, P, Pseg, S,  \
                       C, lag, pm, tol, f, e, r2, stats, status, mom, coef, sums, okm, sync);   \
  }
    if (det) MFA_XS_PIPE(kRepMax, VAR | 32)
    else if (rep8) MFA_XS_PIPE(kRepMax, VAR)
    else MFA_XS_PIPE(1, VAR)
#undef MFA_XS_PIPE
  } else if (chunked) {
    const dim3 g(D * S);
    if (det)
      hipLaunchKernelGGL((xs_moments_kernel<Q, VAR | 32, kRepMax, T>), g, dim3(256), lds1, s, X,
                         cap, ret, indp, N, Pseg, S, C, mom);
    else if (rep8)
      hipLaunchKernelGGL((xs_moments_kernel<Q, VAR, kRepMax, T>), g, dim3(256), lds1, s, X, cap,
                         ret, indp, N, Pseg, S, C, mom);
    else
      hipLaunchKernelGGL((xs_moments_kernel<Q, VAR, 1, T>), g, dim3(256), lds1, s, X, cap, ret,
                         indp, N, Pseg, S, C, mom);
    hipLaunchKernelGGL(xs_solve_kernel<Q>, dim3(D), dim3(64), lds2, s, mom, S, P, Pseg, pm, tol, f,
                       coef, stats, status);
    if (!(VAR & 4)) {
      hipLaunchKernelGGL((xs_resid_kernel<Q, T>), g, dim3(256), 0, s, X, cap, ret, indp, D, N, P,
                         S, C, coef, status, e, r2, S > 1 ? sums : nullptr);
      if (S > 1)
        hipLaunchKernelGGL(xs_r2_combine_kernel<0>, dim3((D + 255) / 256), dim3(256), 0, s, sums, D,
                           S, status, r2);
    }
  } else if (Q == 10 && (mode == 10 || mode == 11 || mode == 12)) {
    // A/B only (headline Q): MFMA-moments fused kernel, 3 / 4 / 2 workgroups per CU (segment
    // replicas 4 / 2 / 8).  Measured slower than the VALU body at every occupancy
    // (profiles/r02_xs_mfma_ab.md), so never the default.
    const int Rm = mode == 12 ? 8 : (mode == 10 ? 4 : 2);
    const size_t ldsm = ((size_t)Rm * Pseg * L::NS + L::NACC) * sizeof(double);
    if (ldsm + fused_mf_ring_bytes<10, T>() > 160 * 1024) return hipErrorInvalidValue;
    if constexpr (Q == 10) {
      if (mode == 12)
        hipLaunchKernelGGL((xs_fused_mf_kernel<Q, 8, VAR, T, 2>), dim3(D), dim3(256), ldsm, s, X,
                           cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom);
      else if (mode == 10)
        hipLaunchKernelGGL((xs_fused_mf_kernel<Q, 4, VAR, T, 3>), dim3(D), dim3(256), ldsm, s, X,
                           cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom);
      else
        hipLaunchKernelGGL((xs_fused_mf_kernel<Q, 2, VAR, T, 4>), dim3(D), dim3(256), ldsm, s, X,
                           cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom);
    }
  } else if (res_lds > 0) {
    if constexpr (kResQ == Q && sizeof(T) == 8) {
      // A/B geometries (TL LDS tiles, TR AGPR tiles, A loads in flight per wave)
#define MFA_XS_RES(TL_, TR_, A_, V_)                                                            \
  {                                                                                             \
    auto kern = xs_resident_kernel<Q, TL_, TR_, A_, T, V_>;                                     \
    static size_t attr = 0; /* raise the dynamic-LDS limit once per size */                     \
    if (attr < res_lds) {                                                                       \
      if (hipError_t err = hipFuncSetAttribute((const void*)kern,                              \
                                               hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                               (int)res_lds))                                  \
        return err;                                                                             \
      attr = res_lds;                                                                           \
    }                                                                                           \
    hipLaunchKernelGGL(kern, dim3(D), dim3(256), res_lds, s, X, cap, ret, indp, N, P, Pseg, pm, \
                       tol, f, e, r2, stats, status, mom, g_mfa_xs_prof);                       \
  }
      if (mode == 32) MFA_XS_RES(5, 8, 3, 0)
      else if (mode == 33) MFA_XS_RES(5, 6, 4, 0)
      else if (mode == 34) MFA_XS_RES(0, 0, 4, 0)
      else if (mode == 35) MFA_XS_RES(5, 0, 4, 0)
      else if (mode == 36) MFA_XS_RES(kResTL, kResTR, kResA, 1)  // timing only: no atomics
      else if (mode == 37) MFA_XS_RES(kResTL, kResTR, kResA, 2)  // timing only: no Gram FMAs
      else if (mode == 38) MFA_XS_RES(kResTL, kResTR, kResA, 3)  // timing only: neither
      else MFA_XS_RES(kResTL, kResTR, kResA, 0)
#undef MFA_XS_RES
    }
  } else if ((mode == 23 || mode == 24) && det) {
    // A/B: residual prefetch during the solve on every storage type (plain-load / LDS-DMA moments)
    if (mode == 23)
      hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32 | 64, true, T>), dim3(D), dim3(256),
                         lds1, s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status,
                         mom, okm);
    else
      hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32, true, T>), dim3(D), dim3(256),
                         lds1, s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status,
                         mom, okm);
  } else if ((mode == 20 || mode == 21) && det) {  // mode 0 takes the production branch below
    // moments from plain vector loads (default for fp32 panels and small fp64 shards)
    if (mode == 21)  // two tiles in flight
      hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32 | 64 | 128, PRE, T>), dim3(D),
                         dim3(256), lds1, s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2,
                         stats, status, mom, okm);
    else
      hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32 | 64, PRE, T>), dim3(D),
                         dim3(256), lds1, s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2,
                         stats, status, mom, okm);
  } else
#endif  // MFA_AB
  if (det && mode == 0 && xs_plain_moments<T>(D)) {
    // moments from plain vector loads (default for fp32 panels and small fp64 shards; A/B mode 7
    // forces the LDS-DMA ring below).  The residual prefetch is on for every storage type, as
    // on the LDS-DMA path: its R^2 sums accumulate in the prefetch path's order, so a date's
    // R^2 is bitwise the same whichever path its launch's date count selects -- a date-sharded
    // run reproduces one process (fp64 D = 315: 65.3 vs 65.5 us, profiles/r03_xs_pre64_ab.jsonl)
    hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32 | 64, true, T>), dim3(D),
                       dim3(256), lds1, s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2,
                       stats, status, mom, okm);
  } else if (det) {  // bitwise-reproducible variant of the default path
    // residual prefetch during the solve on every storage type here (fp64 panels, D > 512:
    // 2520 dates 382 -> 370 us, profiles/r03_xs_pre64_ab.jsonl; no gain on the plain-load path)
    hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 32, true, T>), dim3(D), dim3(256), lds1,
                       s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom, okm);
  } else if (mode == 0 && rep8 && xs_plain_moments<T>(D)) {
    hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR | 64, PRE, T>), dim3(D), dim3(256), lds1,
                       s, X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom, okm);
  } else if (mode == 0 && rep8) {
    hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR, PRE, T>), dim3(D), dim3(256), lds1, s, X,
                       cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom, okm);
  } else if (rep8) {
    hipLaunchKernelGGL((xs_fused_kernel<Q, kRepMax, VAR, false, T>), dim3(D), dim3(256), lds1, s,
                       X, cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom, okm);
  } else {
    hipLaunchKernelGGL((xs_fused_kernel<Q, 1, VAR, false, T>), dim3(D), dim3(256), lds1, s, X,
                       cap, ret, indp, N, P, Pseg, pm, tol, f, e, r2, stats, status, mom, okm);
  }
  if (refine) {
    const size_t lds3 = refine_any_lds_doubles<Q>(P) * sizeof(double);
    hipLaunchKernelGGL((xs_refine_kernel<Q, T, true>), dim3(D), dim3(256), lds3, s, X, cap, ret,
                       indp, N, P, pm, S, mom, f, e, r2, status, (double*)nullptr);
  }
  return hipGetLastError();
}

template <typename T>
int xs_wls_dispatch(const T* X, const T* cap, const T* ret, const int16_t* ind, int D, int N,
                    int P, int Q, int pivot_mode, double tol, double* f, T* e, double* r2,
                    double* stats, int* status, void* ws, void* stream) {
  if (D <= 0) return 0;
  if (Q < 1 || Q > 16 || P < 0 || P > 128 || N <= 0 || (N % 8) != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  double* w = (double*)ws;
  switch (Q) {
#define MFA_Q(qq)                                                                              \
  case qq:                                                                                     \
    return (int)launch_q<qq, 0, T>(X, cap, ret, ind, D, N, P, pivot_mode, tol, f, e, r2,       \
                                   stats, status, w, s);
    MFA_Q(1) MFA_Q(2) MFA_Q(3) MFA_Q(4) MFA_Q(5) MFA_Q(6) MFA_Q(7) MFA_Q(8)
    MFA_Q(9) MFA_Q(10) MFA_Q(11) MFA_Q(12) MFA_Q(13) MFA_Q(14) MFA_Q(15) MFA_Q(16)
#undef MFA_Q
  }
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------
// Stock-sharded (TP) regression pieces, SURVEY.md §2.5: every rank streams ITS stocks of every
// date into raw moments (additive: the caller all-reduces them), solves redundantly from the
// summed moments, and forms its stocks' specific returns plus the five R^2 sums
// [sum e, sum e^2, sum r, sum r^2, n] per date (all-reduced again by the caller).
// what: 0 = moments, 1 = solve (type independent), 2 = residual sums, 3 = device pinv of the
// dates the solve flagged near-singular (rewrites f and coef in place; no host sync).
// ------------------------------------------------------------------------------------------
template <int Q, typename T>
hipError_t split_q(int what, const T* X, const T* cap, const T* ret, const int16_t* ind, int D,
                   int N, int P, int pivot_mode, double tol, double* mom, double* f,
                   double* coef, double* stats, int* status, T* e, double* sums, hipStream_t s) {
  using L = Layout<Q, T>;
  const int Pseg = P > 0 ? P : 1;
  const int16_t* indp = P > 0 ? ind : nullptr;
  if (what == 0) {
    const size_t seg8 = (size_t)L::seg_doubles(kRepMax, Pseg) * sizeof(double);
    const bool rep8 = seg8 <= kSegLdsBudget;
    const size_t lds1 = ((size_t)L::seg_doubles(rep8 ? kRepMax : 1, Pseg) + L::NACC) * sizeof(double);
    if (lds1 + Ring<Q, T>::BYTES > 160 * 1024) return hipErrorInvalidValue;
    if (rep8)
      hipLaunchKernelGGL((xs_moments_kernel<Q, 0, kRepMax, T>), dim3(D), dim3(256), lds1, s, X,
                         cap, ret, indp, N, Pseg, 1, N, mom);
    else
      hipLaunchKernelGGL((xs_moments_kernel<Q, 0, 1, T>), dim3(D), dim3(256), lds1, s, X, cap,
                         ret, indp, N, Pseg, 1, N, mom);
  } else if (what == 1) {
    const size_t lds2 = solve_lds_bytes<Q, T>(Pseg);
    if (lds2 > 64 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xs_solve_kernel<Q>, dim3(D), dim3(64), lds2, s, mom, 1, P, Pseg, pivot_mode,
                       tol, f, coef, stats, status);
  } else if (what == 3) {  // device pinv of flagged dates from the (all-reduced) moments
    const size_t lds3 = refine_any_lds_doubles<Q>(P) * sizeof(double);
    if (lds3 > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL((xs_refine_kernel<Q, T, false>), dim3(D), dim3(256), lds3, s,
                       (const T*)nullptr, (const T*)nullptr, (const T*)nullptr,
                       (const int16_t*)nullptr, 0, P, pivot_mode, 1, mom, f, (T*)nullptr,
                       (double*)nullptr, status, coef);
  } else {
    hipLaunchKernelGGL((xs_resid_kernel<Q, T>), dim3(D), dim3(256), 0, s, X, cap, ret, indp, D, N,
                       P, 1, N, coef, status, e, (double*)nullptr, sums);
  }
  return hipGetLastError();
}

template <typename T>
int split_dispatch(int what, const T* X, const T* cap, const T* ret, const int16_t* ind, int D,
                   int N, int P, int Q, int pivot_mode, double tol, double* mom, double* f,
                   double* coef, double* stats, int* status, T* e, double* sums, void* stream) {
  if (D <= 0) return 0;
  if (Q < 1 || Q > 16 || P < 0 || P > kXsSplitMaxP || N < 0 || (N % 8) != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  switch (Q) {
#define MFA_Q(qq)                                                                              \
  case qq:                                                                                     \
    return (int)split_q<qq, T>(what, X, cap, ret, ind, D, N, P, pivot_mode, tol, mom, f, coef, \
                               stats, status, e, sums, s);
    MFA_Q(1) MFA_Q(2) MFA_Q(3) MFA_Q(4) MFA_Q(5) MFA_Q(6) MFA_Q(7) MFA_Q(8)
    MFA_Q(9) MFA_Q(10) MFA_Q(11) MFA_Q(12) MFA_Q(13) MFA_Q(14) MFA_Q(15) MFA_Q(16)
#undef MFA_Q
  }
  return (int)hipErrorInvalidValue;
}

inline size_t xs_moments_bytes(int P, int Q) {
  const int Pseg = P > 0 ? P : 1;
  return ((size_t)Q * (Q + 1) / 2 + 2 * Q + 4 + (size_t)Pseg * (Q + 3)) * sizeof(double);
}

}  // namespace mfa_xs

using namespace mfa_xs;

// The per-Q instantiations are split over several translation units (xs_inst_*.hip) so the
// build compiles them in parallel; the entry-point TUs see only these declarations.
#define MFA_XS_LAUNCH_SIG(qq, vv, T)                                                            \
  hipError_t mfa_xs::launch_q<qq, vv, T>(const T*, const T*, const T*, const int16_t*, int, int,  \
                                         int, int, double, double*, T*, double*, double*, int*,  \
                                         double*, hipStream_t)
#define MFA_XS_SPLIT_SIG(qq, T)                                                                 \
  hipError_t mfa_xs::split_q<qq, T>(int, const T*, const T*, const T*, const int16_t*, int, int,  \
                                    int, int, double, double*, double*, double*, double*, int*,  \
                                    T*, double*, hipStream_t)
#define MFA_XS_INSTANTIATE(qq, T) template MFA_XS_LAUNCH_SIG(qq, 0, T); template MFA_XS_SPLIT_SIG(qq, T);
#define MFA_XS_DECLARE(qq, T) extern template MFA_XS_LAUNCH_SIG(qq, 0, T); extern template MFA_XS_SPLIT_SIG(qq, T);
#define MFA_XS_DECLARE_ALL(T)                                                                   \
  MFA_XS_DECLARE(1, T) MFA_XS_DECLARE(2, T) MFA_XS_DECLARE(3, T) MFA_XS_DECLARE(4, T)           \
  MFA_XS_DECLARE(5, T) MFA_XS_DECLARE(6, T) MFA_XS_DECLARE(7, T) MFA_XS_DECLARE(8, T)           \
  MFA_XS_DECLARE(9, T) MFA_XS_DECLARE(10, T) MFA_XS_DECLARE(11, T) MFA_XS_DECLARE(12, T)        \
  MFA_XS_DECLARE(13, T) MFA_XS_DECLARE(14, T) MFA_XS_DECLARE(15, T) MFA_XS_DECLARE(16, T)
