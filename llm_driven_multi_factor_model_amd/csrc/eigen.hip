// Batched symmetric eigensolver and Monte-Carlo eigenfactor risk adjustment (K9) for gfx950.
//
// Reference: Barra-master/mfm/utils.py:55-92 (eigen_risk_adj) applied to every date by
// MFM.eigen_risk_adj_by_time (MFM.py:105-126):
//   F0 = U0 D0 U0^T ; for m < M: seed(m+1); b ~ N(0, diag D0) (K x T); F_m = cov(U0 b);
//   (D_m, U_m) = eig(F_m); v_m = diag(U_m^T F0 U_m) / D_m ;  v = sqrt(mean_m v_m);
//   v = a (v - 1) + 1 ;  F^ = U0 diag(v^2 D0) U0^T.
//
// MI355X design:
//   * eigenbasis identity: with b = diag(sqrt D0) z, F_m = U0 C_b U0^T and
//     v_m[k] = sum_l V[l,k]^2 D0[l] / Lambda[k] where (Lambda, V) = eigh(C_b); no U0 rotation
//     of the K x T draws is ever formed;
//   * the reference reseeds with m+1 for EVERY date (quirk Q8), so the draw covariances
//     C_z,m = cov(z_m) are date-independent: they are computed ONCE per call from fp64 Philox
//     normals (53-bit uniforms, fp64 Box-Muller) on the fp64 matrix cores
//     (v_mfma_f64_16x16x4f64), and C_b = S C_z,m S is formed on the fly per (date, sim);
//   * eigh (F0): one wave per matrix, pair-block tournament Jacobi (round-robin ordering,
//     K/2 disjoint rotations per round), packed A + position-space V in LDS, fp64 throughout;
//   * the (date, sim) bias statistic (252k 42x42 problems at the bench shape) is solved by
//     default (bias mode 3) with ONE Householder tridiagonalisation, per-lane count-guided
//     Laguerre eigenvalues, twisted-factorisation eigenvectors and a back-transform
//     (mc_bias_tri_kernel): 2.1x faster than the Jacobi on the pipeline's own inputs, bias
//     ratios equal to 3.5e-12 per sim (profiles/r02_eigen_tridiag.md);
//   * the pair-block Jacobi alternative (mode 0) carries M = V^T D0 V instead of V, works on
//     packed (A, M) pairs in tournament-position space and applies each round as 2x2 pair
//     blocks written straight to their next-round slots (all LDS addresses precomputed);
//   * grid (date, sim) for the simulations, per-(date, sim) bias vectors reduced by a
//     separate deterministic pass (no float atomics -> bitwise reproducible).
#include <utility>

#include "common.h"
#include "jacobi.h"
#include "tridiag.h"
#include "wide_gram.h"

namespace {

using namespace mfa;

// ---------------- Philox4x32-10 ----------------
struct U4 { unsigned x, y, z, w; };
__device__ __forceinline__ U4 philox(U4 c, unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
    const unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// descending-order rank of lane k's eigenvalue (ties broken by index): perm[rank] = k
__device__ void sort_desc(const double* A, int K, int lda, int* perm) {
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < K; k += 64) {
    const double lk = A[k * lda + k];
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const double lj = A[j * lda + j];
      rank += (lj > lk) || (lj == lk && j < k);
    }
    perm[rank] = k;
  }
  wsync();
}

// ---------------- kernels ----------------
#if MFA_AB  // row/column cyclic Jacobi (eigh mode 1, A/B only)
#include "ab/eigen_cyclic.h"
#endif

// C_z,m = cov(z_m) (ddof 1) for z_m [T x K] standard normals, all fp64 like the reference's
// numpy draws (MFM.py:113-120 via utils.py:70-76): 53-bit uniforms from Philox4x32-10, fp64
// Box-Muller, products on the fp64 matrix cores (v_mfma_f64_16x16x4f64) over 64-row LDS
// blocks, fp64 column sums for the centring.  Grid (M), one wave per simulation; KP = 64
// padded factors -> the 10 upper 16 x 16 tiles of the symmetric 64 x 64 sum of squares.
typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double u01_53(unsigned hi, unsigned lo) {  // (0, 1]
  return ((double)(((unsigned long long)(hi >> 5) << 26) | (lo >> 6)) + 1.0) * (1.0 / 9007199254740992.0);
}
// Grid (M sims x C time chunks): wave (m, c) draws the 64-row time blocks [b0, b1) of sim
// m0 + m.  C == 1 writes C_z directly; C > 1 writes its raw partial sums (the 10 MFMA tiles +
// the column sums, lane-major) to `part` [M][C][kCovPart] for mc_cov_reduce_kernel, which adds
// the C chunks in chunk order (deterministic) and centres: the same draws, and with ~20 chunks
// per sim the 100-sim launch fills the chip instead of 100 of its 256 CUs.
constexpr int kCovTiles = 10;
constexpr int kCovPart = kCovTiles * 4 * 64 + 64;  // doubles per (sim, chunk) partial
constexpr int TI_[kCovTiles] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
constexpr int TJ_[kCovTiles] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};

__device__ __forceinline__ void mc_cov_finish(const f64x4 (&acc)[kCovTiles], const double* colsum,
                                              int K, int T, double* __restrict__ C) {
  const int lane = threadIdx.x, r16 = lane & 15, k4 = lane >> 4;
  const double invT1 = 1.0 / (double)(T - 1), invT = 1.0 / (double)T;
#pragma unroll
  for (int t = 0; t < kCovTiles; ++t) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // 16x16x4 f64 output layout (tools/probes/mfma64_probe.hip): register e of lane l holds
      // D[(l >> 4) + 4 e][l & 15]; a diagonal tile writes its upper triangle (both halves)
      const int i = 16 * TI_[t] + k4 + 4 * e, j = 16 * TJ_[t] + r16;
      if (i < K && j < K && (TI_[t] != TJ_[t] || i <= j)) {
        const double v = (acc[t][e] - colsum[i] * colsum[j] * invT) * invT1;
        C[i * K + j] = v;
        C[j * K + i] = v;
      }
    }
  }
}

__global__ __launch_bounds__(64) void mc_cov_kernel(int K, int T, unsigned long long seed,
                                                    int m0, int C, double* __restrict__ Cz,
                                                    double* __restrict__ part) {
  // simulation m0 + blockIdx.x / C: the Philox stream depends only on (seed, global sim index,
  // time row), so any partition of the sims over chunks / ranks and of the time axis over
  // waves draws exactly the single-run normals
  const int mi = blockIdx.x / C, c = blockIdx.x - mi * C;
  const int m = m0 + mi, lane = threadIdx.x;
  const int nblk = (T + 63) / 64;
  const int per = (nblk + C - 1) / C;
  const int b0 = c * per, b1 = min(nblk, b0 + per);
  __shared__ double Z[64][66];  // 64 time rows x 64 (padded) factors; +2 pad: conflict-free
  __shared__ double colsum[64];
  const int r16 = lane & 15, k4 = lane >> 4;
  f64x4 acc[kCovTiles];
#pragma unroll
  for (int t = 0; t < kCovTiles; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  double cs = 0.0;  // column sum for factor `lane`
  for (int blk = b0; blk < b1; ++blk) {
    const int t0 = blk * 64;
    // draw a 64 x 64 block: row = time, col = factor (zero beyond K / T); one Philox call per
    // (time, factor pair) -> two 53-bit uniforms -> one Box-Muller pair
#pragma unroll 4
    for (int r = 0; r < 64; ++r) {
      const int tq = t0 + r;
      const U4 u = philox(U4{(unsigned)m, (unsigned)tq, (unsigned)(lane >> 1), 0x4D464131u},
                          (unsigned)seed, (unsigned)(seed >> 32));
      const double rr = sqrt(-2.0 * log(u01_53(u.x, u.y)));
      double sn, cn;
      sincospi(2.0 * u01_53(u.z, u.w), &sn, &cn);
      const double z = (lane & 1) ? rr * sn : rr * cn;
      Z[r][lane] = (tq < T && lane < K) ? z : 0.0;
    }
    wsync();
#pragma unroll 2
    for (int k = 0; k < 64; k += 4) {
      double a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = Z[k + k4][16 * i + r16];
#pragma unroll
      for (int t = 0; t < kCovTiles; ++t)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[TI_[t]], a[TJ_[t]], acc[t], 0, 0, 0);
    }
    for (int r = 0; r < 64; ++r) cs += Z[r][lane];
    wsync();
  }
  if (C > 1) {  // raw partials, lane-major: [t][e][lane], then the column sums
    double* pp = part + (size_t)blockIdx.x * kCovPart;
#pragma unroll
    for (int t = 0; t < kCovTiles; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) pp[(t * 4 + e) * 64 + lane] = acc[t][e];
    pp[kCovTiles * 4 * 64 + lane] = cs;
    return;
  }
  colsum[lane] = cs;
  wsync();
  mc_cov_finish(acc, colsum, K, T, Cz + (size_t)mi * K * K);
}

// Sum of the C time-chunk partials of each sim in chunk order, then the centring.
__global__ __launch_bounds__(64) void mc_cov_reduce_kernel(int K, int T, int C,
                                                           const double* __restrict__ part,
                                                           double* __restrict__ Cz) {
  const int mi = blockIdx.x, lane = threadIdx.x;
  __shared__ double colsum[64];
  f64x4 acc[kCovTiles];
#pragma unroll
  for (int t = 0; t < kCovTiles; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  double cs = 0.0;
  for (int c = 0; c < C; ++c) {
    const double* pp = part + ((size_t)mi * C + c) * kCovPart;
#pragma unroll
    for (int t = 0; t < kCovTiles; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][e] += pp[(t * 4 + e) * 64 + lane];
    cs += pp[kCovTiles * 4 * 64 + lane];
  }
  colsum[lane] = cs;
  wsync();
  mc_cov_finish(acc, colsum, K, T, Cz + (size_t)mi * K * K);
}

// ---------------- wide draw covariances (64 < K <= 144) on the fp64 matrix cores ----------------
// mc_cov_kernel's scheme on a 4-wave workgroup per (sim, time chunk): a 64-row block of the
// sim's normals (the same Philox counters {sim, time row, factor pair, tag}, so factor k draws
// the same number at any K) is staged in LDS as Z[64][KP], and the KT (KT + 1) / 2 upper
// 16 x 16 tiles of Z^T Z (KT = KP / 16: 21 tiles at KP = 96, 45 at 144) are dealt round-robin
// to the 4 waves, each tile one v_mfma_f64_16x16x4f64 chain over the block's 16 k-steps.
// Every (sim, chunk) writes its raw tile sums + column sums (lane-major) to `part`; the reduce
// kernel adds the chunks in chunk order (mc_cov_chunks: a function of T only) and centres, so a
// sim's matrix is bitwise the same in any launch.  Replaces the philox_normals_kernel +
// rocBLAS batched GEMM of round 4 (no [M][T][K] normals buffer in HBM either).
template <int KP>
__global__ __launch_bounds__(256) void mc_cov_wide_kernel(int K, int T, unsigned long long seed,
                                                          int m0, int C,
                                                          double* __restrict__ part) {
  using G = WideCov<KP>;
  const int mi = blockIdx.x / C, c = blockIdx.x - mi * C;
  const int m = m0 + mi, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nblk = (T + 63) / 64;
  const int per = (nblk + C - 1) / C;
  const int b0 = c * per, b1 = min(nblk, b0 + per);
  __shared__ double Z[64][KP + 2];  // +2: rows 2 banks apart, conflict-free column reads
  f64x4g acc[G::TPW];
#pragma unroll
  for (int u = 0; u < G::TPW; ++u) acc[u] = f64x4g{0.0, 0.0, 0.0, 0.0};
  double cs = 0.0;  // column sum of factor tid (tid < KP)
  constexpr int NPAIR = KP / 2;
  for (int blk = b0; blk < b1; ++blk) {
    const int t0 = blk * 64;
    for (int e = tid; e < 64 * NPAIR; e += 256) {
      const int r = e / NPAIR, pr = e - r * NPAIR, tq = t0 + r;
      const U4 u = philox(U4{(unsigned)m, (unsigned)tq, (unsigned)pr, 0x4D464131u},
                          (unsigned)seed, (unsigned)(seed >> 32));
      const double rr = sqrt(-2.0 * log(u01_53(u.x, u.y)));
      double sn, cn;
      sincospi(2.0 * u01_53(u.z, u.w), &sn, &cn);
      const bool okr = tq < T;
      Z[r][2 * pr] = (okr && 2 * pr < K) ? rr * cn : 0.0;
      Z[r][2 * pr + 1] = (okr && 2 * pr + 1 < K) ? rr * sn : 0.0;
    }
    __syncthreads();
    wide_gram_block<KP>(Z, wv, lane, acc);
    if (tid < KP)
      for (int r = 0; r < 64; ++r) cs += Z[r][tid];
    __syncthreads();
  }
  double* pp = part + (size_t)blockIdx.x * G::PART;
#pragma unroll
  for (int u = 0; u < G::TPW; ++u) {
    const int t = wv + G::NW * u;
    if (t < G::NT)
#pragma unroll
      for (int e = 0; e < 4; ++e) pp[(t * 4 + e) * 64 + lane] = acc[u][e];
  }
  if (tid < KP) pp[G::NT * 4 * 64 + tid] = cs;
}

// Chunk-ordered sum of the C partials of sim mi, centring, both triangles of C_z.  Grid (M),
// 256 threads: thread e of tile t's 256 (register, lane) slots.
template <int KP>
__global__ __launch_bounds__(256) void mc_cov_wide_reduce_kernel(int K, int T, int C,
                                                                 const double* __restrict__ part,
                                                                 double* __restrict__ Cz) {
  using G = WideCov<KP>;
  const int mi = blockIdx.x, tid = threadIdx.x;
  __shared__ double colsum[KP];
  for (int k = tid; k < KP; k += 256) {
    double s = 0.0;
    for (int c = 0; c < C; ++c) s += part[((size_t)mi * C + c) * G::PART + G::NT * 4 * 64 + k];
    colsum[k] = s;
  }
  __syncthreads();
  const double invT1 = 1.0 / (double)(T - 1), invT = 1.0 / (double)T;
  double* Cm = Cz + (size_t)mi * K * K;
  for (int t = 0; t < G::NT; ++t) {
    const int e = tid >> 6, lane = tid & 63;  // register e of lane `lane`
    double s = 0.0;
    for (int c = 0; c < C; ++c) s += part[((size_t)mi * C + c) * G::PART + (t * 4 + e) * 64 + lane];
    const int i = 16 * G::ti(t) + (lane >> 4) + 4 * e, j = 16 * G::tj(t) + (lane & 15);
    if (i < K && j < K && (G::ti(t) != G::tj(t) || i <= j)) {
      const double v = (s - colsum[i] * colsum[j] * invT) * invT1;
      Cm[i * K + j] = v;
      Cm[j * K + i] = v;
    }
  }
}

// ---------------- draw covariances for any K (K > 144) ----------------
// Output-tiled: a 4-wave workgroup per (sim, 64 x 64 block pair (bi <= bj), time chunk) draws
// the two 64-factor column blocks of its 64-row time blocks into LDS (the same Philox counters
// {sim, time row, factor pair, tag}: factor k draws the same number at every K) and accumulates
// Z_bi^T Z_bj on the fp64 matrix cores, wave w owning the 16-row strip w of the block (4 tiles);
// diagonal pairs also form their block's column sums.  Raw partials per (sim, pair, chunk) go
// to `part`; mc_cov_xl_reduce_kernel adds the chunks in chunk order (a function of T only) and
// centres, so a sim's matrix is bitwise the same in any launch.
constexpr int kXlPart = 64 * 64 + 64;  // doubles per (sim, pair, chunk)

__device__ __forceinline__ void xl_pair(int p, int KB, int& bi, int& bj) {
  int r = 0;
  while (p >= KB - r) { p -= KB - r; ++r; }
  bi = r;
  bj = r + p;
}

__device__ __forceinline__ void xl_draw_block(double (*Z)[66], int m, int t0, int T, int K, int b,
                                              unsigned long long seed, int tid) {
  for (int e = tid; e < 64 * 32; e += 256) {
    const int r = e >> 5, pc = e & 31, tq = t0 + r, pr = 32 * b + pc;
    const U4 u = philox(U4{(unsigned)m, (unsigned)tq, (unsigned)pr, 0x4D464131u},
                        (unsigned)seed, (unsigned)(seed >> 32));
    const double rr = sqrt(-2.0 * log(u01_53(u.x, u.y)));
    double sn, cn;
    sincospi(2.0 * u01_53(u.z, u.w), &sn, &cn);
    const bool okr = tq < T;
    Z[r][2 * pc] = (okr && 2 * pr < K) ? rr * cn : 0.0;
    Z[r][2 * pc + 1] = (okr && 2 * pr + 1 < K) ? rr * sn : 0.0;
  }
}

__global__ __launch_bounds__(256) void mc_cov_xl_kernel(int K, int T, unsigned long long seed,
                                                        int m0, int NP, int C,
                                                        double* __restrict__ part) {
  const int c = blockIdx.x % C, p = (blockIdx.x / C) % NP, mi = blockIdx.x / (C * NP);
  const int m = m0 + mi, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int KB = (K + 63) / 64;
  int bi, bj;
  xl_pair(p, KB, bi, bj);
  const int nblk = (T + 63) / 64;
  const int per = (nblk + C - 1) / C;
  const int b0 = c * per, b1 = min(nblk, b0 + per);
  __shared__ double Za[64][66], Zb[64][66];  // +2: conflict-free column reads
  const bool diag = bi == bj;
  f64x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f64x4{0.0, 0.0, 0.0, 0.0};
  double cs = 0.0;
  const int r16 = lane & 15, k4 = lane >> 4;
  for (int blk = b0; blk < b1; ++blk) {
    const int t0 = blk * 64;
    xl_draw_block(Za, m, t0, T, K, bi, seed, tid);
    if (!diag) xl_draw_block(Zb, m, t0, T, K, bj, seed, tid);
    __syncthreads();
    const double (*ZB)[66] = diag ? Za : Zb;
#pragma unroll 2
    for (int k = 0; k < 64; k += 4) {
      const double a = Za[k + k4][16 * wv + r16];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, ZB[k + k4][16 * u + r16], acc[u], 0, 0, 0);
    }
    if (diag && tid < 64)
      for (int r = 0; r < 64; ++r) cs += Za[r][tid];
    __syncthreads();
  }
  double* pp = part + (size_t)blockIdx.x * kXlPart;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) pp[((wv * 4 + u) * 4 + e) * 64 + lane] = acc[u][e];
  if (tid < 64) pp[64 * 64 + tid] = cs;
}

// Grid (M x NP), 256 threads: the chunk-ordered sums of one (sim, block pair), centred with the
// two blocks' column sums (from their diagonal pairs), written to both triangles.
__global__ __launch_bounds__(256) void mc_cov_xl_reduce_kernel(int K, int T, int NP, int C,
                                                               const double* __restrict__ part,
                                                               double* __restrict__ Cz) {
  const int p = blockIdx.x % NP, mi = blockIdx.x / NP, tid = threadIdx.x;
  const int KB = (K + 63) / 64;
  int bi, bj;
  xl_pair(p, KB, bi, bj);
  __shared__ double ca[64], cb[64];
  if (tid < 128) {
    const int bb = tid < 64 ? bi : bj, q = bb * KB - bb * (bb - 1) / 2;  // pair index of (bb, bb)
    double s = 0.0;
    for (int c = 0; c < C; ++c)
      s += part[(((size_t)mi * NP + q) * C + c) * kXlPart + 64 * 64 + (tid & 63)];
    (tid < 64 ? ca : cb)[tid & 63] = s;
  }
  __syncthreads();
  const double invT1 = 1.0 / (double)(T - 1), invT = 1.0 / (double)T;
  double* Cm = Cz + (size_t)mi * K * K;
  for (int x = tid; x < 64 * 64; x += 256) {
    double s = 0.0;
    for (int c = 0; c < C; ++c) s += part[(((size_t)mi * NP + p) * C + c) * kXlPart + x];
    // x = ((w * 4 + u) * 4 + e) * 64 + lane: D[(lane >> 4) + 4 e][lane & 15] of tile (w, u)
    const int ln = x & 63, e = (x >> 6) & 3, u = (x >> 8) & 3, w = x >> 10;
    const int li = 16 * w + (ln >> 4) + 4 * e, lj = 16 * u + (ln & 15);
    const int i = 64 * bi + li, j = 64 * bj + lj;
    if (i < K && j < K && (bi != bj || li <= lj)) {
      const double v = (s - ca[li] * cb[lj] * invT) * invT1;
      Cm[(size_t)i * K + j] = v;
      Cm[(size_t)j * K + i] = v;
    }
  }
}

// Wide factor sets (K > 64): the standard normals of sims [m0, m0 + M) as Z [M][T][Kp]
// (Kp = K rounded up to even, the padding column is a real draw the caller ignores), keyed
// exactly like mc_cov_kernel (Philox counter {sim, time row, factor pair, tag}, one Box-Muller
// pair per counter), so factor k < 64 of a sim draws the same numbers at any K.  The covariance
// is then one batched fp64 GEMM (rocBLAS) on the caller's side: the draw is the only custom step.
// One thread per (sim, row, factor pair): consecutive threads write consecutive 16-B pairs.
__global__ __launch_bounds__(256) void philox_normals_kernel(int M, int m0, int T, int Kp,
                                                             unsigned long long seed,
                                                             double* __restrict__ Z) {
  const int npair = Kp >> 1;
  const size_t n = (size_t)M * T * npair;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (size_t)gridDim.x * blockDim.x) {
    const int pr = (int)(e % npair);
    const size_t mt = e / npair;
    const int tq = (int)(mt % T), mi = (int)(mt / T);
    const U4 u = philox(U4{(unsigned)(m0 + mi), (unsigned)tq, (unsigned)pr, 0x4D464131u},
                        (unsigned)seed, (unsigned)(seed >> 32));
    const double rr = sqrt(-2.0 * log(u01_53(u.x, u.y)));
    double sn, cn;
    sincospi(2.0 * u01_53(u.z, u.w), &sn, &cn);
    *(double2*)(Z + mt * Kp + 2 * pr) = double2{rr * cn, rr * sn};
  }
}

// time chunks per sim: a function of T ONLY (at most 8 chunks of >= 2 64-row blocks), so the
// partial sums of a sim are added in the same order whatever the number of sims in the launch:
// any partition of the sims over chunks / ranks (eigen_chunk, the short last chunk, world size)
// reproduces one unsplit call bit for bit.  (Sizing C by M -- ~2048 waves per launch -- gave a
// 256-sim launch 8 chunks but a 16-sim tail 20 at T = 2520.)  M is unused.
inline int mc_cov_chunks(int /*M*/, int T) {
  const int nblk = (T + 63) / 64;
  const int per = max(2, (nblk + 7) / 8);
  return (nblk + per - 1) / per;  // no empty trailing chunk
}

// ---------------- pair-block Jacobi for the bias statistic ----------------
// Only v[k] = V[:,k]^T D0 V[:,k] / Lambda[k] is needed, so instead of the eigenvectors the
// kernel carries M = V^T D0 V, transformed two-sidedly like A (M <- J^T M J, M0 = diag D0):
// at convergence diag(A) = Lambda and diag(M)[k] = V[:,k]^T D0 V[:,k].  Both symmetric
// matrices are stored packed in LDS; one round of K/2 disjoint rotations is applied as 2x2
// pair blocks (t <= u), each block read and written once, with the block list of every lane
// fixed for the whole solve (round-robin ordering moves indices, not blocks).
//
// Packed layout = BLOCK-INTERLEAVED: element (i, j) lives at slot e * nbp + b, where b is the
// pair block (T, U) = (pair(i), pair(j)) sorted, and e = 2 side(i) + side(j) its entry (side =
// first / second position of the pair).  Lane l reads entry e of blocks l, l + 64, ...: 16
// consecutive lanes touch 16 consecutive 16-B slots (conflict-free ds_read_b128), and the
// next-round writes land on neighbouring blocks too.  The triangular packing it replaces had
// bank-conflict cycles at 89 % of LDS-active cycles (rocprofv3, mc_bias_kernel).
#ifndef MFA_PK_PAD
#define MFA_PK_PAD 16  // entry stride rounding (power of 2)
#endif
__host__ __device__ constexpr int pk_blocks_padded(int Ke) {
  return ((((Ke >> 1) * ((Ke >> 1) + 1)) >> 1) + MFA_PK_PAD - 1) & ~(MFA_PK_PAD - 1);
}
__host__ __device__ constexpr int pk_size(int Ke) { return 4 * pk_blocks_padded(Ke); }
__device__ __forceinline__ int pk(int i, int j, int Ke) {
  const int h = Ke >> 1;
  int pi = i < h ? i : Ke - 1 - i, si = i < h ? 0 : 1;
  int pj = j < h ? j : Ke - 1 - j, sj = j < h ? 0 : 1;
  if (pi > pj || (pi == pj && si > sj)) {  // symmetric: (i, j) and (j, i) share one slot
    const int tp = pi; pi = pj; pj = tp;
    const int ts = si; si = sj; sj = ts;
  }
  const int b = pi * h - ((pi * (pi - 1)) >> 1) + (pj - pi);
  return (2 * si + sj) * pk_blocks_padded(Ke) + b;
}

__device__ __forceinline__ void rot_block(double& x00, double& x01, double& x10, double& x11,
                                          double ct, double st, double cu, double su) {
  // rows (pair t): r0 = c r0 - s r1 ; r1 = s r0 + c r1 ; then columns (pair u) likewise
  const double y00 = ct * x00 - st * x10, y01 = ct * x01 - st * x11;
  const double y10 = st * x00 + ct * x10, y11 = st * x01 + ct * x11;
  x00 = cu * y00 - su * y01;
  x01 = su * y00 + cu * y01;
  x10 = cu * y10 - su * y11;
  x11 = su * y10 + cu * y11;
}

// Jacobi rotation (c, s) zeroing a_pq.  FAST = 1 replaces the IEEE-exact fp64 divisions and
// square roots (~50 dependent instructions) by v_rcp_f64 / v_rsq_f64 seeds refined with two
// Newton steps each (~28): the rotation only needs ~1 ulp, and this chain runs once per round
// on the critical path of every wave.
template <int FAST>
__device__ __forceinline__ double2 jacobi_cs(double app, double aqq, double apq) {
  double c = 1.0, s = 0.0;
  if constexpr (FAST) {
    if (fabs(apq) > 1e-300 && apq * apq > 1e-36 * fabs(app * aqq)) {
      const double th = (aqq - app) * (0.5 * rcp_nr(apq));
      double t;
      if (fabs(th) > 1e150) {
        t = 0.5 * rcp_nr(th);
      } else {
        const double u = fma(th, th, 1.0);
        t = copysign(rcp_nr(fabs(th) + u * rsq_nr(u)), th);
      }
      c = rsq_nr(fma(t, t, 1.0));
      s = t * c;
    }
  } else {
    if (fabs(apq) > 1e-300 && fabs(apq) > 1e-18 * sqrt(fabs(app * aqq))) {
      const double th = (aqq - app) / (2.0 * apq);
      const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
      c = 1.0 / sqrt(fma(t, t, 1.0));
      s = t * c;
    }
  }
  return double2{c, s};
}

// Returns sweeps used.  AM: packed Ke x Ke (A, M) pairs in TOURNAMENT-POSITION space (Ke = K
// rounded up to even; padding zero).  Round-robin ordering with positions fixed: every round
// pairs positions (t, Ke-1-t), and the circle shift (position 0 fixed, x -> x+1, Ke-1 -> 1)
// is applied by writing each rotated 2x2 pair block straight to its NEXT-round positions.  So
// every LDS address a lane touches is precomputed once: no per-round index arithmetic.  All of
// a wave's loads of a round are issued before its stores and LDS executes one wave's accesses
// in order, so the in-place permuted write-back needs no second buffer.
// NB = pair blocks per lane (>= nb / 64).
template <int NB, int FAST = 0>
__device__ int jacobi_pairs(double2* AM, double2* rcs, int Ke, int max_sweeps, double tol) {
  const int lane = threadIdx.x & 63;
  const int npair = Ke >> 1;
  const int nb = npair * (npair + 1) / 2;
  auto nxt = [&](int x) { return x == 0 ? 0 : (x == Ke - 1 ? 1 : x + 1); };
  // this lane's pair blocks (T, U), T <= U, with fixed read / write slots
  int rd[NB][4], wr[NB][4];
  bool has[NB], diag[NB];
  int bT[NB], bU[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int b = lane + 64 * k;
    int t = 0, rem = b;
    while (t < npair && rem >= npair - t) { rem -= npair - t; ++t; }
    has[k] = b < nb;
    const int T = has[k] ? t : 0, U = has[k] ? t + rem : 0;
    bT[k] = T;
    bU[k] = U;
    diag[k] = T == U;
    const int x0 = T, x1 = Ke - 1 - T, y0 = U, y1 = Ke - 1 - U;
    rd[k][0] = pk(x0, y0, Ke); rd[k][1] = pk(x0, y1, Ke);
    rd[k][2] = pk(x1, y0, Ke); rd[k][3] = pk(x1, y1, Ke);
    wr[k][0] = pk(nxt(x0), nxt(y0), Ke); wr[k][1] = pk(nxt(x0), nxt(y1), Ke);
    wr[k][2] = pk(nxt(x1), nxt(y0), Ke); wr[k][3] = pk(nxt(x1), nxt(y1), Ke);
  }
  const int ipp = pk(lane, lane, Ke), iqq = pk(Ke - 1 - lane, Ke - 1 - lane, Ke);
  const int ipq = pk(lane, Ke - 1 - lane, Ke);
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    // every off-diagonal entry lives in exactly one pair block per round, so the squares of
    // the values written in a sweep's LAST round are the exact post-sweep off / diag mass
    double offacc = 0.0, dgacc = 0.0;
    for (int r = 0; r < Ke - 1; ++r) {
      const bool last = r == Ke - 2;
      if (lane < npair)  // rotation of pair `lane`: positions (lane, Ke-1-lane)
        rcs[lane] = jacobi_cs<FAST>(AM[ipp].x, AM[iqq].x, AM[ipq].x);
      wsync();
      double av[NB][4], mv[NB][4];
      double2 rt[NB], ru[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {  // load
        if (has[k]) {
          rt[k] = rcs[bT[k]];
          ru[k] = rcs[bU[k]];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double2 v = AM[rd[k][e]];
            av[k][e] = v.x;
            mv[k][e] = v.y;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {  // rotate + store at next-round positions
        if (!has[k]) continue;
        rot_block(av[k][0], av[k][1], av[k][2], av[k][3], rt[k].x, rt[k].y, ru[k].x, ru[k].y);
        rot_block(mv[k][0], mv[k][1], mv[k][2], mv[k][3], rt[k].x, rt[k].y, ru[k].x, ru[k].y);
        if (diag[k]) {  // symmetric diagonal block: off-diagonal of A -> 0
          const double apq_new = (rt[k].y != 0.0) ? 0.0 : av[k][1];
          AM[wr[k][0]] = double2{av[k][0], mv[k][0]};
          AM[wr[k][1]] = double2{apq_new, 0.5 * (mv[k][1] + mv[k][2])};
          AM[wr[k][3]] = double2{av[k][3], mv[k][3]};
          if (last) {
            dgacc = fma(av[k][0], av[k][0], fma(av[k][3], av[k][3], dgacc));
            offacc = fma(2.0 * apq_new, apq_new, offacc);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            AM[wr[k][e]] = double2{av[k][e], mv[k][e]};
            if (last) offacc = fma(2.0 * av[k][e], av[k][e], offacc);
          }
        }
      }
      wsync();
    }
    const double off = wave_total(offacc), dgt = wave_total(dgacc);
    if (off <= tol * tol * dgt || off == 0.0) { ++sweep; break; }
  }
  return sweep;
}

// Per (date, sim): C_b = S C_z,m S (S = diag sqrt D0, eigen order of F0), Jacobi, bias vector
// vout[d][m][k] = (V[:,k]^T D0 V[:,k]) / Lambda[k]   (both spectra sorted descending)
template <int NB, int FAST = 0>
__global__ __launch_bounds__(64) void mc_bias_kernel(const double* __restrict__ D0, int K, int M,
                                                     const double* __restrict__ Cz,
                                                     const int* __restrict__ dvalid,
                                                     int max_sweeps, double tol,
                                                     double* __restrict__ vout) {
  extern __shared__ double sm[];
  const int d = blockIdx.x / M, m = blockIdx.x % M, lane = threadIdx.x;
  double* vo = vout + ((size_t)d * M + m) * K;
  if (!dvalid[d]) {
    for (int k = lane; k < K; k += 64) vo[k] = qnan();
    return;
  }
  const int Ke = K + (K & 1);
  const int np = pk_size(Ke);
  double2* AM = (double2*)sm;                  // [np] packed (A, M) pairs
  double* dd = (double*)(AM + np);             // [64]
  double2* rcs = (double2*)(dd + 64);          // [32]
  int* perm = (int*)(rcs + 32);                // [64]
  const double* d0 = D0 + (size_t)d * K;
  for (int k = lane; k < 64; k += 64) dd[k] = k < K ? sqrt(fmax(d0[k], 0.0)) : 0.0;
  wsync();
  const double* c = Cz + (size_t)m * K * K;
  for (int i = 0; i < Ke; ++i)
    for (int j = i + lane; j < Ke; j += 64) {
      const double a = (i < K && j < K) ? dd[i] * c[i * K + j] * dd[j] : 0.0;
      AM[pk(i, j, Ke)] = double2{a, (i == j && i < K) ? dd[i] * dd[i] : 0.0};
    }
  wsync();
  jacobi_pairs<NB, FAST>(AM, rcs, Ke, max_sweeps, tol);
  // descending rank of eigenvalue k (ties by index)
  for (int k = lane; k < K; k += 64) {
    const double lk = AM[pk(k, k, Ke)].x;
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const double lj = AM[pk(j, j, Ke)].x;
      rank += (lj > lk) || (lj == lk && j < k);
    }
    perm[rank] = k;
  }
  wsync();
  for (int k = lane; k < K; k += 64) {
    const double2 v = AM[pk(perm[k], perm[k], Ke)];
    vo[k] = v.y / v.x;
  }
}

#if MFA_AB
#include "ab/eigen_split.h"
#endif

#if MFA_AB
#include "ab/eigen_tri_v1.h"
#endif

// ---------------- lean tridiagonal bias solver (bias mode 4, the default) ----------------
// The same four phases and the same arithmetic as mc_bias_tri_kernel, re-laid-out for
// occupancy (the old kernel ran 2 waves / SIMD, bound by 217 VGPRs and 18.7 KB of LDS):
//   * C_z is symmetric, so lane i's row C_z[i][:] is read as the column C_z[:][i]: K coalesced
//     global loads (L2-resident, shared by every date of sim m), no LDS staging area;
//   * the reflector u_s is stored only over the live column range [8 floor(s/8), KP) of its
//     8-step group (packed rows, 16-B aligned) and the tridiagonalisation broadcasts u from that
//     row (no separate broadcast buffer): 12.3 KB of LDS at K = 42;
//   * the twisted factorisation keeps ONLY the eigenvector registers: the forward pivots are
//     written into y, the backward pivots are recomputed in a second pass for the part below
//     the twist instead of being stored (one extra K-step recurrence, 2 x KP fewer VGPRs).
// waves_per_eu(3) caps the registers at 168 -> 3 waves / SIMD (LDS allows 12 workgroups / CU).
#ifndef MFA_TRI2_WPE
#define MFA_TRI2_WPE 3
#endif
// (lds_batch, tri2_rows_doubles / tri2_row_off: csrc/tridiag.h)
// ABL: timing-only ablations (bias modes 61..67 = 60 + ABL, the production mode-5 kernel, KP = 44):
// 1 = no Laguerre iterations, 2 = no eigenvector / back-transform, 4 = no tridiagonalisation;
// outputs meaningless.
// EIG: batched symmetric eigendecomposition with the same machinery (eigh of F0): D0 = the input
// matrices [B][K][K] (symmetrised), M = 1, vout = w [B][K] descending, Uout [B][K][K] with
// U[:, k] = eigenvector k; flag[b] = 1 when the twisted-factorisation eigenvectors of a
// clustered spectrum are not orthogonal to 1e-12 (the caller re-solves those matrices with the
// Jacobi), 0 otherwise.  Non-finite matrices give NaN.
// ACC: a Laguerre step of relative size <= 10^-ACC (and shrinking, same Sturm count) is the
// last one; cubic convergence leaves far less than fp64 resolution after it.  A/B on the
// pipeline's inputs (profiles/r03_risk/bias_laguerre_stop_ab.jsonl): 1e-9 13.26 ms, 1e-8
// 12.40 ms (bias ratios within 3e-14 of the Jacobi, 1.9e-14 of LAPACK), 1e-7 11.65 ms but
// 1.4e-11 off: 1e-8 is the default; modes 8 / 9 select 1e-9 / 1e-7.
// NA: independent accumulators of the Householder matvec and the back-transform dot products
// (2, or 4: half the dependent fma chain per step, A/B bias mode 13).
// PAD: the tridiagonal is padded to KP with decoupled rows (alpha = 1e300, beta = 0) before the
// eigenvector phase, so its unrolled recurrences need no `i < K` tests: with a runtime K each
// test was a 64-bit scalar mask, ~100 of them spilled to VGPR lanes and reloaded (v_readlane +
// hazard nops + a branch) on every step of the dependent pivot chains.  Default for mode 5 at
// KP = 44 (12.0 -> 11.4-11.5 ms, bitwise the same ratios; mode 14 = unpadded, r04z/).
// ZR: reflector rows are stored for every step s < K (rows K-2, K-1 hold u = 0), so the
// Householder matvec always reads its own row: no per-read select of a fallback row (three
// SALU + one VALU per LDS read in the ISA) and constant row offsets (A/B bias modes 15 / 16).
// SK: the steps s >= K - 2 (tau = 0) skip the matvec and the update with a uniform branch, so
// the matvec never needs the fallback row either, without storing extra rows.  Default with PAD
// at KP = 44 (11.42-11.48 -> 11.36-11.38 ms, bitwise; `r04zc/`); mode 18 = the same kernel.
// FL: the Laguerre loop's square root and divisions (laguerre_toward, sturm_gh_p's 1 / f) as
// Newton-refined v_rsq / v_rcp (A/B bias mode 19).
// BT (with PAD): the back-transform skips a step on tau = 0 alone -- tau is 0 for s >= K - 2 and
// padded to 0 past K -- instead of also testing s + 2 >= K (a spilled scalar mask per step, A/B
// bias mode 20).
// CH: dates per wave (warm-started eigenvalues, bias mode 21).  Wave (c, m) solves the
// problems of dates CH c .. CH c + CH - 1 of sim m in order; each lane starts its Laguerre
// iteration for the k-th largest eigenvalue from the previous date's k-th eigenvalue (a
// slowly moving Newey-West spectrum: Weyl's bound |lambda_k(A) - lambda_k(B)| <= ||A - B||)
// instead of the k-th largest diagonal entry.  The first date of a chain and every date after
// an invalid one start cold.  Chains begin at global multiples of CH (Dn = D, dates counted
// from 0 in every launch), so a sims-sharded or chunked run reproduces the one-shot result.
template <int KP, bool PF = false, int ABL = 0, int WPE = MFA_TRI2_WPE, bool EIG = false,
          int ACC = 8, int LB = 8, int NA = 2, bool PAD = false, bool ZR = false, bool SK = false,
          bool FL = false, bool BT = false, int CH = 1, int GS = 8, bool LT = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void
mc_bias_tri2_kernel(const double* __restrict__ D0, int K, int M, const double* __restrict__ Cz,
                    const int* __restrict__ dvalid, double* __restrict__ vout,
                    double* __restrict__ Uout, int* __restrict__ flag, int Dn, int doff) {
  static_assert(CH == 1 || (!EIG && ABL == 0), "date chains: bias problems only");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int m = blockIdx.x % M, lane = threadIdx.x;
  // chains start at global dates that are multiples of CH: local date d is global d + date0,
  // and doff = date0 % CH shifts the first chain (CH == 1: doff = 0)
  const int d_first = (blockIdx.x / M) * CH - (CH > 1 ? doff : 0);
  double lam_prev = 0.0;  // this lane's eigenvalue of the previous date (CH > 1)
  bool warm = false;
  for (int ci = 0; ci < CH; ++ci) {
  const int d = d_first + ci;
  if (CH > 1 && d < 0) continue;
  if (CH > 1 && d >= Dn) break;
  lds_order();  // the previous date's LDS reads precede this date's writes
  double* vo = vout + ((size_t)d * M + m) * K;
  const double* Ain = D0 + (size_t)d * K * K;  // EIG input matrix
  if constexpr (EIG) {
    bool fin = true;
    for (int e = lane; e < K * K; e += 64) fin = fin && __builtin_isfinite(Ain[e]);
    if (!__all(fin)) {
      for (int k = lane; k < K; k += 64) vo[k] = qnan();
      for (int e = lane; e < K * K; e += 64) Uout[(size_t)d * K * K + e] = qnan();
      if (lane == 0) flag[d] = 0;
      return;
    }
  } else if (!dvalid[d]) {
    for (int k = lane; k < K; k += 64) vo[k] = qnan();
    warm = false;
    continue;
  }
  const int nrow = (tri2_rows_doubles<KP, GS>(ZR ? K + 2 : K) + 1) & ~1;
  double* R = sm;                          // packed reflector rows
  // LT: tables of KP entries instead of 64 (every lane-indexed write is guarded by lane < TS,
  // every read stays below KP; tb has one more entry, tb[KP] = {1e300, 0}, which the PAD
  // backward pivots read as the row past the last): 10.5 instead of 11.6 KB of LDS per
  // workgroup at K = 42, KP = 44 (15 workgroups per CU instead of 13), 9.7 KB at KP = 42 (16)
  constexpr int TS = LT ? KP : 64;
  double* wb = R + nrow;                   // [TS] broadcast w; Sturm counts later
  double2* tb = (double2*)(wb + TS);       // [TS (+1)] {alpha_i, beta_{i-1}^2}
  double* be = (double*)(tb + TS + (LT ? 1 : 0));  // [TS] beta_i
  double* ta = be + TS;                    // [TS] tau_s
  double* dd = ta + TS;                    // [TS] sqrt(D0)
  double* gs = dd + TS;                    // [TS] diagonal of A, descending; Laguerre x later
  const int li = lane < K ? lane : 0;
  double a[KP];
  double di = 0.0;
  const double* c = Cz + (size_t)m * K * K;
  if constexpr (EIG) {  // lane i's row of the symmetrised input
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      a[j] = j < K ? 0.5 * (Ain[j * K + li] + Ain[li * K + j]) : 0.0;
      if ((j & 7) == 7) lds_batch();
    }
  } else {
    const double* d0 = D0 + (size_t)d * K;
    di = lane < K ? sqrt(fmax(d0[lane], 0.0)) : 0.0;
    if (lane < TS) dd[lane] = di;
    lds_order();
    // lane i's row of A = S C_z S from the coalesced columns of the symmetric C_z
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      a[j] = j < K ? di * c[j * K + li] * dd[j] : 0.0;
      if ((j & 7) == 7) lds_batch();  // 8 loads in flight, not all 44 (register peak)
    }
  }
  {
    const double g = lane < K ? (EIG ? Ain[li * K + li] : di * c[li * K + li] * di) : 0.0;
    if (lane < TS) wb[lane] = g;
    lds_order();
    if (lane < K) {  // descending rank of the diagonal (ties by index): initial guesses
      int rank = 0;
      for (int j = 0; j < K; ++j) {
        const double h = wb[j];
        rank += (h > g) || (h == g && j < lane);
      }
      gs[rank] = g;
    }
    lds_order();
  }
  // ---- 1. Householder tridiagonalisation (rows in registers, u broadcast from its row) ----
  // Step s < K (runtime trip count); for s >= K - 2 the column below the subdiagonal is zero,
  // so tau = 0 and the step only records alpha_s / beta_s: s = K-2, K-1 are the final 2 x 2.
  auto steps = [&](auto J0c) {
    constexpr int J0 = decltype(J0c)::value;
    for (int s = J0; s < J0 + GS && s < K; ++s) {
      double xs = a[J0];
#pragma unroll
      for (int k = 1; k < GS; ++k)
        if (J0 + k < KP) {
          double t = a[J0 + k];
          asm volatile("" : "+v"(t));
          xs = s == J0 + k ? t : xs;
        }
      const bool act = lane > s && lane < K;
      const double x = act ? xs : 0.0;
      const double x0 = s + 1 < 64 ? readlane(xs, s + 1) : 0.0;
      const double sig = wave_total(lane > s + 1 && lane < K ? x * x : 0.0);
      const double alpha = readlane(xs, s);
      double u = 0.0, tau = 0.0, beta = x0;
      if (sig != 0.0) {
        // v_rsq / v_rcp seeds + two Newton steps (~1 ulp) instead of the IEEE sequences: they
        // sit on the per-step critical path of every problem
        const double n2 = fma(x0, x0, sig);
        const double nrm = n2 * rsq_nr(n2);
        beta = x0 >= 0.0 ? -nrm : nrm;
        tau = rcp_nr(nrm * (nrm + fabs(x0)));
        u = act ? (lane == s + 1 ? x0 - beta : x) : 0.0;
      }
      double* us = R + tri2_row_off<KP, GS>(s) - J0;  // us[j], j in [J0, KP)
      if ((ZR || s + 2 < K) && lane >= J0 && lane < KP) us[lane] = u;  // u_s, zero outside (s, K)
      if (lane == 0) {
        tb[s] = double2{alpha, s > 0 ? be[s - 1] * be[s - 1] : 0.0};
        be[s] = beta;
        ta[s] = tau;
      }
      lds_order();
      // branch-free: tau = 0 (nothing to reflect) gives u = p = w = 0, and lanes <= s have
      // u = p = w = 0, so the update is a no-op there (no divergent copies of the row)
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
      // rows s >= K - 2 are not stored (tau = 0 there): read the group's first row instead,
      // finite values times u = w = p = 0
      if constexpr (SK) {
        if (s + 2 >= K) continue;  // tau = 0: u = p = w = 0, nothing to update
      } else if (!ZR && s + 2 >= K) {
        us = R + tri2_row_off<KP, GS>(J0) - J0;
      }
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        if (NA == 4 && ((j - J0) & 2) != 0) {
          p2 = fma(a[j], uu.x, p2);
          p3 = fma(a[j + 1], uu.y, p3);
        } else {
          p0 = fma(a[j], uu.x, p0);
          p1 = fma(a[j + 1], uu.y, p1);
        }
        if (((j - J0) & (LB - 1)) == LB - 2) lds_batch();
      }
      const double p = act ? tau * (NA == 4 ? (p0 + p1) + (p2 + p3) : p0 + p1) : 0.0;
      const double kk = 0.5 * tau * wave_total(u * p);
      const double w = p - kk * u;
      if (lane < TS) wb[lane] = w;
      lds_order();
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 ww = *(const double2*)(wb + j), uu = *(const double2*)(us + j);
        // two fmas per element (the rank-2 update a - u w^T - w u^T): fma(u, w, w * u) then
        // a subtraction cost three VALU ops, and the kernel is VALU-issue bound
        a[j] = fma(-u, ww.x, fma(-w, uu.x, a[j]));
        a[j + 1] = fma(-u, ww.y, fma(-w, uu.y, a[j + 1]));
        if (((j - J0) & (LB - 1)) == LB - 2) lds_batch();
      }
      lds_order();
    }
  };
  static_assert(KP % (GS < 4 ? 2 : 4) == 0, "KP: multiple of 4 (of 2 with 2-step groups)");
  if constexpr ((ABL & 4) == 0) {
    [&]<int... G>(std::integer_sequence<int, G...>) {
      (steps(std::integral_constant<int, GS * G>{}), ...);
    }(std::make_integer_sequence<int, (KP + GS - 1) / GS>{});
  } else {  // ablation: T = the sorted diagonal with a weak coupling, no reflectors
    const double g = gs[lane < TS ? lane : 0];
    if (lane < TS) {
      tb[lane] = double2{g, lane > 0 ? 1e-12 * g * g : 0.0};
      be[lane] = 1e-6 * g;
      ta[lane] = 0.0;
    }
  }
  lds_order();
  // ---- 2. eigenvalue of rank `lane` (descending): as mc_bias_tri_kernel ----
  double lo_l = 0.0, hi_l = 0.0, b2max = 0.0;
  if (lane < K) {
    const double ad = tb[lane].x;
    const double r = (lane > 0 ? fabs(be[lane - 1]) : 0.0) + (lane + 1 < K ? fabs(be[lane]) : 0.0);
    lo_l = ad - r;
    hi_l = ad + r;
    b2max = tb[lane].y;
  } else {
    lo_l = tb[0].x;
    hi_l = tb[0].x;
  }
  const double gl = wave_min(lo_l), gu = wave_max(hi_l);
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, wave_max(b2max));
  constexpr double kEps = 2.220446049250313e-16;
  // LAPACK's absolute eigenvalue accuracy eps ||T|| (dstebz's default), not 1e-22 ||T||: the
  // smallest eigenvalues sit below what the fp64 Sturm recurrences resolve, so the extra
  // accuracy was bought with bisection steps on one lane that the whole wave waited for.  F0
  // eigh 0.86 -> 0.34 ms at K = 42, 4.0 -> 0.95 ms at K = 140 (same errors against LAPACK,
  // profiles/r05/r05l, r05m); bias problems 12.54 -> 11.99 ms at 2520 x 100, ratios within
  // 8.7e-16 of the 1e-22 setting and 5.9e-15 of LAPACK (r05n)
  const double abstol = kEps * tnorm + pivmin;
  const int jt = K - 1 - lane;
  double lo = gl - 2.0 * kEps * tnorm - pivmin, hi = gu + 2.0 * kEps * tnorm + pivmin;
  double x = lane < K ? fmin(fmax(gs[lane], lo), hi) : 0.5 * (lo + hi);
  if (CH > 1 && warm && lane < K) x = fmin(fmax(lam_prev, lo), hi);
  double G = 0.0, H = 0.0;
  auto sturm = [&](double xx) {
    if constexpr (PF) return sturm_gh_p<FL>(tb, K, xx, G, H);
    else return sturm_gh(tb, K, xx, pivmin, G, H);
  };
  int cnt = sturm(x);
  double* xsv = gs;  // each lane read its own gs slot above
  int* csv = (int*)wb;
  if (lane < TS) {
    xsv[lane] = x;
    csv[lane] = cnt;
  }
  lds_order();
  for (int l = 0; l < K; ++l) {
    const double xl = xsv[l];
    const int cl = csv[l];
    if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
  }
  double lam = x;
  constexpr double kAccTol = ACC == 9 ? 1e-9 : (ACC == 8 ? 1e-8 : (ACC == 7 ? 1e-7 : 1e-5));
  int nit = 0;  // Sturm evaluations after the first (ABL & 32: the diagnostic output)
  if (lane < K && (ABL & 1) == 0) {
    int prev = -1;
    double sprev = __builtin_inf();
    for (int it = 0; it < 256; ++it) {
      bool lag = false;
      double xn = 0.0;
      if (cnt == jt || cnt == jt + 1) {
        xn = laguerre_toward<FL>(x, G, H, K, cnt == jt);
        double st = fabs(xn - x);
        if (prev == cnt && st >= 1.5 * sprev) {
          xn = fma(8.0, xn - x, x);
          st *= 8.0;
        }
        lag = __builtin_isfinite(xn) && xn >= lo && xn <= hi;
        if (lag && prev == cnt && (st <= kAccTol * fabs(x) || st <= abstol) &&
            st <= 0.25 * sprev) { x = xn; break; }
        sprev = lag ? st : __builtin_inf();
      }
      if (!lag) { xn = 0.5 * (lo + hi); sprev = __builtin_inf(); }
      if (hi - lo <= 2.0 * kEps * (fabs(lo) + fabs(hi)) + abstol) { x = 0.5 * (lo + hi); break; }
      prev = lag ? cnt : -1;
      x = xn;
      cnt = sturm(x);
      ++nit;
      if (cnt <= jt) lo = x; else hi = x;
    }
    lam = x;
  }
  lam_prev = lam;
  warm = true;
  if constexpr ((ABL & 32) != 0) {  // diagnostic (A/B mode 68): each rank's Sturm evaluations
    if (lane < K) vo[lane] = (double)(nit + 1);
    return;
  }
  if constexpr ((ABL & 2) != 0) {  // ablation: no eigenvectors / back-transform
    if (lane < K) vo[lane] = lam;
    return;
  }
  // ---- 3. eigenvector of T at lam: twisted factorisation in the y registers only ----
  double y[KP];
  if constexpr (PAD) {
    // rows K .. 63 decoupled: alpha huge (never an eigenvalue rank a lane targets, pivots finite),
    // beta = 0 (be[K-1] is 0 already: column K of the reduced matrix is zero)
    lds_order();
    if (lane >= K && lane < TS) {
      tb[lane] = double2{1e300, 0.0};
      be[lane] = 0.0;
      if constexpr (BT) ta[lane] = 0.0;
    }
    // the row past the last (read by the backward pivots at i = KP - 1): lane TS, or lane 0
    // when the table spans the whole wave (KP = 64)
    if (LT && lane == (TS < 64 ? TS : 0)) tb[TS] = double2{1e300, 0.0};
    lds_order();
  }
  if (PAD && lane < K) {
    double dp = 0.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {  // forward pivots -> y
      const double2 t = tb[i];
      // the laundered copy keeps hipcc from keeping these 44 reciprocals alive for the
      // rcp_nr1(y[i]) of the below-the-twist loop (it spilled them to scratch)
      double q = dp;
      asm volatile("" : "+v"(q));
      dp = guard_pivot(i == 0 ? t.x - lam : (t.x - lam) - t.y * rcp_nr1(q), pivmin);
      y[i] = dp;
      if ((i & 3) == 3) lds_batch();  // not all 44 coefficient reads hoisted (register peak)
    }
    // backward pivots on the fly: the twist index r (padded rows: |gamma| ~ 1e300, never chosen)
    double dm = 1.0, gmin = 1e308;
    int r = K - 1;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      const double ai = tb[i].x - lam;
      double q = dm;  // laundered: the above-the-twist pass recomputes, not keeps, these
      asm volatile("" : "+v"(q));
      dm = guard_pivot(ai - tb[i + 1].y * rcp_nr1(q), pivmin);
      const double g = fabs(y[i] + dm - ai);
      if (g < gmin) { gmin = g; r = i; }
      if ((i & 3) == 0) lds_batch();
    }
    double cz = 1.0, nrm = 1.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {  // below the twist: y_i = -beta_i y_{i+1} / P_i
      if (i < r) {
        cz = -be[i] * cz * rcp_nr1(y[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
      if ((i & 3) == 0) lds_batch();
    }
    dm = 1.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {  // above the twist: recompute Q_i into y_i
      if (i > r) {
        const double ai = tb[i].x - lam;
        dm = guard_pivot(ai - tb[i + 1].y * rcp_nr1(dm), pivmin);
        y[i] = dm;
      }
      if ((i & 3) == 0) lds_batch();
    }
    cz = 1.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {  // padded rows: be[i-1] = 0 -> y_i = -0
      if (i == r) y[i] = 1.0;
      if (i > r) {
        cz = -be[i - 1] * cz * rcp_nr1(y[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
      if ((i & 3) == 3) lds_batch();
    }
    const double sc = rsq_nr(nrm);
#pragma unroll
    for (int i = 0; i < KP; ++i) y[i] *= sc;
  } else if (!PAD && lane < K) {
    double dp = 0.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {  // forward pivots -> y
      if (i < K) {
        const double2 t = tb[i];
        dp = guard_pivot(i == 0 ? t.x - lam : (t.x - lam) - t.y * rcp_nr1(dp), pivmin);
      }
      y[i] = i < K ? dp : 0.0;
    }
    double dm = 0.0, gmin = 0.0;
    int r = K - 1;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {  // backward pivots on the fly: the twist index r
      if (i < K) {
        const double ai = tb[i].x - lam;
        dm = guard_pivot(i == K - 1 ? ai : ai - tb[i + 1].y * rcp_nr1(dm), pivmin);
        const double g = fabs(y[i] + dm - ai);
        if (i == K - 1 || g < gmin) { gmin = g; r = i; }
      }
    }
    double cz = 1.0, nrm = 1.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {  // below the twist: y_i = -beta_i y_{i+1} / P_i
      if (i < r) {
        cz = -be[i] * cz * rcp_nr1(y[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
    }
    dm = 0.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {  // above the twist: recompute Q_i into y_i
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
      if (!(PAD && BT) && s + 2 >= K) continue;
      const double tau = ta[s];
      if (tau == 0.0) continue;
      const double* us = R + tri2_row_off<KP, GS>(s) - J0;
      double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        if (NA == 4 && ((j - J0) & 2) != 0) {
          t2 = fma(uu.x, y[j], t2);
          t3 = fma(uu.y, y[j + 1], t3);
        } else {
          t0 = fma(uu.x, y[j], t0);
          t1 = fma(uu.y, y[j + 1], t1);
        }
        if (((j - J0) & (LB - 1)) == LB - 2) lds_batch();
      }
      const double f = tau * (NA == 4 ? (t0 + t1) + (t2 + t3) : t0 + t1);
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        y[j] = fma(-f, uu.x, y[j]);
        y[j + 1] = fma(-f, uu.y, y[j + 1]);
        if (((j - J0) & (LB - 1)) == LB - 2) lds_batch();
      }
    }
  };
  [&]<int... G>(std::integer_sequence<int, G...>) {
    constexpr int NG = (KP + GS - 1) / GS;
    (back(std::integral_constant<int, GS * (NG - 1 - G)>{}, GS * (NG - 1 - G) + GS - 1), ...);
  }(std::make_integer_sequence<int, (KP + GS - 1) / GS>{});
  if constexpr (EIG) {
    // w (descending by lane rank), U[:, k] = y of lane k, and the orthogonality check of the
    // eigenvectors through the rows of Y in LDS, over the reflector rows and tables (all dead
    // now; one wave's DS instructions execute in order): 14.8 KB per workgroup at K = 42 instead
    // of 27 KB keeps ~2.5 waves per SIMD resident (0.93 -> ~0.2 ms for 2520 matrices)
    double* Ys = sm;
    lds_order();
    double* Ub = Uout + (size_t)d * K * K;
    if (lane < K) {
      vo[lane] = lam;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        if (j < K) Ub[j * K + lane] = y[j];
        Ys[lane * KP + j] = y[j];
      }
    }
    lds_order();
    double err = 0.0;
    if (lane < K) {
      for (int l = 0; l < K; ++l) {
        const double* yl = Ys + l * KP;
        double t0 = 0.0, t1 = 0.0;
#pragma unroll
        for (int j = 0; j < KP; j += 2) {
          t0 = fma(y[j], yl[j], t0);
          t1 = fma(y[j + 1], yl[j + 1], t1);
        }
        err = fmax(err, fabs(t0 + t1 - (l == lane ? 1.0 : 0.0)));
      }
    }
    err = wave_max(err);
    if (lane == 0) flag[d] = (err > 1e-12 || !(err == err)) ? 1 : 0;
    return;
  }
  if (lane < K) {
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < KP; ++j)  // dd[j] = 0 past K (and y[j] = 0 there)
      if (PAD || j < K) v = fma(dd[j] * dd[j], y[j] * y[j], v);
    vo[lane] = v / lam;
  }
  }  // date chain
}

#if MFA_AB
#include "ab/eigen_tri3.h"
#endif

// Householder steps per reflector-row group of the production tridiagonal kernels: a group of
// GS steps stores / reads / updates columns [GS floor(s / GS), KP), so smaller groups waste
// fewer fmas on the columns left of s (exact zeros: bitwise the same results) and select the
// step's column from fewer registers, at more unrolled code.  Bias solver at 2520 x 100 (A/B
// modes 27 / 25 / 5, profiles/r05/r05ai): GS = 8 11.64, 4 11.14, 2 10.82 ms.  Every bias
// instantiation runs GS = 2 with KP-entry tables (round 6: K = 32 6.65 -> 5.77 ms, K = 48 / 64
// -20 %, bitwise the same ratios, profiles/r06/bias_k_bench_*.log); the date chains and the
// EIG mode keep GS = 8.
constexpr int kTri2GS = 2;


size_t bias_tri2_lds(int K, int KP, int GS = 8, bool LT = false) {
  int n = 0;
  for (int s = 0; s + 2 < K; ++s) n += KP - GS * (s / GS);
  // tables (mc_bias_tri2_kernel's TS entries each; LT: tb has TS + 1)
  return ((size_t)((n + 1) & ~1) + (LT ? 7 * KP + 2 : 7 * 64)) * sizeof(double);
}
size_t eigh_tri2_lds(int K, int KP, int GS = 8) {
  const size_t b = bias_tri2_lds(K, KP, GS), y = (size_t)K * KP * sizeof(double);
  return b > y ? b : y;
}

// ---------------- pair-block Jacobi WITH eigenvectors (batched eigh of F0) ----------------
// Same tournament-position scheme as jacobi_pairs, carrying packed A and the full eigenvector
// matrix V [K][Ke] whose COLUMNS are positions: a round's column rotation of V uses the same
// (c, s) as A's and writes every rotated column pair straight to its next-round positions, so
// V[:, x] is always the eigenvector belonging to A's diagonal position x.
template <int NB, int NBV, int FAST = 0>
__device__ int jacobi_pairs_vec(double* A, double* V, double2* rcs, int K, int Ke,
                                int max_sweeps, double tol) {
  const int lane = threadIdx.x & 63;
  const int npair = Ke >> 1;
  const int nb = npair * (npair + 1) / 2;
  auto nxt = [&](int x) { return x == 0 ? 0 : (x == Ke - 1 ? 1 : x + 1); };
  int rd[NB][4], wr[NB][4];
  bool has[NB], diag[NB];
  int bT[NB], bU[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int b = lane + 64 * k;
    int t = 0, rem = b;
    while (t < npair && rem >= npair - t) { rem -= npair - t; ++t; }
    has[k] = b < nb;
    const int T = has[k] ? t : 0, U = has[k] ? t + rem : 0;
    bT[k] = T; bU[k] = U; diag[k] = T == U;
    const int x0 = T, x1 = Ke - 1 - T, y0 = U, y1 = Ke - 1 - U;
    rd[k][0] = pk(x0, y0, Ke); rd[k][1] = pk(x0, y1, Ke);
    rd[k][2] = pk(x1, y0, Ke); rd[k][3] = pk(x1, y1, Ke);
    wr[k][0] = pk(nxt(x0), nxt(y0), Ke); wr[k][1] = pk(nxt(x0), nxt(y1), Ke);
    wr[k][2] = pk(nxt(x1), nxt(y0), Ke); wr[k][3] = pk(nxt(x1), nxt(y1), Ke);
  }
  // V items: every lane serves ONE pair t (columns t and Ke-1-t) for rows sub, sub + lpp, ...
  // (lpp = lanes per pair), so one (c, s) per lane covers all of its items.
  const int lpp = 64 / npair;
  const int vt = lane % npair, vsub = lane / npair;
  const bool vlane = vsub < lpp;
  const int nvrow = vlane ? (K - vsub + lpp - 1) / lpp : 0;  // rows of this lane (<= NBV)
  const int ipp = pk(lane, lane, Ke), iqq = pk(Ke - 1 - lane, Ke - 1 - lane, Ke);
  const int ipq = pk(lane, Ke - 1 - lane, Ke);
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    double offacc = 0.0, dgacc = 0.0;
    for (int r = 0; r < Ke - 1; ++r) {
      const bool last = r == Ke - 2;
      if (lane < npair) rcs[lane] = jacobi_cs<FAST>(A[ipp], A[iqq], A[ipq]);
      wsync();
      double av[NB][4];
      double2 rt[NB], ru[NB];
      double v0[NBV], v1[NBV];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (has[k]) {
          rt[k] = rcs[bT[k]];
          ru[k] = rcs[bU[k]];
#pragma unroll
          for (int e = 0; e < 4; ++e) av[k][e] = A[rd[k][e]];
        }
      }
      const double2 rv = rcs[vt];
#pragma unroll
      for (int k = 0; k < NBV; ++k) {
        if (k < nvrow) {
          const int base = (vsub + lpp * k) * Ke;
          v0[k] = V[base + vt];
          v1[k] = V[base + Ke - 1 - vt];
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (!has[k]) continue;
        rot_block(av[k][0], av[k][1], av[k][2], av[k][3], rt[k].x, rt[k].y, ru[k].x, ru[k].y);
        if (diag[k]) {
          const double apq_new = (rt[k].y != 0.0) ? 0.0 : av[k][1];
          A[wr[k][0]] = av[k][0];
          A[wr[k][1]] = apq_new;
          A[wr[k][3]] = av[k][3];
          if (last) {
            dgacc = fma(av[k][0], av[k][0], fma(av[k][3], av[k][3], dgacc));
            offacc = fma(2.0 * apq_new, apq_new, offacc);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            A[wr[k][e]] = av[k][e];
            if (last) offacc = fma(2.0 * av[k][e], av[k][e], offacc);
          }
        }
      }
      // columns: V <- V J, written to next-round positions:
      // nxt(t) = t == 0 ? 0 : t + 1 ;  nxt(Ke-1-t) = t == 0 ? 1 : Ke - t
      const int c0 = vt == 0 ? 0 : vt + 1, c1 = vt == 0 ? 1 : Ke - vt;
#pragma unroll
      for (int k = 0; k < NBV; ++k) {
        if (k < nvrow) {
          const int base = (vsub + lpp * k) * Ke;
          V[base + c0] = rv.x * v0[k] - rv.y * v1[k];
          V[base + c1] = rv.y * v0[k] + rv.x * v1[k];
        }
      }
      wsync();
    }
    const double off = wave_total(offacc), dgt = wave_total(dgacc);
    if (off <= tol * tol * dgt || off == 0.0) { ++sweep; break; }
  }
  return sweep;
}

size_t eigh_pairs_lds(int K) {
  const int Ke = K + (K & 1);
  return ((size_t)pk_size(Ke) + (size_t)K * Ke + 64) * sizeof(double) +
         32 * sizeof(double2) + 64 * sizeof(int);
}

// only != nullptr: re-solve only the matrices with only[b] != 0 (the tridiagonal eigh's flags),
// warm-started from their tridiagonal eigenvectors when WARM
// (WARM: a separate instantiation -- its register-resident setup takes 256 VGPRs, which the
// cold batched Jacobi must not pay in occupancy)
template <int NB, int NBV, int FAST = 0, bool WARM = false>
__global__ __launch_bounds__(64) void eigh_pairs_kernel(const double* __restrict__ Ain, int K,
                                                        int max_sweeps, double tol,
                                                        double* __restrict__ w,
                                                        double* __restrict__ U,
                                                        int* __restrict__ sweeps,
                                                        const int* __restrict__ only) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, lane = threadIdx.x;
  if (only && !only[b]) return;
  const int Ke = K + (K & 1);
  const int np = pk_size(Ke);
  double* A = sm;
  double* V = A + np;
  double2* rcs = (double2*)(V + (size_t)K * Ke + ((np + K * Ke) & 1));
  int* perm = (int*)(rcs + 32);
  const double* a = Ain + (size_t)b * K * K;
  bool finite = true;
  for (int e = lane; e < K * K; e += 64) finite = finite && __builtin_isfinite(a[e]);
  if (!__all(finite)) {  // propagate NaN (reference: eig raises -> empty frame)
    for (int k = lane; k < K; k += 64) w[(size_t)b * K + k] = qnan();
    for (int e = lane; e < K * K; e += 64) U[(size_t)b * K * K + e] = qnan();
    if (lane == 0 && sweeps) sweeps[b] = -1;
    return;
  }
  bool diag_ok = false;  // warm start: B already diagonal to tol, the Jacobi has nothing to do
  if constexpr (WARM) {
    // Warm start of a flagged matrix (the tridiagonal eigh's eigenvectors U of a clustered
    // spectrum are accurate but not orthogonal to 1e-12): Q = U orthonormalised, then the
    // Jacobi runs on B = Q^T A Q -- diagonal off the clusters -- with V = Q accumulating its
    // rotations (0-1 sweeps instead of ~8 from I).
    // (1) Q by right-looking modified Gram-Schmidt, twice, with lane x holding column x in
    // registers: at step y lane y normalises its column and broadcasts it through LDS, every
    // later column subtracts its projection locally (no cross-lane reductions).  A column that
    // the second pass finds numerically inside the span of the earlier ones (a duplicated
    // vector: it keeps < 1/2 of its norm) is replaced by the first unit vector e_k that keeps
    // > 1/(2K) of its norm outside that span (one exists: the squared norms sum to K - y).
    // Q is kept as a zero-padded 64 x 64 block Qs (LDS past the Jacobi's buffers), so every
    // loop below runs over 64 rows / columns with no `< K` test: runtime-K tests in unrolled
    // loops cost one scalar mask per element, which spill and reload on every pass.
    double* t = (double*)rcs;  // 64 doubles of broadcast scratch before the Jacobi needs them
    double* Qs = (double*)(perm + 64);
    const bool col = lane < K;
    {
      double q[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) {  // unconditional loads (all in flight), masked by a
        // factor: a select lets the compiler sink each load into its own branch + wait
        const double u = U[(size_t)b * K * K + (size_t)min(i, K - 1) * K + min(lane, K - 1)];
        q[i] = u * ((col && i < K) ? 1.0 : 0.0);  // the input is finite (checked above)
      }
      if (!col) {
#pragma unroll
        for (int i = 0; i < 64; ++i) Qs[i * 64 + lane] = 0.0;
      }
      for (int pass = 0; pass < 2; ++pass) {
        for (int y = 0; y < K; ++y) {
          if (lane == y) {
            double n2 = 0.0;
#pragma unroll
            for (int i = 0; i < 64; ++i) n2 = fma(q[i], q[i], n2);
            if (pass == 1 && !(n2 > 0.25)) {
              for (int k = 0; k < K; ++k) {
#pragma unroll
                for (int i = 0; i < 64; ++i) q[i] = i == k ? 1.0 : 0.0;
                for (int rep = 0; rep < 2; ++rep)
                  for (int z = 0; z < y; ++z) {
                    double r = 0.0;
#pragma unroll
                    for (int i = 0; i < 64; ++i) r = fma(Qs[i * 64 + z], q[i], r);
#pragma unroll
                    for (int i = 0; i < 64; ++i) q[i] = fma(-r, Qs[i * 64 + z], q[i]);
                  }
                n2 = 0.0;
#pragma unroll
                for (int i = 0; i < 64; ++i) n2 = fma(q[i], q[i], n2);
                if (n2 > 0.5 / K) break;
              }
            }
            const double sc = n2 > 1e-30 ? 1.0 / sqrt(n2) : 0.0;
#pragma unroll
            for (int i = 0; i < 64; ++i) {
              q[i] *= sc;
              t[i] = q[i];
            }
            if (pass == 1) {
#pragma unroll
              for (int i = 0; i < 64; ++i) Qs[i * 64 + y] = q[i];
            }
          }
          wsync();
          if (lane > y && col) {
            double r0 = 0.0, r1 = 0.0;
#pragma unroll
            for (int i = 0; i < 64; i += 2) {
              r0 = fma(t[i], q[i], r0);
              r1 = fma(t[i + 1], q[i + 1], r1);
            }
            const double r = r0 + r1;
#pragma unroll
            for (int i = 0; i < 64; ++i) q[i] = fma(-r, t[i], q[i]);
          }
          wsync();
        }
      }
    }
    // V = Q for the Jacobi (K x Ke; the padding column is Qs's zero column K)
    for (int e = lane; e < K * Ke; e += 64) V[e] = Qs[(e / Ke) * 64 + e % Ke];
    // (2) B = Q^T A Q one column at a time with lane i holding row i of the symmetrised A in
    // registers: t = A q_y, then B[x][y] = q_x^T t for x <= y (lane x); the padding row /
    // column stay zero.  Off-diagonal and diagonal mass of B feed the Jacobi's own
    // convergence test, applied before its first sweep.
    double ar[64];
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const int jj = min(j, K - 1), ll = min(lane, K - 1);
      const double v = 0.5 * (a[ll * K + jj] + a[jj * K + ll]);
      ar[j] = v * ((col && j < K) ? 1.0 : 0.0);
    }
    wsync();
    double offacc = 0.0, dgacc = 0.0;
    for (int y = 0; y < Ke; ++y) {
      if (y >= K) {
        for (int x = lane; x <= y; x += 64) A[pk(x, y, Ke)] = 0.0;
        continue;
      }
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int j = 0; j < 64; j += 2) {
        t0 = fma(ar[j], Qs[j * 64 + y], t0);
        t1 = fma(ar[j + 1], Qs[(j + 1) * 64 + y], t1);
      }
      t[lane] = t0 + t1;
      wsync();
      if (lane <= y) {
        double b0 = 0.0, b1 = 0.0;
#pragma unroll
        for (int i = 0; i < 64; i += 2) {
          b0 = fma(Qs[i * 64 + lane], t[i], b0);
          b1 = fma(Qs[(i + 1) * 64 + lane], t[i + 1], b1);
        }
        const double bxy = b0 + b1;
        A[pk(lane, y, Ke)] = bxy;
        if (lane == y) dgacc = fma(bxy, bxy, dgacc);
        else offacc = fma(2.0 * bxy, bxy, offacc);
      }
      wsync();
    }
    const double off = wave_total(offacc), dgt = wave_total(dgacc);
    diag_ok = off <= tol * tol * dgt || off == 0.0;
  } else {
    // packed upper triangle of the symmetrised input (padding row / column zero), V = I
    for (int i = 0; i < Ke; ++i)
      for (int j = i + lane; j < Ke; j += 64)
        A[pk(i, j, Ke)] = (i < K && j < K) ? 0.5 * (a[i * K + j] + a[j * K + i]) : 0.0;
    for (int e = lane; e < K * Ke; e += 64) V[e] = (e / Ke == e % Ke) ? 1.0 : 0.0;
  }
  wsync();
  const int ns = diag_ok ? 0 : jacobi_pairs_vec<NB, NBV, FAST>(A, V, rcs, K, Ke, max_sweeps, tol);
  // descending rank of each real position's eigenvalue (ties by position); padding excluded:
  // the padded position holds an exact-zero row/column that no rotation ever mixes in
  int pad = -1;
  if (Ke != K) {  // find the padded coordinate's position: the column of V with V[:, x] == 0
    for (int x = lane; x < Ke; x += 64) {
      double nrm = 0.0;
      for (int i = 0; i < K; ++i) nrm = fma(V[i * Ke + x], V[i * Ke + x], nrm);
      if (nrm == 0.0) pad = x;
    }
    for (int off = 32; off > 0; off >>= 1) pad = max(pad, __shfl_xor(pad, off, 64));
  }
  for (int x = lane; x < Ke; x += 64) {
    if (x == pad) continue;
    const double lx = A[pk(x, x, Ke)];
    int rank = 0;
    for (int y = 0; y < Ke; ++y) {
      if (y == pad) continue;
      const double ly = A[pk(y, y, Ke)];
      rank += (ly > lx) || (ly == lx && y < x);
    }
    perm[rank] = x;
  }
  wsync();
  for (int k = lane; k < K; k += 64) w[(size_t)b * K + k] = A[pk(perm[k], perm[k], Ke)];
  for (int e = lane; e < K * K; e += 64) {
    const int i = e / K, k = e % K;
    U[(size_t)b * K * K + e] = V[i * Ke + perm[k]];
  }
  if (lane == 0 && sweeps) sweeps[b] = ns;
}

size_t bias_lds(int K) {
  const int Ke = K + (K & 1);
  return ((size_t)2 * pk_size(Ke) + 64) * sizeof(double) + 32 * sizeof(double2) + 64 * sizeof(int);
}

// Sum of the per-sim bias values over this chunk's sims, accumulated into S[d][k] (fixed
// order: deterministic).  Grid (D), block 64.
__global__ __launch_bounds__(64) void bias_sum_kernel(const double* __restrict__ vin, int K,
                                                      int M, double* __restrict__ S) {
  const int d = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += 64) {
    double s = 0.0;
    for (int m = 0; m < M; ++m) s += vin[((size_t)d * M + m) * K + k];
    S[(size_t)d * K + k] += s;
  }
}

// finalize: v = sqrt(mean_m v_m); v = a (v - 1) + 1; F^ = U0 diag(v^2 D0) U0^T.  Grid (D).
// `vin` holds per-sim values [D][M][K], or (M_sum > 0) per-date sums [D][K] over M_sum sims.
// STAGE (K <= 64): U0 of the date staged in LDS; larger K (any-K finalize) reads it from L1 / L2.
template <bool STAGE>
__global__ __launch_bounds__(256) void eigen_finalize_kernel(const double* __restrict__ vin,
                                                             const double* __restrict__ D0,
                                                             const double* __restrict__ U0,
                                                             const int* __restrict__ dvalid,
                                                             int K, int M, int M_sum, double scale,
                                                             double* __restrict__ Fout,
                                                             double* __restrict__ vbias) {
  extern __shared__ double g[];  // [K], then U0 of the date [K][K + 1] (odd row stride)
  double* us = g + K;
  const int d = blockIdx.x, tid = threadIdx.x;
  const bool ok = dvalid[d] != 0;
  const double* u = U0 + (size_t)d * K * K;
  if constexpr (STAGE)
    for (int e = tid; e < K * K; e += blockDim.x) us[(e / K) * (K + 1) + e % K] = u[e];
  for (int k = tid; k < K; k += blockDim.x) {
    double s = 0.0;
    if (M_sum > 0) {
      s = vin[(size_t)d * K + k];
    } else {  // same left-to-right sum; 8 loads in flight instead of one per dependent add
      const double* vk = vin + (size_t)d * M * K + k;
      int m = 0;
      for (; m + 8 <= M; m += 8) {
        double t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) t[q] = vk[(size_t)(m + q) * K];
#pragma unroll
        for (int q = 0; q < 8; ++q) s += t[q];
      }
      for (; m < M; ++m) s += vk[(size_t)m * K];
    }
    double v = sqrt(s / (M_sum > 0 ? M_sum : M));
    v = scale * (v - 1.0) + 1.0;
    if (vbias) vbias[(size_t)d * K + k] = ok ? v : qnan();
    g[k] = ok ? v * v * D0[(size_t)d * K + k] : qnan();
  }
  __syncthreads();
  // the same fma order as before, from LDS (U0 was re-read from L1 / L2 for every entry)
  for (int e = tid; e < K * K; e += blockDim.x) {
    const int i = e / K, j = e % K;
    const double* ui = STAGE ? us + i * (K + 1) : u + (size_t)i * K;
    const double* uj = STAGE ? us + j * (K + 1) : u + (size_t)j * K;
    double s = 0.0;
    for (int k = 0; k < K; ++k) s = fma(ui[k] * g[k], uj[k], s);
    Fout[(size_t)d * K * K + e] = ok ? s : qnan();
  }
}

size_t eigen_finalize_lds(int K, bool stage) {
  return ((size_t)K + (stage ? (size_t)K * (K + 1) : 0)) * sizeof(double);
}

int g_eigh_mode = 2;  // 0 = pair-block tournament Jacobi, 1 = row/column cyclic Jacobi (A/B),
                      // 2 = Householder tridiagonal (mc_bias_tri2_kernel<EIG>) + the pair-block
                      //     Jacobi for the matrices it flags (non-orthogonal eigenvectors)
int g_fast_rot = 1;   // 1 = rcp/rsq + Newton rotation parameters (jacobi_cs<1>); 0 = IEEE div/sqrt
int g_eigh_warm = 1;  // flagged-matrix re-solve warm-started from the tridiagonal eigenvectors
int g_bias_mode = 5;   // 21 = mode 5 walking 8 consecutive dates per wave with warm-
                       // started Laguerre eigenvalues (eigen stage 12.73-12.79 vs 13.10-13.26 ms,
                       // profiles/r05/r05b/bias_chain_ab.jsonl) -- opt-in: a date shard whose
                       // first date is not a chain start (global multiple of 8) cold-starts where
                       // one process warm-starts, so date-sharded runs are bitwise rank-invariant
                       // only with mode 5; 5 (default) = lean layout + division-free Sturm +
                       // padded eigenvector phase + skipped no-op Householder steps, one date per
                       // wave; 0 = packed (A, M) Jacobi.  A/B builds: 1 / 2 = split
                       // Jacobi, 3 = round-2 tridiagonal, 4 = lean layout, 14 = mode 5 unpadded,
                       // 22 / 23 = chains of 4 / 16 dates, 41-67 ablations, 71-77 phase
                       // ablations of the production K = 42 instantiation.

#if MFA_AB
size_t eigh_lds(int K) { return ((size_t)2 * K * (K + 1) + 4 * 64 + 64) * sizeof(double) + 64 * sizeof(int); }
#endif

}  // namespace

MFA_API int mfa_ab_build() { return MFA_AB; }

// Global index of date 0 of the next bias launches (date-chained modes 21-23: chains start at
// global multiples of the chain length, so a date-sharded or resumed run reproduces one
// process bit for bit).  0 by default.
int g_bias_date0 = 0;
MFA_API int mfa_eigen_set_date_origin(int d0) {
  if (d0 < 0) return (int)hipErrorInvalidValue;
  g_bias_date0 = d0;
  return 0;
}

// Setters return hipErrorInvalidValue for a variant this build does not contain (the A/B
// variants are compiled only with MFA_AB=1: python -m ..._build --ab).
MFA_API int mfa_eigh_set_warm(int on) {
  g_eigh_warm = on != 0;
  return 0;
}
MFA_API int mfa_eigh_set_mode(int mode) {
  if (!MFA_AB && mode == 1) return (int)hipErrorInvalidValue;
  g_eigh_mode = mode;
  return 0;
}
MFA_API int mfa_eigen_set_fast_rotation(int on) {
  if (!MFA_AB && !on) return (int)hipErrorInvalidValue;
  g_fast_rot = on;
  return 0;
}
MFA_API int mfa_eigen_set_bias_mode(int mode) {
  if (!MFA_AB && mode != 0 && mode != 5 && mode != 21) return (int)hipErrorInvalidValue;
  g_bias_mode = mode;
  return 0;
}

#if MFA_AB
#include "ab/eigen_ab_launch.h"
#endif  // MFA_AB

// Householder-tridiagonal solver (mode 5, the default): KP = K rounded up to an instantiated
// register width; the padded eigenvector phase and skipped no-op steps at the measured width
// (K <= 44).  The losing variants live behind MFA_AB (launch_bias_tri_ab).
bool launch_bias_tri(const double* D0, int D, int K, int M, const double* Cz, const int* dvalid,
                     double* ws, hipStream_t s) {
  const bool chain_mode = g_bias_mode == 21 || (MFA_AB && (g_bias_mode == 22 || g_bias_mode == 23));
  if (g_bias_mode == 5 || (chain_mode && K > 44)) {  // chains are instantiated at KP = 44
    // Every register width runs the lean form measured at K = 42 (profiles/r05/r05al: 10.74 ->
    // 9.18 ms at 2520 x 100): the padded eigenvector phase, skipped no-op Householder steps,
    // 2-step reflector groups and KP-entry LDS tables; the waves per SIMD are the most each
    // width holds without scratch (-Rpass-analysis=kernel-resource-usage: KP 8 / 16 -> 58 / 64
    // VGPRs, 8 waves; 24 -> 85, 5; 32 -> 101, 4; 42 / 44 -> 128, 4; 48 -> 132, 3; 64 -> 166, 3).
    // KP = 42 serves 32 < K <= 42 (the reference's 1 + 31 + 10 factors), KP = 32 the SSE50 run.
#define MFA_TRI2(KP_, WPE_)                                                                      \
    if (K <= KP_) {                                                                            \
      hipLaunchKernelGGL((mc_bias_tri2_kernel<KP_, true, 0, WPE_, false, 8, 8, 2, true, false,   \
                                              true, false, false, 1, kTri2GS, true>),           \
                         dim3(D * M), dim3(64), bias_tri2_lds(K, KP_, kTri2GS, true), s, D0, K, \
                         M, Cz, dvalid, ws, nullptr, nullptr, D, 0);                            \
      return true;                                                                             \
    }
    MFA_TRI2(8, 8)
    MFA_TRI2(16, 8)
    MFA_TRI2(24, 5)
    MFA_TRI2(32, 4)
    MFA_TRI2(42, 4)
    MFA_TRI2(44, 4)
    MFA_TRI2(48, 3)
    MFA_TRI2(64, 3)
#undef MFA_TRI2
    return false;
  }
#if MFA_AB
  if ((g_bias_mode == 25 || g_bias_mode == 27) && K <= 44) {  // A/B: 4- / 8-step groups
    if (g_bias_mode == 25)
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, true, false,
                                              true, false, false, 1, 4>),
                         dim3(D * M), dim3(64), bias_tri2_lds(K, 44, 4), s, D0, K, M, Cz, dvalid,
                         ws, nullptr, nullptr, D, 0);
    else
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, true, false,
                                              true, false, false, 1, 8>),
                         dim3(D * M), dim3(64), bias_tri2_lds(K, 44, 8), s, D0, K, M, Cz, dvalid,
                         ws, nullptr, nullptr, D, 0);
    return true;
  }
#endif
  if (chain_mode) {  // mode 5 + warm-started date chains (8 dates per wave; 4 / 16: A/B)
#define MFA_TRI2_CH(CH_)                                                                       \
    {                                                                                          \
      const int doff = g_bias_date0 % CH_;                                                     \
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, true, false, \
                                              true, false, false, CH_>),                         \
                         dim3(((D + doff + CH_ - 1) / CH_) * M), dim3(64), bias_tri2_lds(K, 44), s, \
                         D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, doff);                  \
    }
#if MFA_AB
    if (g_bias_mode == 22) MFA_TRI2_CH(4)
    else if (g_bias_mode == 23) MFA_TRI2_CH(16)
    else
#endif
    MFA_TRI2_CH(8)
#undef MFA_TRI2_CH
    return true;
  }
#if MFA_AB
  return launch_bias_tri_ab(D0, D, K, M, Cz, dvalid, ws, s);
#else
  return false;
#endif
}

#if MFA_AB
#define MFA_BIAS_LAUNCH_AB(NBV_)                                                                \
    else if (g_bias_mode == 1)                                                                 \
      hipLaunchKernelGGL((mc_bias_split_kernel<NBV_, 1, double>), dim3(D * M), dim3(64),       \
                         bias_lds(K), s, D0, K, M, Cz, dvalid, max_sweeps, tol, ws);           \
    else if (g_bias_mode == 2)                                                                 \
      hipLaunchKernelGGL((mc_bias_split_kernel<NBV_, 1, float>), dim3(D * M), dim3(64),        \
                         bias_lds(K), s, D0, K, M, Cz, dvalid, max_sweeps, tol, ws);           \
    else if (!g_fast_rot)                                                                      \
      hipLaunchKernelGGL((mc_bias_kernel<NBV_, 0>), dim3(D * M), dim3(64), bias_lds(K), s, D0, \
                         K, M, Cz, dvalid, max_sweeps, tol, ws);
#else
#define MFA_BIAS_LAUNCH_AB(NBV_)
#endif
// mode 0: pair-block Jacobi (fast rotations); every other mode: the tridiagonal dispatcher
#define MFA_BIAS_LAUNCH(NBV_)                                                                   \
  {                                                                                            \
    if (g_bias_mode != 0 && g_bias_mode != 1 && g_bias_mode != 2) {                            \
      if (!launch_bias_tri(D0, D, K, M, Cz, dvalid, ws, s)) return (int)hipErrorInvalidValue;  \
    }                                                                                          \
    MFA_BIAS_LAUNCH_AB(NBV_)                                                                   \
    else                                                                                       \
      hipLaunchKernelGGL((mc_bias_kernel<NBV_, 1>), dim3(D * M), dim3(64), bias_lds(K), s, D0, \
                         K, M, Cz, dvalid, max_sweeps, tol, ws);                               \
  }

MFA_API int mfa_eigh_batched(const double* A, int B, int K, int max_sweeps, double tol, double* w,
                             double* U, int* sweeps, void* stream) {
  if (B <= 0) return 0;
  if (K < 1 || K > 64) return (int)hipErrorInvalidValue;
  const int Ke = K + (K & 1), npair = Ke / 2, nb = npair * (npair + 1) / 2, nv = K * npair;
  hipStream_t s = (hipStream_t)stream;
  const int lpp = 64 / npair, rows_per_lane = (K + lpp - 1) / lpp;
  (void)nv;
  // mode 2: `sweeps` receives the tridiagonal solver's per-matrix fallback flags (required)
  const int* only = nullptr;
  if (g_eigh_mode == 2 && sweeps) {
    bool done = false;
#define MFA_EIGT(KP_)                                                                          \
    if (!done && K <= KP_) {                                                                 \
      hipLaunchKernelGGL((mc_bias_tri2_kernel<KP_, true, 0, MFA_TRI2_WPE, true>), dim3(B),   \
                         dim3(64), eigh_tri2_lds(K, KP_), s, A, K, 1, (const double*)nullptr, \
                         (const int*)nullptr, w, U, sweeps, B, 0);                               \
      done = true;                                                                           \
    }
    MFA_EIGT(8) MFA_EIGT(16) MFA_EIGT(24) MFA_EIGT(32) MFA_EIGT(44) MFA_EIGT(48) MFA_EIGT(64)
#undef MFA_EIGT
    only = sweeps;  // the Jacobi below re-solves the flagged matrices only
    sweeps = nullptr;
  }
  if (nb <= 4 * 64 && rows_per_lane <= 14 && (g_fast_rot || !MFA_AB)) {
    if (only && g_eigh_warm)  // + the 64 x 64 zero-padded Q block of the warm setup
      hipLaunchKernelGGL((eigh_pairs_kernel<4, 14, 1, true>), dim3(B), dim3(64),
                         eigh_pairs_lds(K) + 64 * 64 * sizeof(double), s, A, K, max_sweeps, tol, w,
                         U, sweeps, only);
    else
      hipLaunchKernelGGL((eigh_pairs_kernel<4, 14, 1>), dim3(B), dim3(64), eigh_pairs_lds(K), s, A,
                         K, max_sweeps, tol, w, U, sweeps, only);
  }
#if MFA_AB
  else if (g_eigh_mode == 1)  // A/B: row/column cyclic Jacobi
    hipLaunchKernelGGL(eigh_kernel, dim3(B), dim3(64), eigh_lds(K), s, A, K, max_sweeps, tol, w, U,
                       sweeps);
  else if (nb <= 4 * 64 && rows_per_lane <= 14)  // A/B: IEEE rotation parameters
    hipLaunchKernelGGL((eigh_pairs_kernel<4, 14>), dim3(B), dim3(64), eigh_pairs_lds(K), s, A, K,
                       max_sweeps, tol, w, U, sweeps, only);
#endif
  else
    hipLaunchKernelGGL((eigh_pairs_kernel<9, 32>), dim3(B), dim3(64), eigh_pairs_lds(K), s, A, K,
                       max_sweeps, tol, w, U, sweeps, only);
  return (int)hipGetLastError();
}

MFA_API int mfa_mc_cov(int M, int K, int T, unsigned long long seed, double* Cz, void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || K > 64 || T < 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mc_cov_kernel, dim3(M), dim3(64), 0, (hipStream_t)stream, K, T, seed, 0, 1,
                     Cz, (double*)nullptr);
  return (int)hipGetLastError();
}

// Draw covariances of sims [m0, m0 + M) (identical to those of a single mfa_mc_cov over all sims).
MFA_API int mfa_mc_cov_range(int M, int m0, int K, int T, unsigned long long seed, double* Cz,
                             void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || K > 64 || T < 2 || m0 < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mc_cov_kernel, dim3(M), dim3(64), 0, (hipStream_t)stream, K, T, seed, m0, 1,
                     Cz, (double*)nullptr);
  return (int)hipGetLastError();
}

// Wide draw covariances (64 < K <= 144, mc_cov_wide_kernel): scratch doubles for (M, K, T).
MFA_API size_t mfa_mc_cov_wide_ws_doubles(int M, int K, int T) {
  const int C = mc_cov_chunks(M, T);
  return (size_t)M * C * (K <= 96 ? WideCov<96>::PART : K <= 144 ? WideCov<144>::PART
                                                                : WideCov<160>::PART);
}

// Draw covariances of sims [m0, m0 + M), 64 < K <= 144, on the fp64 matrix cores: a sim's
// matrix is bitwise the same in any launch containing it (chunking by T only).
MFA_API int mfa_mc_cov_wide(int M, int m0, int K, int T, unsigned long long seed, double* ws,
                            double* Cz, void* stream) {
  if (M <= 0) return 0;
  if (K <= 64 || K > 160 || T < 2 || m0 < 0 || ws == nullptr) return (int)hipErrorInvalidValue;
  const int C = mc_cov_chunks(M, T);
  hipStream_t s = (hipStream_t)stream;
  if (K > 144) {
    hipLaunchKernelGGL(mc_cov_wide_kernel<160>, dim3(M * C), dim3(256), 0, s, K, T, seed, m0, C, ws);
    hipLaunchKernelGGL(mc_cov_wide_reduce_kernel<160>, dim3(M), dim3(256), 0, s, K, T, C, ws, Cz);
  } else if (K <= 96) {
    hipLaunchKernelGGL(mc_cov_wide_kernel<96>, dim3(M * C), dim3(256), 0, s, K, T, seed, m0, C, ws);
    hipLaunchKernelGGL(mc_cov_wide_reduce_kernel<96>, dim3(M), dim3(256), 0, s, K, T, C, ws, Cz);
  } else {
    hipLaunchKernelGGL(mc_cov_wide_kernel<144>, dim3(M * C), dim3(256), 0, s, K, T, seed, m0, C, ws);
    hipLaunchKernelGGL(mc_cov_wide_reduce_kernel<144>, dim3(M), dim3(256), 0, s, K, T, C, ws, Cz);
  }
  return (int)hipGetLastError();
}

// Draw covariances for any K (mc_cov_xl_kernel): scratch doubles for (M, K, T).
MFA_API size_t mfa_mc_cov_xl_ws_doubles(int M, int K, int T) {
  if (M <= 0 || K < 1 || T < 2) return 0;
  const int KB = (K + 63) / 64;
  return (size_t)M * (KB * (KB + 1) / 2) * mc_cov_chunks(M, T) * kXlPart;
}

// Draw covariances of sims [m0, m0 + M) for any K on the fp64 matrix cores (bitwise the same
// matrix for a sim in any launch containing it).
MFA_API int mfa_mc_cov_xl(int M, int m0, int K, int T, unsigned long long seed, double* ws,
                          double* Cz, void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || T < 2 || m0 < 0 || ws == nullptr) return (int)hipErrorInvalidValue;
  const int KB = (K + 63) / 64, NP = KB * (KB + 1) / 2, C = mc_cov_chunks(M, T);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mc_cov_xl_kernel, dim3(M * NP * C), dim3(256), 0, s, K, T, seed, m0, NP, C, ws);
  hipLaunchKernelGGL(mc_cov_xl_reduce_kernel, dim3(M * NP), dim3(256), 0, s, K, T, NP, C, ws, Cz);
  return (int)hipGetLastError();
}

// Normals of sims [m0, m0 + M) for any K (Z: [M][T][K + (K & 1)] doubles); see
// philox_normals_kernel.
MFA_API int mfa_philox_normals(int M, int m0, int K, int T, unsigned long long seed, double* Z,
                               void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || T < 1 || m0 < 0) return (int)hipErrorInvalidValue;
  const int Kp = K + (K & 1);
  const size_t n = (size_t)M * T * (Kp >> 1);
  const int blocks = (int)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
  hipLaunchKernelGGL(philox_normals_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, M,
                     m0, T, Kp, seed, Z);
  return (int)hipGetLastError();
}

// Scratch doubles mfa_mc_cov_range_ws needs for (M, T) (0: single-pass launch).
MFA_API size_t mfa_mc_cov_ws_doubles(int M, int T) {
  const int C = mc_cov_chunks(M, T);
  return C > 1 ? (size_t)M * C * kCovPart : 0;
}

// As mfa_mc_cov_range with the time axis split into mc_cov_chunks(T) chunks (partials in `ws`,
// summed in chunk order by a second launch).
MFA_API int mfa_mc_cov_range_ws(int M, int m0, int K, int T, unsigned long long seed, double* ws,
                                double* Cz, void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || K > 64 || T < 2 || m0 < 0) return (int)hipErrorInvalidValue;
  const int C = mc_cov_chunks(M, T);
  hipStream_t s = (hipStream_t)stream;
  if (C > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mc_cov_kernel, dim3(M * C), dim3(64), 0, s, K, T, seed, m0, C, Cz, ws);
  if (C > 1) hipLaunchKernelGGL(mc_cov_reduce_kernel, dim3(M), dim3(64), 0, s, K, T, C, ws, Cz);
  return (int)hipGetLastError();
}

// D0: [D][K] descending eigenvalues of F0 (valid dates only), U0: [D][K][K], dvalid: [D] int,
// Cz: [M][K][K]; ws: D*M*K doubles; outputs Fout [D][K][K], vbias [D][K] (nullable).
MFA_API int mfa_eigen_adjust(const double* D0, const double* U0, const int* dvalid, int D, int K,
                             int M, const double* Cz, double scale, int max_sweeps, double tol,
                             double* ws, double* Fout, double* vbias, void* stream) {
  if (D <= 0) return 0;
  if (K < 1 || K > 64 || M < 1) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int Ke = K + (K & 1), npair = Ke / 2, nb = npair * (npair + 1) / 2;
  if (nb <= 4 * 64)
    MFA_BIAS_LAUNCH(4)
  else
    MFA_BIAS_LAUNCH(9)
  hipLaunchKernelGGL(eigen_finalize_kernel<true>, dim3(D), dim3(256), eigen_finalize_lds(K, true), s,
                     ws, D0, U0, dvalid, K, M, 0, scale, Fout, vbias);
  return (int)hipGetLastError();
}

// Chunked / sharded Monte Carlo: S[d][k] += sum over this call's M sims of v_m[d][k].
// ws: D*M*K doubles.  Invalid dates accumulate NaN (finalize masks them anyway).
MFA_API int mfa_eigen_bias_accumulate(const double* D0, const int* dvalid, int D, int K, int M,
                                      const double* Cz, int max_sweeps, double tol, double* ws,
                                      double* S, void* stream) {
  if (D <= 0 || M <= 0) return 0;
  if (K < 1 || K > 64) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int Ke = K + (K & 1), npair = Ke / 2, nb = npair * (npair + 1) / 2;
  if (nb <= 4 * 64)
    MFA_BIAS_LAUNCH(4)
  else
    MFA_BIAS_LAUNCH(9)
  hipLaunchKernelGGL(bias_sum_kernel, dim3(D), dim3(64), 0, s, ws, K, M, S);
  return (int)hipGetLastError();
}

// Finalize from accumulated sums S [D][K] over M_total sims.
MFA_API int mfa_eigen_finalize_sum(const double* S, int M_total, const double* D0, const double* U0,
                                   const int* dvalid, int D, int K, double scale, double* Fout,
                                   double* vbias, void* stream) {
  if (D <= 0) return 0;
  if (K < 1 || K > 4096 || M_total < 1) return (int)hipErrorInvalidValue;  // any K (LDS: K doubles)
  if (K <= 64)
    hipLaunchKernelGGL(eigen_finalize_kernel<true>, dim3(D), dim3(256), eigen_finalize_lds(K, true),
                       (hipStream_t)stream, S, D0, U0, dvalid, K, 1, M_total, scale, Fout, vbias);
  else
    hipLaunchKernelGGL(eigen_finalize_kernel<false>, dim3(D), dim3(256), eigen_finalize_lds(K, false),
                       (hipStream_t)stream, S, D0, U0, dvalid, K, 1, M_total, scale, Fout, vbias);
  return (int)hipGetLastError();
}
