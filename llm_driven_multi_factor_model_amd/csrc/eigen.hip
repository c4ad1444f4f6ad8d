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
//     C_z,m = cov(z_m) are date-independent: they are computed ONCE per call with Philox
//     normals and fp32 MFMA (v_mfma_f32_32x32x2_f32, exact-f32 products, fp64 cross-chunk
//     accumulation) and C_b = S C_z,m S is formed on the fly per (date, sim);
//   * eigh (F0): one wave per matrix, pair-block tournament Jacobi (round-robin ordering,
//     K/2 disjoint rotations per round), packed A + position-space V in LDS, fp64 throughout;
//   * the (date, sim) Jacobi of the bias statistic carries M = V^T D0 V instead of V, works on
//     packed (A, M) pairs in tournament-position space and applies each round as 2x2 pair
//     blocks written straight to their next-round slots (all LDS addresses precomputed);
//   * grid (date, sim) for the simulations, per-(date, sim) bias vectors reduced by a
//     separate deterministic pass (no float atomics -> bitwise reproducible).
#include "common.h"
#include "jacobi.h"

namespace {

using namespace mfa;

// ---------------- Philox4x32-10 + Box-Muller ----------------
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
__device__ __forceinline__ float u01(unsigned v) {  // (0, 1]
  return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
// 4 standard normals for counter (a, b, c)
__device__ __forceinline__ void normal4(unsigned a, unsigned b, unsigned c, unsigned long long seed,
                                        float& n0, float& n1, float& n2, float& n3) {
  const U4 r = philox(U4{a, b, c, 0x4D464131u}, (unsigned)seed, (unsigned)(seed >> 32));
  const float r0 = sqrtf(-2.0f * __logf(u01(r.x))), r1 = sqrtf(-2.0f * __logf(u01(r.z)));
  float s0, c0, s1, c1;
  __sincosf(6.283185307179586f * u01(r.y), &s0, &c0);
  __sincosf(6.283185307179586f * u01(r.w), &s1, &c1);
  n0 = r0 * c0; n1 = r0 * s0; n2 = r1 * c1; n3 = r1 * s1;
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
// batched eigh: A [B][K][K] -> w [B][K] (descending), U [B][K][K] (U[:, k] = eigenvector k)
__global__ __launch_bounds__(64) void eigh_kernel(const double* __restrict__ Ain, int K,
                                                  int max_sweeps, double tol,
                                                  double* __restrict__ w, double* __restrict__ U,
                                                  int* __restrict__ sweeps) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int lda = K + 1;
  double* A = sm;
  double* V = A + K * lda;
  double* rot = V + K * lda;
  int* perm = (int*)(rot + 4 * 64);
  const double* a = Ain + (size_t)b * K * K;
  bool finite = true;
  for (int e = lane; e < K * K; e += 64) {
    const double x = a[e];
    finite = finite && __builtin_isfinite(x);
    A[(e / K) * lda + e % K] = x;
  }
  const bool ok = __all(finite);
  wsync();
  if (!ok) {  // propagate NaN (reference: eig raises -> empty frame)
    for (int k = lane; k < K; k += 64) w[(size_t)b * K + k] = qnan();
    for (int e = lane; e < K * K; e += 64) U[(size_t)b * K * K + e] = qnan();
    if (lane == 0 && sweeps) sweeps[b] = -1;
    return;
  }
  // symmetrise (NW matrices are symmetric up to rounding)
  for (int e = lane; e < K * K; e += 64) {
    const int i = e / K, j = e % K;
    if (i < j) {
      const double m = 0.5 * (A[i * lda + j] + A[j * lda + i]);
      A[i * lda + j] = m;
      A[j * lda + i] = m;
    }
  }
  wsync();
  const int ns = jacobi_wave(A, V, K, lda, rot, max_sweeps, tol);
  sort_desc(A, K, lda, perm);
  for (int k = lane; k < K; k += 64) w[(size_t)b * K + k] = A[perm[k] * lda + perm[k]];
  for (int e = lane; e < K * K; e += 64) {
    const int i = e / K, k = e % K;
    U[(size_t)b * K * K + e] = V[i * lda + perm[k]];
  }
  if (lane == 0 && sweeps) sweeps[b] = ns;
}

// C_z,m = cov(z_m) (ddof 1) for z_m [T x K] standard normals, fp32 MFMA 32x32x2 per 2 rows.
// Grid (M).  One wave: KP = 64 padded columns -> 2 x 2 output tiles of 32 x 32.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(64) void mc_cov_kernel(int K, int T, unsigned long long seed,
                                                    int m0, double* __restrict__ Cz) {
  // simulation m0 + blockIdx.x: the Philox stream depends only on (seed, global sim index), so
  // any partition of the sims over chunks / ranks draws exactly the single-run covariances
  const int m = m0 + blockIdx.x, lane = threadIdx.x;
  __shared__ float Z[64][65];   // 64 time rows x 64 (padded) factors
  __shared__ double colsum[64];
  const int col = lane & 31, half = lane >> 5;
  double acc64[3][16];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc64[t][r] = 0.0;
  double cs = 0.0;  // column sum for factor `lane`
  for (int t0 = 0; t0 < T; t0 += 64) {
    // draw a 64 x 64 block: row = time, col = factor (zero beyond K / T)
    for (int r = 0; r < 64; ++r) {
      // lane handles 1 factor; 4 normals per philox call -> use lane/4 counters
      const int tq = t0 + r;
      float n0, n1, n2, n3;
      normal4((unsigned)m, (unsigned)tq, (unsigned)(lane >> 2), seed, n0, n1, n2, n3);
      const int sub = lane & 3;
      const float z = sub == 0 ? n0 : (sub == 1 ? n1 : (sub == 2 ? n2 : n3));
      Z[r][lane] = (tq < T && lane < K) ? z : 0.0f;
    }
    wsync();
    f32x16 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
#pragma unroll 4
    for (int k = 0; k < 64; k += 2) {
      const float a0 = Z[k + half][col];        // tile row/col block 0
      const float a1 = Z[k + half][32 + col];   // block 1
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a0, acc[0], 0, 0, 0);  // (0,0)
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a1, acc[1], 0, 0, 0);  // (0,1)
      acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, a1, acc[2], 0, 0, 0);  // (1,1)
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc64[t][r] += (double)acc[t][r];
    for (int r = 0; r < 64; ++r) cs += (double)Z[r][lane];
    wsync();
  }
  colsum[lane] = cs;
  wsync();
  double* C = Cz + (size_t)blockIdx.x * K * K;
  const double invT1 = 1.0 / (double)(T - 1), invT = 1.0 / (double)T;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int bi = t == 2 ? 1 : 0, bj = t == 0 ? 0 : 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      const int j = bj * 32 + col;
      if (i < K && j < K) {
        const double v = (acc64[t][r] - colsum[i] * colsum[j] * invT) * invT1;
        C[i * K + j] = v;
        C[j * K + i] = v;
      }
    }
  }
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
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = fma(0.5 * y, fma(-x * y, y, 1.0), y);
  return fma(0.5 * y, fma(-x * y, y, 1.0), y);
}
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

// ---------------- split-layout variant of the bias Jacobi (A/B, mfa_eigen_set_bias_mode) --------
// Same tournament / pair-block schedule as jacobi_pairs, but A and M live in two separate
// packed arrays (same pk() slot index): A as fp64, M as MT (double, or float = storage-only
// fp32 with the rotation itself in fp64).  Per entry one ds_*_b64 (+ one b64 / b32) instead of
// one b128: with MT = float the LDS bytes per round drop by 25 %.  M only feeds the bias ratio
// diag(M)/diag(A); A (which decides convergence and Lambda) stays fp64.
template <int NB, int FAST, typename MT>
__device__ int jacobi_pairs_split(double* A, MT* Mm, double2* rcs, int Ke, int max_sweeps,
                                  double tol) {
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
    double offacc = 0.0, dgacc = 0.0;
    for (int r = 0; r < Ke - 1; ++r) {
      const bool last = r == Ke - 2;
      if (lane < npair) rcs[lane] = jacobi_cs<FAST>(A[ipp], A[iqq], A[ipq]);
      wsync();
      double av[NB][4], mv[NB][4];
      double2 rt[NB], ru[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (has[k]) {
          rt[k] = rcs[bT[k]];
          ru[k] = rcs[bU[k]];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            av[k][e] = A[rd[k][e]];
            mv[k][e] = (double)Mm[rd[k][e]];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (!has[k]) continue;
        rot_block(av[k][0], av[k][1], av[k][2], av[k][3], rt[k].x, rt[k].y, ru[k].x, ru[k].y);
        rot_block(mv[k][0], mv[k][1], mv[k][2], mv[k][3], rt[k].x, rt[k].y, ru[k].x, ru[k].y);
        if (diag[k]) {
          const double apq_new = (rt[k].y != 0.0) ? 0.0 : av[k][1];
          A[wr[k][0]] = av[k][0];
          A[wr[k][1]] = apq_new;
          A[wr[k][3]] = av[k][3];
          Mm[wr[k][0]] = (MT)mv[k][0];
          Mm[wr[k][1]] = (MT)(0.5 * (mv[k][1] + mv[k][2]));
          Mm[wr[k][3]] = (MT)mv[k][3];
          if (last) {
            dgacc = fma(av[k][0], av[k][0], fma(av[k][3], av[k][3], dgacc));
            offacc = fma(2.0 * apq_new, apq_new, offacc);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            A[wr[k][e]] = av[k][e];
            Mm[wr[k][e]] = (MT)mv[k][e];
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

template <int NB, int FAST, typename MT>
__global__ __launch_bounds__(64) void mc_bias_split_kernel(const double* __restrict__ D0, int K,
                                                           int M, const double* __restrict__ Cz,
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
  double* A = sm;                              // [np] fp64
  MT* Mm = (MT*)(A + np);                      // [np] MT (fits in the [np] doubles after A)
  double* dd = A + 2 * np;                     // [64]
  double2* rcs = (double2*)(dd + 64);          // [32]
  int* perm = (int*)(rcs + 32);                // [64]
  const double* d0 = D0 + (size_t)d * K;
  for (int k = lane; k < 64; k += 64) dd[k] = k < K ? sqrt(fmax(d0[k], 0.0)) : 0.0;
  wsync();
  const double* c = Cz + (size_t)m * K * K;
  for (int i = 0; i < Ke; ++i)
    for (int j = i + lane; j < Ke; j += 64) {
      const int s = pk(i, j, Ke);
      A[s] = (i < K && j < K) ? dd[i] * c[i * K + j] * dd[j] : 0.0;
      Mm[s] = (MT)((i == j && i < K) ? dd[i] * dd[i] : 0.0);
    }
  wsync();
  jacobi_pairs_split<NB, FAST, MT>(A, Mm, rcs, Ke, max_sweeps, tol);
  for (int k = lane; k < K; k += 64) {
    const double lk = A[pk(k, k, Ke)];
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const double lj = A[pk(j, j, Ke)];
      rank += (lj > lk) || (lj == lk && j < k);
    }
    perm[rank] = k;
  }
  wsync();
  for (int k = lane; k < K; k += 64) {
    const int s = pk(perm[k], perm[k], Ke);
    vo[k] = (double)Mm[s] / A[s];
  }
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

template <int NB, int NBV, int FAST = 0>
__global__ __launch_bounds__(64) void eigh_pairs_kernel(const double* __restrict__ Ain, int K,
                                                        int max_sweeps, double tol,
                                                        double* __restrict__ w,
                                                        double* __restrict__ U,
                                                        int* __restrict__ sweeps) {
  extern __shared__ double sm[];
  const int b = blockIdx.x, lane = threadIdx.x;
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
  // packed upper triangle of the symmetrised input (padding row / column zero), V = I
  for (int i = 0; i < Ke; ++i)
    for (int j = i + lane; j < Ke; j += 64)
      A[pk(i, j, Ke)] = (i < K && j < K) ? 0.5 * (a[i * K + j] + a[j * K + i]) : 0.0;
  for (int e = lane; e < K * Ke; e += 64) V[e] = (e / Ke == e % Ke) ? 1.0 : 0.0;
  wsync();
  const int ns = jacobi_pairs_vec<NB, NBV, FAST>(A, V, rcs, K, Ke, max_sweeps, tol);
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
__global__ __launch_bounds__(256) void eigen_finalize_kernel(const double* __restrict__ vin,
                                                             const double* __restrict__ D0,
                                                             const double* __restrict__ U0,
                                                             const int* __restrict__ dvalid,
                                                             int K, int M, int M_sum, double scale,
                                                             double* __restrict__ Fout,
                                                             double* __restrict__ vbias) {
  __shared__ double g[64];
  const int d = blockIdx.x, tid = threadIdx.x;
  const bool ok = dvalid[d] != 0;
  for (int k = tid; k < K; k += blockDim.x) {
    double s = 0.0;
    if (M_sum > 0) {
      s = vin[(size_t)d * K + k];
    } else {
      for (int m = 0; m < M; ++m) s += vin[((size_t)d * M + m) * K + k];
    }
    double v = sqrt(s / (M_sum > 0 ? M_sum : M));
    v = scale * (v - 1.0) + 1.0;
    if (vbias) vbias[(size_t)d * K + k] = ok ? v : qnan();
    g[k] = ok ? v * v * D0[(size_t)d * K + k] : qnan();
  }
  __syncthreads();
  const double* u = U0 + (size_t)d * K * K;
  for (int e = tid; e < K * K; e += blockDim.x) {
    const int i = e / K, j = e % K;
    double s = 0.0;
    for (int k = 0; k < K; ++k) s = fma(u[i * K + k] * g[k], u[j * K + k], s);
    Fout[(size_t)d * K * K + e] = ok ? s : qnan();
  }
}

int g_eigh_mode = 0;  // 0 = pair-block tournament Jacobi, 1 = row/column cyclic Jacobi (A/B)
int g_fast_rot = 1;   // 1 = rcp/rsq + Newton rotation parameters (jacobi_cs<1>); 0 = IEEE div/sqrt
int g_bias_mode = 0;  // 0 = packed (A, M) double2; 1 = split fp64 A / fp64 M; 2 = split, fp32 M

size_t eigh_lds(int K) { return ((size_t)2 * K * (K + 1) + 4 * 64 + 64) * sizeof(double) + 64 * sizeof(int); }

}  // namespace

MFA_API void mfa_eigh_set_mode(int mode) { g_eigh_mode = mode; }
MFA_API void mfa_eigen_set_fast_rotation(int on) { g_fast_rot = on; }
MFA_API void mfa_eigen_set_bias_mode(int mode) { g_bias_mode = mode; }

#define MFA_BIAS_LAUNCH(NBV_)                                                                   \
  {                                                                                            \
    if (g_bias_mode == 1)                                                                      \
      hipLaunchKernelGGL((mc_bias_split_kernel<NBV_, 1, double>), dim3(D * M), dim3(64),       \
                         bias_lds(K), s, D0, K, M, Cz, dvalid, max_sweeps, tol, ws);           \
    else if (g_bias_mode == 2)                                                                 \
      hipLaunchKernelGGL((mc_bias_split_kernel<NBV_, 1, float>), dim3(D * M), dim3(64),        \
                         bias_lds(K), s, D0, K, M, Cz, dvalid, max_sweeps, tol, ws);           \
    else if (g_fast_rot)                                                                       \
      hipLaunchKernelGGL((mc_bias_kernel<NBV_, 1>), dim3(D * M), dim3(64), bias_lds(K), s, D0, \
                         K, M, Cz, dvalid, max_sweeps, tol, ws);                               \
    else                                                                                       \
      hipLaunchKernelGGL((mc_bias_kernel<NBV_, 0>), dim3(D * M), dim3(64), bias_lds(K), s, D0, \
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
  if (g_eigh_mode == 0 && nb <= 4 * 64 && rows_per_lane <= 14 && g_fast_rot)
    hipLaunchKernelGGL((eigh_pairs_kernel<4, 14, 1>), dim3(B), dim3(64), eigh_pairs_lds(K), s, A,
                       K, max_sweeps, tol, w, U, sweeps);
  else if (g_eigh_mode == 0 && nb <= 4 * 64 && rows_per_lane <= 14)
    hipLaunchKernelGGL((eigh_pairs_kernel<4, 14>), dim3(B), dim3(64), eigh_pairs_lds(K), s, A, K,
                       max_sweeps, tol, w, U, sweeps);
  else if (g_eigh_mode == 0)
    hipLaunchKernelGGL((eigh_pairs_kernel<9, 32>), dim3(B), dim3(64), eigh_pairs_lds(K), s, A, K,
                       max_sweeps, tol, w, U, sweeps);
  else
    hipLaunchKernelGGL(eigh_kernel, dim3(B), dim3(64), eigh_lds(K), s, A, K, max_sweeps, tol, w, U,
                       sweeps);
  return (int)hipGetLastError();
}

MFA_API int mfa_mc_cov(int M, int K, int T, unsigned long long seed, double* Cz, void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || K > 64 || T < 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mc_cov_kernel, dim3(M), dim3(64), 0, (hipStream_t)stream, K, T, seed, 0, Cz);
  return (int)hipGetLastError();
}

// Draw covariances of sims [m0, m0 + M) (identical to those of a single mfa_mc_cov over all sims).
MFA_API int mfa_mc_cov_range(int M, int m0, int K, int T, unsigned long long seed, double* Cz,
                             void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || K > 64 || T < 2 || m0 < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mc_cov_kernel, dim3(M), dim3(64), 0, (hipStream_t)stream, K, T, seed, m0, Cz);
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
  hipLaunchKernelGGL(eigen_finalize_kernel, dim3(D), dim3(256), 0, s, ws, D0, U0, dvalid, K, M,
                     0, scale, Fout, vbias);
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
  if (K < 1 || K > 64 || M_total < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(eigen_finalize_kernel, dim3(D), dim3(256), 0, (hipStream_t)stream, S, D0, U0,
                     dvalid, K, 1, M_total, scale, Fout, vbias);
  return (int)hipGetLastError();
}
