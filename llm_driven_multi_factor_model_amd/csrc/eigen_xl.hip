// Eigen solver and Monte-Carlo eigenfactor bias statistic for factor sets wider than the
// register / LDS-resident kernels (144 < K <= 1024, e.g. SW-L3 industries) on gfx950.
//
// Reference: Barra-master/mfm/utils.py:55-92 (eigen_risk_adj: np.linalg.eig of every simulated
// covariance, v_m = diag(U_m^T F0 U_m) / D_m) applied per date by MFM.py:105-126, which works
// at any K.  The K <= 144 solvers (csrc/eigen.hip, csrc/eigen_wide.hip) keep a problem's rows in
// registers and its reflectors in LDS; a 200 x 200 fp64 matrix alone is 320 KB, twice a CU's
// LDS, so here a problem's working matrix lives in a per-workgroup global slot (L2 / MALL
// resident while the workgroup works on it) and only vectors sit in LDS:
//   * one 8-wave workgroup per problem, persistent over the batch (grid = slots, problem
//     b = blockIdx.x + q gridDim.x): no host synchronisation and no vendor library;
//   * Householder tridiagonalisation on the lower triangle with the rank-2 update of step s fused
//     into the matrix-vector product of step s + 1: one read + one write of the trailing
//     triangle per step.  Waves own rows and lanes own 64-column chunks, so every access is a
//     coalesced row segment; by symmetry y = A v is a column sum over the rows below (each lane
//     its own column, the 8 wave partials meet in LDS in wave order) plus a row sum left of the
//     diagonal (one wave total per row);
//   * eigenvalues by bisection on the division-free Sturm recurrence (tridiag.h's determinant
//     form, count only), one lane per eigenvalue, the tridiagonal scaled to unit norm and every
//     eigenvalue resolved to LAPACK's eps ||T||;
//   * eigenvectors by twisted factorisation (one lane per eigenvalue; its pivots in a
//     lane-interleaved global scratch), written column-wise: coalesced over the lanes;
//   * eigh only: max |Y^T Y - I| of the tridiagonal eigenvectors on the fp64 matrix cores (the
//     back-transform is orthogonal, so that is U's orthogonality); a matrix that fails it (a
//     clustered spectrum) is re-solved in its slot by a cyclic round-robin Jacobi;
//   * the back-transform by the reflectors stored in the working matrix's rows, in compact-WY
//     blocks of 16 on the fp64 matrix cores (xl_back_wy): waves own 32-column chunks of Y, so
//     the K - 2 reflector applications need no workgroup barrier.
// Deterministic: fixed reduction orders, no atomics.  Replaces rocSOLVER's batched syevd, a
// rocBLAS GEMM and a host-syncing torch.nonzero (round 5's K > 144 path).
#include "common.h"
#include "tridiag.h"
#include "wide_gram.h"

namespace {

using namespace mfa;

constexpr int XW = 8;        // waves per workgroup
constexpr int XT = XW * 64;  // threads per workgroup
constexpr int XL_MAX_K = 1024;
// Waves per SIMD the solver is compiled for (both instantiated, bitwise the same results;
// mfa_eigen_xl_set_wpe): 2 = one 8-wave workgroup per CU without spills (~200 VGPRs), 4 = two
// workgroups per CU in 128 VGPRs (some scratch spills): more problems in flight to cover the
// tridiagonalisation's memory round trips.  0 (default) = 4 for the bias batches (25k problems:
// 193 -> 137 ms at K = 150, 351 -> 280 ms at K = 200), 2 for the eigh (a few hundred matrices:
// 2.48 -> 2.21 ms at K = 150; profiles/r06/xl/xl_bench.log).
int g_xl_wpe = 0;

// Timing-only phase ablations (A/B builds: mfa_eigen_xl_set_ablation): bit 1 skips the fused
// Householder pass, 2 the eigenvalues, 4 the twisted-factorisation vectors, 8 the back-transform.
// Results are meaningless with any bit set.  Production builds compile the checks out.
#if MFA_AB
__device__ int d_xl_abl = 0;
#define XL_SKIP(bit) ((d_xl_abl & (bit)) != 0)
#else
#define XL_SKIP(bit) false
#endif

__device__ __forceinline__ double xl_ext(double v, double* red, bool mx) {
  v = mx ? wave_max(v) : wave_min(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
  for (int w = 1; w < XW; ++w) s = mx ? fmax(s, red[w]) : fmin(s, red[w]);
  return s;
}

// Block sum in wave order WITHOUT the leading barrier of common.h's block_sum: for call sites
// where a barrier already separates this write of red[0..XW) from the previous reads of it.
__device__ __forceinline__ double xl_sum_nb(double v, double* red) {
  v = wave_total(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int w = 1; w < XW; ++w) s += red[w];
  return s;
}

// #{eigenvalues of T < x}, T scaled to unit norm (tb[i] = {d_i, e_{i-1}^2}): the leading
// minors' recurrence f_i = (d_{i-1} - x) f_{i-1} - e_{i-2}^2 f_{i-2}, rescaled by a power of
// two every 4 steps (exact), sign changes counted.
__device__ __forceinline__ int xl_sturm(const double2* tb, int K, double x) {
  double f2 = 1.0, f1 = tb[0].x - x;
  int cnt = f1 < 0.0;
  int i = 1;
  for (; i + 3 < K; i += 4) {
    const double2 t0 = tb[i], t1 = tb[i + 1], t2 = tb[i + 2], t3 = tb[i + 3];
    double f0 = fma(t0.x - x, f1, -t0.y * f2);
    cnt += (f0 < 0.0) != (f1 < 0.0);
    f2 = fma(t1.x - x, f0, -t1.y * f1);
    cnt += (f2 < 0.0) != (f0 < 0.0);
    f1 = fma(t2.x - x, f2, -t2.y * f0);
    cnt += (f1 < 0.0) != (f2 < 0.0);
    f0 = fma(t3.x - x, f1, -t3.y * f2);
    cnt += (f0 < 0.0) != (f1 < 0.0);
    f2 = f1;
    f1 = f0;
    int e;
    frexp(fmax(fabs(f1), fabs(f2)), &e);
    f1 = ldexp(f1, -e);
    f2 = ldexp(f2, -e);
  }
  for (; i < K; ++i) {
    const double2 t = tb[i];
    const double f0 = fma(t.x - x, f1, -t.y * f2);
    cnt += (f0 < 0.0) != (f1 < 0.0);
    f2 = f1;
    f1 = f0;
  }
  return cnt;
}

__host__ __device__ constexpr int xl_ld(int K) { return (K + 7) & ~7; }
__host__ __device__ constexpr int xl_ts(int K) { return ((K + 63) & ~63) < XT ? ((K + 63) & ~63) : XT; }
__host__ __device__ constexpr size_t xl_slot_doubles(int K) {
  return 2 * (size_t)K * xl_ld(K) + 2 * (size_t)K * xl_ts(K);
}
// wave partials of the tridiagonalisation [XW][K], reused by the back-transform (512 doubles of
// G / T per wave) and the Jacobi re-solve (round-robin order, rotations)
__host__ __device__ constexpr int xl_yp(int K) { return XW * K > 512 * XW ? XW * K : 512 * XW; }
constexpr size_t xl_lds_bytes(int K) { return (10 * (size_t)K + xl_yp(K) + 16) * sizeof(double); }

// Cyclic round-robin Jacobi of the symmetric S (global, row stride LD) with V <- V J (V starts
// at I): the eigh re-solve of a matrix whose tridiagonal eigenvectors failed the orthogonality
// test.  Rotation of pair (p, q), zeroing S_pq: J_pp = J_qq = c, J_pq = s, J_qp = -s.
__device__ void xl_jacobi(double* S, double* V, int K, int LD, int* idx, double* cs_c,
                          double* cs_s, double* red) {
  const int tid = threadIdx.x;
  const int Ke = K + (K & 1), np = Ke / 2;
  for (int k = tid; k < Ke; k += XT) idx[k] = k;
  __syncthreads();
  auto at = [&](int i, int j) -> double { return (i < K && j < K) ? S[(size_t)i * LD + j] : 0.0; };
  for (int sweep = 0; sweep < 40; ++sweep) {
    double nrot = 0.0;
    for (int round = 0; round < Ke - 1; ++round) {
      for (int i = tid; i < np; i += XT) {
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
      for (int e = tid; e < np * np; e += XT) {  // S <- J^T S J, one 2 x 2 pair block each
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
        if (p < K && r < K) S[(size_t)p * LD + r] = y00;
        if (p < K && t < K) S[(size_t)p * LD + t] = y01;
        if (q < K && r < K) S[(size_t)q * LD + r] = y10;
        if (q < K && t < K) S[(size_t)q * LD + t] = y11;
      }
      for (int e = tid; e < K * np; e += XT) {  // V <- V J
        const int r = e / np, i = e - r * np;
        const double c = cs_c[i], s = cs_s[i];
        if (s == 0.0) continue;
        int p = idx[i], q = idx[Ke - 1 - i];
        if (p > q) { const int x = p; p = q; q = x; }
        if (q >= K) continue;
        const double vp = V[(size_t)r * LD + p], vq = V[(size_t)r * LD + q];
        V[(size_t)r * LD + p] = c * vp - s * vq;
        V[(size_t)r * LD + q] = s * vp + c * vq;
      }
      __syncthreads();
      if (tid == 0) {  // round-robin: position 0 fixed, the others shift by one
        const int last = idx[Ke - 1];
        for (int k = Ke - 1; k > 1; --k) idx[k] = idx[k - 1];
        idx[1] = last;
      }
      __syncthreads();
    }
    if (block_sum(nrot, red) == 0.0) break;
  }
}

__device__ __forceinline__ void xl_wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Back-transform Y <- H_0 H_1 ... H_{K-3} Y of the wave's NU x 16 columns [c0, c0 + 16 NU) in
// compact-WY blocks of 16 reflectors (LAPACK dlarft, forward: H_s0 ... H_s0+15 = I - V T V^T,
// T upper triangular), last block first, on the fp64 matrix cores (v_mfma_f64_16x16x4f64):
//   G = V^T V and W = V^T Y share one pass over the rows (same A operand), T from G (lanes
//   0..15, wave-private LDS), W2 = T W straight from W's registers (the MFMA output layout of
//   W is the B-operand layout of the next product), Y -= V W2 tile by tile (16 rows x 16 cols,
//   Y loaded as the accumulator).  Y is read twice and written once per 16 reflectors instead
//   of read twice and written once per reflector.  Reflector s: v[s + 1] = 1, v[r] = Aw[s][r]
//   for r > s + 1.  16x16x4 f64 layouts: A lane l = A[l & 15][l >> 4], B lane l =
//   B[l >> 4][l & 15], register e of lane l = D[(l >> 4) + 4 e][l & 15].
template <int NU>
__device__ void xl_back_wy(const double* __restrict__ Aw, double* __restrict__ Y,
                           const double* tau, int K, int LD, int c0, double* wl, int lane) {
  const int hi = lane >> 4, lo = lane & 15;
  double* gl = wl;        // G [16][16]
  double* tl = wl + 256;  // T [16][16]
  auto vat = [&](int s, int r) -> double {  // reflector s at row r (0 outside)
    if (s > K - 3 || r >= K || r <= s) return 0.0;
    return r == s + 1 ? 1.0 : Aw[(size_t)s * LD + r];
  };
  const int nblk = (K - 2 + 15) / 16;
  for (int bk = nblk - 1; bk >= 0; --bk) {
    const int s0 = 16 * bk, r_lo = s0 + 1;
    f64x4g G = f64x4g{0.0, 0.0, 0.0, 0.0};
    f64x4g W[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) W[u] = f64x4g{0.0, 0.0, 0.0, 0.0};
    for (int r = r_lo; r < K; r += 4) {
      const int rr = r + hi;
      const double a = vat(s0 + lo, rr);
      G = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, G, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int c = c0 + 16 * u + lo;
        const double y = (rr < K && c < K) ? Y[(size_t)rr * LD + c] : 0.0;
        W[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, y, W[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) gl[(hi + 4 * e) * 16 + lo] = G[e];
    xl_wsync();
    // T[j][i] = -tau_i sum_{m = j}^{i - 1} T[j][m] G[m][i] (j < i), T[i][i] = tau_i
    for (int i = 0; i < 16; ++i) {
      if (lane < 16) {
        const double ti = s0 + i <= K - 3 ? tau[s0 + i] : 0.0;
        double acc = 0.0;
        for (int m = lane; m < i; ++m) acc = fma(tl[lane * 16 + m], gl[m * 16 + i], acc);
        tl[lane * 16 + i] = lane < i ? -ti * acc : (lane == i ? ti : 0.0);
      }
      xl_wsync();
    }
    f64x4g W2[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) W2[u] = f64x4g{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double ta = tl[lo * 16 + 4 * q + hi];
#pragma unroll
      for (int u = 0; u < NU; ++u) W2[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ta, W[u][q], W2[u], 0, 0, 0);
    }
    for (int r0 = r_lo; r0 < K; r0 += 16) {
      double va[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) va[q] = -vat(s0 + 4 * q + hi, r0 + lo);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int c = c0 + 16 * u + lo;
        f64x4g acc;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = r0 + hi + 4 * e;
          acc[e] = (r < K && c < K) ? Y[(size_t)r * LD + c] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[q], W2[u][q], acc, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = r0 + hi + 4 * e;
          if (r < K && c < K) Y[(size_t)r * LD + c] = acc[e];
        }
      }
    }
    xl_wsync();  // gl / tl reused by the next block
  }
}

// max |U^T U - I| of the K columns of U (row stride LD) on the fp64 matrix cores: the
// KT (KT + 1) / 2 upper 16 x 16 tiles of U^T U dealt round-robin to the waves; NaN -> +inf.
__device__ double xl_ortho_err(const double* U, int K, int LD, double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int KT = (K + 15) / 16, NT = KT * (KT + 1) / 2;
  double err = 0.0;
  for (int t = wv; t < NT; t += XW) {
    int ti = 0, tt = t;
    while (tt >= KT - ti) { tt -= KT - ti; ++ti; }
    const int tj = ti + tt;
    const int ca = 16 * ti + (lane & 15), cb = 16 * tj + (lane & 15);
    f64x4g acc = f64x4g{0.0, 0.0, 0.0, 0.0};
    for (int r0 = 0; r0 < K; r0 += 4) {
      const int r = r0 + (lane >> 4);
      const double a = (r < K && ca < K) ? U[(size_t)r * LD + ca] : 0.0;
      const double c = (r < K && cb < K) ? U[(size_t)r * LD + cb] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, c, acc, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 16 * ti + (lane >> 4) + 4 * e, j = 16 * tj + (lane & 15);
      if (i < K && j < K) {
        const double g = fabs(acc[e] - (i == j ? 1.0 : 0.0));
        err = (g > err || g != g) ? g : err;
      }
    }
  }
  return xl_ext(err != err ? INFINITY : err, red, true);
}

// C = op(A) B for K x K operands (op(A) = A^T if TA), 16 x 16 output tiles dealt to the waves,
// fp64 matrix cores; leading dimensions lda / ldb / ldc.  Caller brackets with barriers.
template <bool TA>
__device__ void xl_mm(const double* A, int lda, const double* B, int ldb, double* C, int ldc,
                      int K) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hi = lane >> 4, lo = lane & 15;
  const int KT = (K + 15) / 16;
  for (int t = wv; t < KT * KT; t += XW) {
    const int ti = t / KT, tj = t - ti * KT;
    const int i = 16 * ti + lo, j = 16 * tj + lo;
    f64x4g acc = f64x4g{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < K; k0 += 4) {
      const int k = k0 + hi;
      const double a = (i < K && k < K) ? (TA ? A[(size_t)k * lda + i] : A[(size_t)i * lda + k]) : 0.0;
      const double bb = (k < K && j < K) ? B[(size_t)k * ldb + j] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 16 * ti + hi + 4 * e;
      if (r < K && j < K) C[(size_t)r * ldc + j] = acc[e];
    }
  }
}

// EIG: problem b = matrix Ain[b] -> w[b] (descending), U[b] (U[:, k] = eigenvector k), flags[b]
// (1 = re-solved by the Jacobi; nullable).  !EIG: problem b = (date d = b / M, sim m = b % M),
// A = S C_z[m] S with S = diag(sqrt D0[d]) -> v[b][k] = sum_i D0[d][i] V[i][k]^2 / Lambda[k].
template <bool EIG, int WPE>
__global__ __launch_bounds__(XT) __attribute__((amdgpu_waves_per_eu(WPE))) void eig_xl_kernel(int B, int K, const double* __restrict__ Ain,
                                                    const double* __restrict__ D0,
                                                    const int* __restrict__ dvalid, int M,
                                                    const double* __restrict__ Cz, double tol,
                                                    double psd_tol,
                                                    double* __restrict__ wout,
                                                    double* __restrict__ out,
                                                    int* __restrict__ flags,
                                                    double* __restrict__ scratch) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int LD = xl_ld(K), TS = xl_ts(K);
  double2* tb = reinterpret_cast<double2*>(sm);  // {d_i, e_{i-1}^2}
  double* es = sm + 2 * K;                       // e_i (signed)
  double* tau = es + K;
  double* lam = tau + K;                         // sqrt D0 during the setup, then eigenvalues
  double* dd = lam + K;                          // D0 (bias)
  double* va = dd + K;
  double* vb = va + K;
  double* wp = vb + K;
  double* yr = wp + K;                           // row parts of y = A v (lower triangle)
  double* yp = yr + K;                           // [XW][K] column parts per wave (xl_yp doubles)
  double* red = yp + xl_yp(K);
  double* Aw = scratch + (size_t)blockIdx.x * xl_slot_doubles(K);
  double* Y = Aw + (size_t)K * LD;
  double* tw = Y + (size_t)K * LD;               // [2K][TS] twisted-factorisation pivots
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    __syncthreads();  // LDS of the previous problem
    // ---- working matrix ----
    bool fin = true;
    if (EIG) {
      const double* A = Ain + (size_t)b * K * K;
      for (int e = tid; e < K * K; e += XT) {
        const int i = e / K, j = e - i * K;
        const double a = 0.5 * (A[e] + A[(size_t)j * K + i]);
        fin = fin && __builtin_isfinite(a);
        if (j <= i) Aw[(size_t)i * LD + j] = a;  // the lower triangle is the working matrix
      }
    } else {
      const int d = b / M, m = b - d * M;
      fin = dvalid[d] != 0;
      for (int i = tid; i < K; i += XT) {
        const double x = D0[(size_t)d * K + i];
        dd[i] = x;
        lam[i] = sqrt(x);
      }
      __syncthreads();
      const double* C = Cz + (size_t)m * K * K;
      for (int e = tid; e < K * K; e += XT) {
        const int i = e / K, j = e - i * K;
        if (j <= i) Aw[(size_t)i * LD + j] = lam[i] * C[e] * lam[j];
      }
    }
    if (block_sum(fin ? 0.0 : 1.0, red) != 0.0) {
      if (EIG) {
        for (int k = tid; k < K; k += XT) wout[(size_t)b * K + k] = qnan();
        for (int e = tid; e < K * K; e += XT) out[(size_t)b * K * K + e] = qnan();
        if (tid == 0 && flags) flags[b] = 0;
      } else {
        for (int k = tid; k < K; k += XT) out[(size_t)b * K + k] = qnan();
      }
      continue;
    }
    __syncthreads();  // the finiteness sum's reads of red precede step 0's writes (xl_sum_nb)
    // ---- Householder tridiagonalisation, update of step s fused into the product of s + 1 ----
    double* vp = va;  // v of step s - 1 (pending update with wp)
    double* vc = vb;  // v of step s
    for (int s = 0; s + 2 < K; ++s) {
      const bool pend = s > 0;
      double sg = 0.0;
      for (int j = s + tid; j < K; j += XT) {  // column s, final after the pending update
        double a = Aw[(size_t)j * LD + s];
        if (pend) a = fma(-vp[s], wp[j], fma(-wp[s], vp[j], a));
        if (j == s) {
          tb[s].x = a;
        } else {
          vc[j] = a;
          if (j == s + 1) red[XW + 1] = a;  // alpha: vc[s + 1] becomes 1 below while slower
          if (j >= s + 2) sg = fma(a, a, sg);  // waves may still be reading
        }
      }
      // the previous step's last barrier follows its reads of red
      const double sigma = xl_sum_nb(sg, red);
      const double alpha = red[XW + 1];
      double ts = 0.0, beta = alpha, scal = 0.0;
      if (sigma != 0.0) {
        const double nrm = sqrt(fma(alpha, alpha, sigma));
        beta = alpha >= 0.0 ? -nrm : nrm;
        ts = (beta - alpha) / beta;
        scal = 1.0 / (alpha - beta);
      }
      if (tid == 0) {
        es[s] = beta;
        tau[s] = ts;
      }
      for (int j = s + 1 + tid; j < K; j += XT) {
        const double v = j == s + 1 ? 1.0 : vc[j] * scal;
        vc[j] = v;
        if (j >= s + 2) Aw[(size_t)s * LD + j] = v;  // reflector s, v_{s+1} = 1 implied
      }
      __syncthreads();
      if (!XL_SKIP(1)) {
        // Lower triangle only (half the traffic of the full square): the wave's rows
        // j = s + 1 + wv + XW q (q < nrw), columns s + 1 <= i <= j in batches of NC 64-column
        // chunks, streamed with the next batch's loads issued before the current batch's
        // updates are stored.  By symmetry y_i = sum_{j >= i} A_ji v_j (column part: lane i,
        // this wave's partial in yp[wv][i], wave-private) + sum_{i' < i} A_ii' v_i' (row part:
        // a wave total per row j, yr[j]).
        constexpr int NC = 4;
        const int n1 = K - s - 1;
        const int nrw = n1 > wv ? (n1 - wv + XW - 1) / XW : 0;
        double* ypw = yp + wv * K;
        for (int i = s + 1 + lane; i < K; i += 64) ypw[i] = 0.0;
        // the first NC chunks' per-column constants and column partials stay in registers for
        // the whole step (they do not depend on the row); chunks beyond (K > 257) use LDS
        double rv[NC], rw[NC], rc[NC], cacc[NC];
#pragma unroll
        for (int u = 0; u < NC; ++u) {
          const int i = s + 1 + 64 * u + lane;
          const bool ok = i < K;
          rv[u] = (ok && pend) ? vp[i] : 0.0;
          rw[u] = (ok && pend) ? wp[i] : 0.0;
          rc[u] = ok ? vc[i] : 0.0;
          cacc[u] = 0.0;
        }
        double cur[NC], nxt[NC];
        int q = 0, bt = 0;
#pragma unroll
        for (int u = 0; u < NC; ++u) {
          const int j = s + 1 + wv, i = s + 1 + 64 * u + lane;
          if (64 * u > wv) break;  // chunk u starts right of the diagonal of row s + 1 + wv
          cur[u] = (nrw > 0 && i <= j) ? Aw[(size_t)j * LD + i] : 0.0;
        }
        double rsum = 0.0;
        while (q < nrw) {
          const int j = s + 1 + wv + XW * q;
          const int nbt = (j - s - 1) / (64 * NC) + 1;
          int qn = q, bn = bt + 1;
          if (bn >= nbt) {
            qn = q + 1;
            bn = 0;
          }
          if (qn < nrw) {
            const int jn = s + 1 + wv + XW * qn;
#pragma unroll
            for (int u = 0; u < NC; ++u) {
              if (64 * (NC * bn + u) > jn - s - 1) break;  // past the diagonal: no load
              const int i = s + 1 + 64 * (NC * bn + u) + lane;
              nxt[u] = i <= jn ? Aw[(size_t)jn * LD + i] : 0.0;
            }
          }
          const double vj = vc[j], vpj = pend ? vp[j] : 0.0, wpj = pend ? wp[j] : 0.0;
#pragma unroll
          for (int u = 0; u < NC; ++u) {
            if (64 * (NC * bt + u) > j - s - 1) break;
            const int i = s + 1 + 64 * (NC * bt + u) + lane;
            if (i <= j) {
              double x = cur[u];
              if (bt == 0) {
                if (pend) {
                  x = fma(-vpj, rw[u], fma(-wpj, rv[u], x));
                  Aw[(size_t)j * LD + i] = x;
                }
                cacc[u] = fma(x, vj, cacc[u]);
                if (i < j) rsum = fma(x, rc[u], rsum);
              } else {
                if (pend) {
                  x = fma(-vpj, wp[i], fma(-wpj, vp[i], x));
                  Aw[(size_t)j * LD + i] = x;
                }
                ypw[i] = fma(x, vj, ypw[i]);
                if (i < j) rsum = fma(x, vc[i], rsum);
              }
            }
          }
          if (bn == 0) {  // row j done: its row part
            const double t = wave_total(rsum);
            if (lane == 0) yr[j] = t;
            rsum = 0.0;
          }
#pragma unroll
          for (int u = 0; u < NC; ++u) cur[u] = nxt[u];
          q = qn;
          bt = bn;
        }
#pragma unroll
        for (int u = 0; u < NC; ++u) {
          const int i = s + 1 + 64 * u + lane;
          if (i < K) ypw[i] = cacc[u];  // chunks 0..NC-1 were never accumulated in LDS
        }
      }
      __syncthreads();
      double dp = 0.0;
      for (int i = s + 1 + tid; i < K; i += XT) {
        double y = yr[i];
        for (int w = 0; w < XW; ++w) y += yp[w * K + i];
        const double p = ts * y;
        wp[i] = p;
        dp = fma(p, vc[i], dp);
      }
      // red was last read before the barrier that follows the v broadcast
      const double hc = 0.5 * ts * xl_sum_nb(dp, red);
      for (int i = s + 1 + tid; i < K; i += XT) wp[i] = fma(-hc, vc[i], wp[i]);
      __syncthreads();
      double* t = vp;
      vp = vc;
      vc = t;
    }
    if (tid == 0) {  // the last 2 x 2 block with the pending update of step K - 3
      const int p = K - 2, q = K - 1;
      double a00 = Aw[(size_t)p * LD + p], a01 = Aw[(size_t)q * LD + p], a11 = Aw[(size_t)q * LD + q];
      if (K >= 3) {
        a00 -= 2.0 * vp[p] * wp[p];
        a01 -= vp[p] * wp[q] + wp[p] * vp[q];
        a11 -= 2.0 * vp[q] * wp[q];
      }
      tb[p].x = a00;
      tb[q].x = a11;
      es[p] = a01;
      es[q] = 0.0;
      tau[p] = 0.0;
      tau[q] = 0.0;
    }
    __syncthreads();
    // ---- scale T to unit norm (Gershgorin) ----
    double lo = INFINITY, hi = -INFINITY;
    for (int i = tid; i < K; i += XT) {
      const double r = (i > 0 ? fabs(es[i - 1]) : 0.0) + fabs(es[i]);
      lo = fmin(lo, tb[i].x - r);
      hi = fmax(hi, tb[i].x + r);
    }
    lo = xl_ext(lo, red, false);
    hi = xl_ext(hi, red, true);
    double tn = fmax(fabs(lo), fabs(hi));
    if (!(tn > 0.0) || !__builtin_isfinite(tn)) tn = 1.0;
    const double is = 1.0 / tn;
    for (int i = tid; i < K; i += XT) {
      const double e0 = i > 0 ? es[i - 1] * is : 0.0;
      tb[i] = double2{tb[i].x * is, e0 * e0};
    }
    __syncthreads();
    for (int i = tid; i < K; i += XT) es[i] *= is;
    lo = lo * is - 1e-15;
    hi = hi * is + 1e-15;
    // ---- eigenvalues (descending: lane k finds ascending index K - 1 - k) ----
    for (int k = tid; k < K; k += XT) {
      if (XL_SKIP(2)) {
        lam[k] = tb[k].x;
        continue;
      }
      const int ix = K - 1 - k;
      double a = lo, c = hi;
      for (int it = 0; it < 128; ++it) {
        if (!(c - a > fmax(2.3e-16, 4.5e-16 * fmax(fabs(a), fabs(c))))) break;
        const double mid = 0.5 * (a + c);
        if (xl_sturm(tb, K, mid) > ix) c = mid; else a = mid;
      }
      lam[k] = 0.5 * (a + c);
    }
    __syncthreads();
    // ---- eigenvectors of T by twisted factorisation ----
    const double pivmin = 1e-290;
    for (int k = tid; k < K && !XL_SKIP(4); k += XT) {
      const double x = lam[k];
      double* tp = tw + tid;
      double* tm = tw + (size_t)K * TS + tid;
      double dp = guard_pivot(tb[0].x - x, pivmin);
      tp[0] = dp;
      for (int i = 1; i < K; ++i) {
        dp = guard_pivot((tb[i].x - x) - tb[i].y / dp, pivmin);
        tp[(size_t)i * TS] = dp;
      }
      double dm = guard_pivot(tb[K - 1].x - x, pivmin);
      tm[(size_t)(K - 1) * TS] = dm;
      double best = fabs(dp);
      int r = K - 1;
      for (int i = K - 2; i >= 0; --i) {
        const double di = tb[i].x - x;
        dm = guard_pivot(di - tb[i + 1].y / dm, pivmin);
        tm[(size_t)i * TS] = dm;
        const double g = fabs(tp[(size_t)i * TS] + dm - di);
        if (g < best) {
          best = g;
          r = i;
        }
      }
      double z = 1.0, nrm = 1.0;
      Y[(size_t)r * LD + k] = 1.0;
      for (int i = r - 1; i >= 0; --i) {
        z = -(es[i] / tp[(size_t)i * TS]) * z;
        Y[(size_t)i * LD + k] = z;
        nrm = fma(z, z, nrm);
      }
      z = 1.0;
      for (int i = r + 1; i < K; ++i) {
        z = -(es[i - 1] / tm[(size_t)i * TS]) * z;
        Y[(size_t)i * LD + k] = z;
        nrm = fma(z, z, nrm);
      }
      const double sc = 1.0 / sqrt(nrm);
      for (int i = 0; i < K; ++i) Y[(size_t)i * LD + k] *= sc;
    }
    __syncthreads();
    // ---- eigh: orthogonality of the tridiagonal eigenvectors; Jacobi re-solve on failure ----
    if (EIG) {
      const double err = xl_ortho_err(Y, K, LD, red);
      // psd_tol >= 0 (the eigen adjustment): a matrix with an eigenvalue below -psd_tol lambda_max
      // is an invalid date whose eigenvectors nobody reads -- flagged 2, not re-solved
      const bool need = psd_tol < 0.0 || lam[K - 1] >= -psd_tol * fabs(lam[0]);
      if (!(err <= tol) && !need) {
        if (tid == 0 && flags) flags[b] = 2;
      } else if (!(err <= tol)) {
        // Warm start: U0 = Q Y (back-transform), orthonormalised by Newton-Schulz steps
        // U <- U (3 I - U^T U) / 2 (quadratic once |U^T U - I| < 1: the small-gap case, where
        // the twisted vectors are nearly orthonormal); then the Jacobi only has to rotate
        // S = U0^T A U0 inside its clusters, and U = U0 V.  Exactly repeated eigenvalues give
        // (nearly) parallel vectors the iteration cannot separate: cold Jacobi on A, V = I.
        const double* A = Ain + (size_t)b * K * K;
        double* T2 = tw;  // one K x LD matrix (tw holds 2K x TS >= K x LD doubles)
        for (int c0 = 32 * wv; c0 < K; c0 += 32 * XW)
          xl_back_wy<2>(Aw, Y, tau, K, LD, c0, yp + 512 * wv, lane);
        __syncthreads();
        double e2 = err;
        for (int it = 0; it < 4 && e2 < 0.5; ++it) {
          xl_mm<true>(Y, LD, Y, LD, Aw, LD, K);       // G = U^T U
          __syncthreads();
          xl_mm<false>(Y, LD, Aw, LD, T2, LD, K);      // H = U G
          __syncthreads();
          for (int e = tid; e < K * K; e += XT) {
            const int i = e / K, j = e - i * K;
            Y[(size_t)i * LD + j] = 1.5 * Y[(size_t)i * LD + j] - 0.5 * T2[(size_t)i * LD + j];
          }
          __syncthreads();
          e2 = xl_ortho_err(Y, K, LD, red);
          if (e2 <= 1e-14) break;
        }
        const bool warm = e2 <= 1e-14;
        if (warm) {
          xl_mm<false>(A, K, Y, LD, T2, LD, K);        // A U0 (A symmetric up to rounding)
          __syncthreads();
          xl_mm<true>(Y, LD, T2, LD, Aw, LD, K);       // S = U0^T A U0
          __syncthreads();
          for (int e = tid; e < K * K; e += XT) {      // U0 -> T2, V = I
            const int i = e / K, j = e - i * K;
            T2[(size_t)i * LD + j] = Y[(size_t)i * LD + j];
            Y[(size_t)i * LD + j] = i == j ? 1.0 : 0.0;
          }
        } else {
          for (int e = tid; e < K * K; e += XT) {
            const int i = e / K, j = e - i * K;
            Aw[(size_t)i * LD + j] = 0.5 * (A[e] + A[(size_t)j * K + i]);
            Y[(size_t)i * LD + j] = i == j ? 1.0 : 0.0;
          }
        }
        __syncthreads();
        int* idx = reinterpret_cast<int*>(yp);
        double* cs_c = yp + (K + 2) / 2 + 2;
        double* cs_s = cs_c + K / 2 + 2;
        xl_jacobi(Aw, Y, K, LD, idx, cs_c, cs_s, red);
        __syncthreads();
        if (warm) {  // eigenvalues to LDS, then U = U0 V into Aw, read back as Y below
          for (int k = tid; k < K; k += XT) lam[k] = Aw[(size_t)k * LD + k];
          __syncthreads();
          xl_mm<false>(T2, LD, Y, LD, Aw, LD, K);
          __syncthreads();
          for (int e = tid; e < K * K; e += XT) {
            const int i = e / K, j = e - i * K;
            Y[(size_t)i * LD + j] = Aw[(size_t)i * LD + j];
          }
          for (int k = tid; k < K; k += XT) Aw[(size_t)k * LD + k] = lam[k];
          __syncthreads();
        }
        for (int k = tid; k < K; k += XT) {  // descending rank of diag entry k (ties by index)
          const double dk = Aw[(size_t)k * LD + k];
          int rank = 0;
          for (int j = 0; j < K; ++j) {
            const double dj = Aw[(size_t)j * LD + j];
            rank += (dj > dk) || (dj == dk && j < k);
          }
          idx[k] = rank;
          wout[(size_t)b * K + rank] = dk;
        }
        __syncthreads();
        double* Ub = out + (size_t)b * K * K;
        for (int e = tid; e < K * K; e += XT) {
          const int r = e / K, k = e - r * K;
          Ub[(size_t)r * K + idx[k]] = Y[(size_t)r * LD + k];
        }
        if (tid == 0 && flags) flags[b] = 1;
        continue;
      } else if (tid == 0 && flags) {
        flags[b] = 0;
      }
    }
    // ---- back-transform Y <- H_0 ... H_{K-3} Y: waves own 32-column chunks ----
    for (int c0 = 32 * wv; c0 < K && !XL_SKIP(8); c0 += 32 * XW)
      xl_back_wy<2>(Aw, Y, tau, K, LD, c0, yp + 512 * wv, lane);
    __syncthreads();
    // ---- outputs: lane k owns column k ----
    for (int k = tid; k < K; k += XT) {
      const double lk = lam[k] * tn;
      if (EIG) {
        wout[(size_t)b * K + k] = lk;
        double* Ub = out + (size_t)b * K * K;
        for (int r = 0; r < K; ++r) Ub[(size_t)r * K + k] = Y[(size_t)r * LD + k];
      } else {
        double sm0 = 0.0;
        for (int r = 0; r < K; ++r) {
          const double y = Y[(size_t)r * LD + k];
          sm0 = fma(dd[r] * y, y, sm0);
        }
        out[(size_t)b * K + k] = sm0 / lk;
      }
    }
  }
}

// S[d][k] += sum over m < M of v[d * M + m][k] (sim order: deterministic)
__global__ __launch_bounds__(256) void xl_bias_sum_kernel(const double* __restrict__ v, int K, int M,
                                                          double* __restrict__ S) {
  const int d = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += 256) {
    double s = 0.0;
    for (int m = 0; m < M; ++m) s += v[((size_t)d * M + m) * K + k];
    S[(size_t)d * K + k] += s;
  }
}

template <bool EIG, int WPE>
int xl_prepare() {
  return (int)hipFuncSetAttribute((const void*)eig_xl_kernel<EIG, WPE>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)xl_lds_bytes(XL_MAX_K));
}

// Persistent grid: as many workgroups as can be resident at once (a slot beyond that would start
// only after a resident one has finished its whole share of the batch), at most B.
template <bool EIG, int WPE>
int xl_slots(int B, int K) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  (void)xl_prepare<EIG, WPE>();
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, eig_xl_kernel<EIG, WPE>, XT, xl_lds_bytes(K)) !=
          hipSuccess || per <= 0)
    per = 1;
  return B < per * cus ? B : per * cus;
}


}  // namespace

// Scratch doubles of the XL solvers for a batch of B problems of order K (144 < K <= 1024).
MFA_API size_t mfa_eigen_xl_ws_doubles(int B, int K) {
  if (B <= 0 || K < 3 || K > XL_MAX_K) return 0;
  int n = xl_slots<true, 2>(B, K);
  n = n > xl_slots<false, 2>(B, K) ? n : xl_slots<false, 2>(B, K);
  n = n > xl_slots<true, 4>(B, K) ? n : xl_slots<true, 4>(B, K);
  n = n > xl_slots<false, 4>(B, K) ? n : xl_slots<false, 4>(B, K);
  return (size_t)n * xl_slot_doubles(K);
}

// Batched eigendecomposition of symmetric [B][K][K] fp64 matrices (3 <= K <= 1024): w [B][K]
// descending, U [B][K][K] with U[:, k] = eigenvector k, NaN for non-finite inputs; a matrix
// whose tridiagonal eigenvectors miss max |Y^T Y - I| <= tol is re-solved by the Jacobi
// (fixed[b] = 1; nullable) -- with psd_tol >= 0 only if its smallest eigenvalue is >= -psd_tol
// lambda_max (else fixed[b] = 2: an invalid date of the eigen adjustment; psd_tol < 0 = always).
// ws: mfa_eigen_xl_ws_doubles(B, K).
MFA_API int mfa_eigh_xl(const double* A, int B, int K, double tol, double psd_tol, double* w,
                        double* U, int* fixed, double* ws, void* stream) {
  if (B <= 0) return 0;
  if (K < 3 || K > XL_MAX_K || ws == nullptr) return (int)hipErrorInvalidValue;
#define MFA_XL_EIG(W)                                                                          \
  {                                                                                            \
    if (int e = xl_prepare<true, W>()) return e;                                               \
    hipLaunchKernelGGL((eig_xl_kernel<true, W>), dim3(xl_slots<true, W>(B, K)), dim3(XT),      \
                       xl_lds_bytes(K), (hipStream_t)stream, B, K, A, (const double*)nullptr,  \
                       (const int*)nullptr, 1, (const double*)nullptr, tol, psd_tol, w, U, fixed, ws);   \
  }
  if (g_xl_wpe == 4) MFA_XL_EIG(4) else MFA_XL_EIG(2)  // auto: 2
#undef MFA_XL_EIG
  return (int)hipGetLastError();
}

// Bias statistic, 3 <= K <= 1024: S[d][k] += sum over this call's M sims of v_m[d][k] (A =
// S C_z[m] S per (date, sim)); w [D][K] the clamped F0 eigenvalues, dvalid [D] (0 -> NaN),
// vws: D * M * K doubles, ws: mfa_eigen_xl_ws_doubles(D * M, K).
MFA_API int mfa_eigen_bias_accumulate_xl(const double* w, const int* dvalid, int D, int K, int M,
                                         const double* Cz, double* vws, double* ws, double* S,
                                         void* stream) {
  if (D <= 0 || M <= 0) return 0;
  if (K < 3 || K > XL_MAX_K || ws == nullptr || vws == nullptr) return (int)hipErrorInvalidValue;
  const int B = D * M;
  hipStream_t s = (hipStream_t)stream;
#define MFA_XL_BIAS(W)                                                                         \
  {                                                                                            \
    if (int e = xl_prepare<false, W>()) return e;                                              \
    hipLaunchKernelGGL((eig_xl_kernel<false, W>), dim3(xl_slots<false, W>(B, K)), dim3(XT),    \
                       xl_lds_bytes(K), s, B, K, (const double*)nullptr, w, dvalid, M, Cz, 0.0, -1.0,\
                       (double*)nullptr, vws, (int*)nullptr, ws);                              \
  }
  if (g_xl_wpe == 2) MFA_XL_BIAS(2) else MFA_XL_BIAS(4)  // auto: 4
#undef MFA_XL_BIAS
  hipLaunchKernelGGL(xl_bias_sum_kernel, dim3(D), dim3(256), 0, s, vws, K, M, S);
  return (int)hipGetLastError();
}

// Waves per SIMD of the XL solver for the next calls: 0 (auto, default), 2 or 4.
MFA_API int mfa_eigen_xl_set_wpe(int w) {
  if (w != 0 && w != 2 && w != 4) return (int)hipErrorInvalidValue;
  g_xl_wpe = w;
  return 0;
}

// Timing-only phase ablation bits of the XL solver (A/B builds; hipErrorInvalidValue otherwise).
MFA_API int mfa_eigen_xl_set_ablation(int bits) {
#if MFA_AB
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(d_xl_abl), &bits, sizeof(int));
#else
  return bits == 0 ? 0 : (int)hipErrorInvalidValue;
#endif
}
