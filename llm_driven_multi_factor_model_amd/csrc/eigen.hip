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
//   * eigh: one wave per matrix, parallel cyclic Jacobi (round-robin tournament ordering,
//     K/2 disjoint rotations per round) with A and V resident in LDS, fp64 throughout;
//   * grid (date, sim) for the simulations, per-(date, sim) bias vectors reduced by a
//     separate deterministic pass (no float atomics -> bitwise reproducible).
#include "common.h"

namespace {

using namespace mfa;

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

// ---------------- one-wave parallel cyclic Jacobi ----------------
// A: K x K symmetric in LDS (row stride lda), overwritten (diag -> eigenvalues).
// V: K x K in LDS (stride lda), set to the eigenvectors (columns).  rot: 4*64 doubles scratch.
__device__ int jacobi_wave(double* A, double* V, int K, int lda, double* rot, int max_sweeps,
                           double tol) {
  const int lane = threadIdx.x & 63;
  const int Ke = K + (K & 1);
  const int npair = Ke / 2;
  for (int e = lane; e < K * K; e += 64) V[(e / K) * lda + e % K] = (e / K == e % K) ? 1.0 : 0.0;
  wsync();
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    // convergence test: off-diagonal mass vs diagonal mass
    double off = 0.0, dg = 0.0;
    for (int e = lane; e < K * K; e += 64) {
      const int i = e / K, j = e % K;
      const double a = A[i * lda + j];
      if (i == j) dg = fma(a, a, dg);
      else off = fma(a, a, off);
    }
    off = wave_sum(off);
    dg = wave_sum(dg);
    if (off <= tol * tol * dg || off == 0.0) break;
    for (int r = 0; r < Ke - 1; ++r) {
      if (lane < npair) {  // rotation of pair `lane` in round r (circle method)
        int p, q;
        if (lane == 0) { p = 0; q = 1 + r % (Ke - 1); }
        else {
          p = 1 + (r + lane) % (Ke - 1);
          q = 1 + (r - lane + (Ke - 1)) % (Ke - 1);
        }
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        if (q < K) {
          const double apq = A[p * lda + q];
          const double app = A[p * lda + p], aqq = A[q * lda + q];
          if (fabs(apq) > 1e-300 && fabs(apq) > 1e-18 * sqrt(fabs(app * aqq))) {
            const double th = (aqq - app) / (2.0 * apq);
            const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
            c = 1.0 / sqrt(fma(t, t, 1.0));
            s = t * c;
          }
        }
        rot[lane * 4 + 0] = c;
        rot[lane * 4 + 1] = s;
        rot[lane * 4 + 2] = (double)p;
        rot[lane * 4 + 3] = (double)(q < K ? q : -1);
      }
      wsync();
      // rows: A <- J^T A
      for (int it = lane; it < npair * K; it += 64) {
        const int t = it / K, j = it % K;
        const int q = (int)rot[t * 4 + 3];
        if (q < 0) continue;
        const int p = (int)rot[t * 4 + 2];
        const double c = rot[t * 4 + 0], s = rot[t * 4 + 1];
        const double ap = A[p * lda + j], aq = A[q * lda + j];
        A[p * lda + j] = c * ap - s * aq;
        A[q * lda + j] = s * ap + c * aq;
      }
      wsync();
      // columns: A <- A J ; V <- V J
      for (int it = lane; it < npair * K; it += 64) {
        const int t = it / K, j = it % K;
        const int q = (int)rot[t * 4 + 3];
        if (q < 0) continue;
        const int p = (int)rot[t * 4 + 2];
        const double c = rot[t * 4 + 0], s = rot[t * 4 + 1];
        const double ap = A[j * lda + p], aq = A[j * lda + q];
        A[j * lda + p] = c * ap - s * aq;
        A[j * lda + q] = s * ap + c * aq;
        const double vp = V[j * lda + p], vq = V[j * lda + q];
        V[j * lda + p] = c * vp - s * vq;
        V[j * lda + q] = s * vp + c * vq;
      }
      wsync();
    }
  }
  return sweep;
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
                                                    double* __restrict__ Cz) {
  const int m = blockIdx.x, lane = threadIdx.x;
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
  double* C = Cz + (size_t)m * K * K;
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

// Per (date, sim): C_b = S C_z,m S (S = diag sqrt D0, eigen order of F0), eigh, bias vector
// vout[d][m][k] = sum_l V[l,k]^2 D0[l] / Lambda[k]   (both spectra sorted descending)
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
  const int lda = K + 1;
  double* A = sm;
  double* V = A + K * lda;
  double* rot = V + K * lda;
  double* dd = rot + 4 * 64;
  int* perm = (int*)(dd + 64);
  const double* d0 = D0 + (size_t)d * K;
  for (int k = lane; k < K; k += 64) dd[k] = d0[k];
  wsync();
  const double* c = Cz + (size_t)m * K * K;
  for (int e = lane; e < K * K; e += 64) {
    const int i = e / K, j = e % K;
    A[i * lda + j] = sqrt(dd[i]) * c[e] * sqrt(dd[j]);
  }
  wsync();
  jacobi_wave(A, V, K, lda, rot, max_sweeps, tol);
  sort_desc(A, K, lda, perm);
  for (int k = lane; k < K; k += 64) {
    const int pk = perm[k];
    double num = 0.0;
    for (int l = 0; l < K; ++l) {
      const double v = V[l * lda + pk];
      num = fma(v * v, dd[l], num);
    }
    vo[k] = num / A[pk * lda + pk];
  }
}

// finalize: v = sqrt(mean_m v_m); v = a (v - 1) + 1; F^ = U0 diag(v^2 D0) U0^T.  Grid (D).
__global__ __launch_bounds__(256) void eigen_finalize_kernel(const double* __restrict__ vin,
                                                             const double* __restrict__ D0,
                                                             const double* __restrict__ U0,
                                                             const int* __restrict__ dvalid,
                                                             int K, int M, double scale,
                                                             double* __restrict__ Fout,
                                                             double* __restrict__ vbias) {
  __shared__ double g[64];
  const int d = blockIdx.x, tid = threadIdx.x;
  const bool ok = dvalid[d] != 0;
  for (int k = tid; k < K; k += blockDim.x) {
    double s = 0.0;
    for (int m = 0; m < M; ++m) s += vin[((size_t)d * M + m) * K + k];
    double v = sqrt(s / M);
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

size_t eigh_lds(int K) { return ((size_t)2 * K * (K + 1) + 4 * 64 + 64) * sizeof(double) + 64 * sizeof(int); }

}  // namespace

MFA_API int mfa_eigh_batched(const double* A, int B, int K, int max_sweeps, double tol, double* w,
                             double* U, int* sweeps, void* stream) {
  if (B <= 0) return 0;
  if (K < 1 || K > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(eigh_kernel, dim3(B), dim3(64), eigh_lds(K), (hipStream_t)stream, A, K,
                     max_sweeps, tol, w, U, sweeps);
  return (int)hipGetLastError();
}

MFA_API int mfa_mc_cov(int M, int K, int T, unsigned long long seed, double* Cz, void* stream) {
  if (M <= 0) return 0;
  if (K < 1 || K > 64 || T < 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mc_cov_kernel, dim3(M), dim3(64), 0, (hipStream_t)stream, K, T, seed, Cz);
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
  hipLaunchKernelGGL(mc_bias_kernel, dim3(D * M), dim3(64), eigh_lds(K), s, D0, K, M, Cz, dvalid,
                     max_sweeps, tol, ws);
  hipLaunchKernelGGL(eigen_finalize_kernel, dim3(D), dim3(256), 0, s, ws, D0, U0, dvalid, K, M,
                     scale, Fout, vbias);
  return (int)hipGetLastError();
}
