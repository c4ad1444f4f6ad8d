// One-wave parallel cyclic Jacobi eigensolver for small symmetric fp64 matrices in LDS.
// Shared by the batched eigh / eigen-adjustment kernels (eigen.hip) and the pseudo-inverse
// refinement of near-singular cross-sections (xs_wls_impl.h).
#pragma once
#include "common.h"

namespace mfa {

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------- one-wave parallel cyclic Jacobi ----------------
// A: K x K symmetric in LDS (row stride lda), overwritten (diag -> eigenvalues).
// V: K x K in LDS (stride lda), set to the eigenvectors (columns).  rot: 4*64 doubles scratch.
__device__ inline int jacobi_wave(double* A, double* V, int K, int lda, double* rot, int max_sweeps,
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

}  // namespace mfa
