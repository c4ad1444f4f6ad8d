// A/B-only eigen kernels / launchers (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build
// --ab).  Included by eigen.hip at the position they held in it; the production library never
// compiles them.  Their measurements against the production solvers: profiles/ (r01-r05).
#pragma once
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
