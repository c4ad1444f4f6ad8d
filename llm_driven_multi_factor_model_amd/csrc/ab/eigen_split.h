// A/B-only eigen kernels / launchers (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build
// --ab).  Included by eigen.hip at the position they held in it; the production library never
// compiles them.  Their measurements against the production solvers: profiles/ (r01-r05).
#pragma once
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

