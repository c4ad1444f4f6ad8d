// A/B-only eigen kernels / launchers (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build
// --ab).  Included by eigen.hip at the position they held in it; the production library never
// compiles them.  Their measurements against the production solvers: profiles/ (r01-r05).
#pragma once
// ---------------- Householder-tridiagonal bias solver (bias mode 3) ----------------
// Per (date, sim) the same output as mc_bias_kernel, v[k] = V[:,k]^T D0 V[:,k] / Lambda[k]
// (descending), from one O(K^3) reduction instead of ~6 Jacobi sweeps of 2 LDS passes each:
//   1. tridiagonalise A = S C_z S with K-2 Householder reflections H_s = I - tau_s u_s u_s^T:
//      lane i owns row i (LDS, odd stride: conflict-free row-per-lane reads), p = tau A u,
//      w = p - (tau/2)(u^T p) u, A -= u w^T + w u^T on the trailing block; u_s is kept,
//      zero-padded to KP, in row s (that row is finished once its column is reduced);
//   2. lane k finds the k-th largest eigenvalue of T by count-guided Laguerre iteration on
//      det(T - x I) (f'/f and its derivative from the LDL^T pivot recurrence), bracketed by
//      the pivots' Sturm count, started from the k-th largest diagonal entry of A (C_b is
//      close to diagonal) and with the first brackets shared between all lanes;
//   3. eigenvector of T by the twisted factorisation at that eigenvalue (forward / backward
//      pivots, twist at min |gamma|), in registers;
//   4. y = H_0 ... H_{K-3} z (u_s broadcast from LDS) and v = sum_l D0[l] y_l^2 / lambda.
// Everything stays fp64; the outputs are sorted by construction (lane k = rank k).
// ABL: timing-only ablations (bias modes 41..47, KP = 44): 1 = no Laguerre iterations,
// 2 = no eigenvector / back-transform, 4 = no tridiagonalisation, 8 = setup only (mode 48),
// 16 = setup + tridiagonalisation only (mode 56); outputs meaningless
#ifndef MFA_TRI_WPE
#define MFA_TRI_WPE 1
#endif
template <int KP, int ABL = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MFA_TRI_WPE))) void mc_bias_tri_kernel(const double* __restrict__ D0, int K, int M,
                                                         const double* __restrict__ Cz,
                                                         const int* __restrict__ dvalid,
                                                         double* __restrict__ vout) {
  extern __shared__ double sm[];
  constexpr int LD = KP + 1;  // staging stride of C_z (odd: row-per-lane ds_read_b64 conflict-free)
  constexpr int LU = KP;      // reflector rows (16-B aligned: broadcast ds_read_b128 pairs)
  const int d = blockIdx.x / M, m = blockIdx.x % M, lane = threadIdx.x;
  double* vo = vout + ((size_t)d * M + m) * K;
  if (!dvalid[d]) {
    for (int k = lane; k < K; k += 64) vo[k] = qnan();
    return;
  }
  double* A = sm;                          // [K][LD]: row s <- reflector u_s (zero-padded)
  double* ub = A + (((size_t)K * LD + 1) & ~(size_t)1);  // [64] broadcast u (16-B aligned)
  double* wb = ub + 64;                    // [64] broadcast w
  double2* tb = (double2*)(wb + 64);       // [64] {alpha_i, beta_{i-1}^2}
  double* be = (double*)(tb + 64);         // [64] beta_i
  double* ta = be + 64;                    // [64] tau_s
  double* dd = ta + 64;                    // [64] sqrt(D0)
  double* gs = dd + 64;                    // [64] diagonal of A, descending
  const double* d0 = D0 + (size_t)d * K;
  dd[lane] = lane < K ? sqrt(fmax(d0[lane], 0.0)) : 0.0;
  lds_order();
  // C_z (shared by every date of sim m, L2-resident) staged coalesced into LDS, then lane i
  // keeps row i of A = S C_z S in registers (static indices; padding columns zero)
  const double* c = Cz + (size_t)m * K * K;
  for (int e = lane; e < K * K; e += 64) {
    const int i = e / K;
    A[i * LD + (e - i * K)] = c[e];
  }
  lds_order();
  double a[KP];
  {
    const int i = lane < K ? lane : 0;
    const double di = lane < K ? dd[i] : 0.0;
#pragma unroll
    for (int j = 0; j < KP; ++j) a[j] = j < K ? di * A[i * LD + j] * dd[j] : 0.0;
  }
  if (lane < K) {  // descending rank of the diagonal (ties by index): initial eigenvalue guesses
    const double g = dd[lane] * A[lane * LD + lane] * dd[lane];
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const double h = dd[j] * A[j * LD + j] * dd[j];
      rank += (h > g) || (h == g && j < lane);
    }
    gs[rank] = g;
  }
  lds_order();  // the staging area becomes the reflector store (stride LU)
  if constexpr ((ABL & 8) != 0) {  // timing: setup only
    if (lane < K) vo[lane] = a[lane % KP] + gs[lane];
    return;
  }
  // ---- 1. Householder tridiagonalisation (rows in registers) ----
  // Step s takes column s from each lane's own row (x_i = A[i][s], a static select within the
  // step group), forms u_s, p = tau A u, w = p - (tau/2)(u^T p) u and updates its own row
  // a -= u_i w + w_i u with u, w broadcast as 16-B LDS pairs.  Columns j < 8 floor(s / 8) are
  // finished, so each group of 8 steps runs a static column range [J0, KP): ~35 % fewer FMAs.
  auto steps = [&](auto J0c, int s_begin) {
    constexpr int J0 = decltype(J0c)::value;
    for (int s = s_begin; s < s_begin + 8 && s + 2 < K; ++s) {
      // column s of the (symmetric) matrix is each lane's own a[s]: select it from the group's
      // 8 static candidates (publishing row s through LDS cost ~22 single-lane 16-B stores per
      // step, each paying the whole wave's VGPR transfer: the phase's LDS-array time)
      // (each candidate goes through an empty asm: without it the compiler turns the select
      // chain into a dynamically indexed load, which demotes the whole row to scratch memory
      // and re-stores it after every step)
      double xs = a[J0];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (J0 + k < KP) {
          double t = a[J0 + k];
          asm volatile("" : "+v"(t));
          xs = s == J0 + k ? t : xs;
        }
      const bool act = lane > s && lane < K;
      const double x = act ? xs : 0.0;
      const double x0 = readlane(xs, s + 1);
      const double sig = wave_total(lane > s + 1 && lane < K ? x * x : 0.0);
      const double alpha = readlane(xs, s);
      double u = 0.0, tau = 0.0, beta = x0;
      if (sig != 0.0) {
        const double nrm = sqrt(fma(x0, x0, sig));
        beta = x0 >= 0.0 ? -nrm : nrm;
        tau = 1.0 / (nrm * (nrm + fabs(x0)));
        u = act ? (lane == s + 1 ? x0 - beta : x) : 0.0;
      }
      ub[lane] = u;
      if (lane < KP) A[s * LU + lane] = u;  // u_s, zero outside (s, K)
      if (lane == 0) {
        tb[s] = double2{alpha, s > 0 ? be[s - 1] * be[s - 1] : 0.0};
        be[s] = beta;
        ta[s] = tau;
      }
      lds_order();
      if (tau != 0.0) {
        double p0 = 0.0, p1 = 0.0;
#pragma unroll
        for (int j = J0; j < KP; j += 2) {
          const double2 uu = *(const double2*)(ub + j);
          p0 = fma(a[j], uu.x, p0);
          p1 = fma(a[j + 1], uu.y, p1);
        }
        const double p = act ? tau * (p0 + p1) : 0.0;
        const double kk = 0.5 * tau * wave_total(u * p);
        const double w = p - kk * u;
        wb[lane] = w;
        lds_order();
        if (act) {
#pragma unroll
          for (int j = J0; j < KP; j += 2) {
            const double2 ww = *(const double2*)(wb + j), uu = *(const double2*)(ub + j);
            a[j] -= fma(u, ww.x, w * uu.x);
            a[j + 1] -= fma(u, ww.y, w * uu.y);
          }
        }
      }
      lds_order();
    }
  };
  if constexpr ((ABL & 4) != 0) {
    if (lane < K) {
      tb[lane] = double2{gs[lane], 0.0};
      be[lane] = 0.0;
      ta[lane] = 0.0;
    }
    lds_order();
  } else {
    static_assert(KP % 8 == 0 || KP % 4 == 0, "KP: multiple of 4");
    [&]<int... G>(std::integer_sequence<int, G...>) {
      (steps(std::integral_constant<int, (8 * G < KP ? 8 * G : 0)>{}, 8 * G), ...);
    }(std::make_integer_sequence<int, (KP + 7) / 8>{});
    // final 2 x 2: alpha_{K-2} = A[K-2][K-2], beta_{K-2} = A[K-1][K-2], alpha_{K-1}
    double c2 = 0.0, c1 = 0.0;  // each lane's a[K-2], a[K-1] (dynamic index: static select)
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      double t = a[j];
      asm volatile("" : "+v"(t));  // keep `a` in registers (see the step select above)
      c2 = j == K - 2 ? t : c2;
      c1 = j == K - 1 ? t : c1;
    }
    const double a22 = K >= 2 ? readlane(c2, K - 2) : readlane(c1, 0);
    const double b21 = K >= 2 ? readlane(c2, K - 1) : 0.0;
    const double a11 = readlane(c1, K - 1);
    if (lane == 0) {
      if (K >= 2) {
        tb[K - 2] = double2{a22, K > 2 ? be[K - 3] * be[K - 3] : 0.0};
        be[K - 2] = b21;
        tb[K - 1] = double2{a11, b21 * b21};
      } else {
        tb[0] = double2{a11, 0.0};
      }
    }
    lds_order();
  }
  if constexpr ((ABL & 16) != 0) {  // timing: setup + tridiagonalisation only
    if (lane < K) vo[lane] = tb[lane].x + be[lane];
    return;
  }
  // ---- 2. eigenvalue of rank `lane` (descending) ----
  double lo_l = 0.0, hi_l = 0.0, b2max = 0.0;
  if (lane < K) {
    const double a = tb[lane].x;
    const double r = (lane > 0 ? fabs(be[lane - 1]) : 0.0) + (lane + 1 < K ? fabs(be[lane]) : 0.0);
    lo_l = a - r;
    hi_l = a + r;
    b2max = tb[lane].y;
  } else {
    lo_l = tb[0].x;
    hi_l = tb[0].x;
  }
  const double gl = wave_min(lo_l), gu = wave_max(hi_l);
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, wave_max(b2max));
  constexpr double kEps = 2.220446049250313e-16;
  const double abstol = 1e-22 * tnorm + pivmin;
  const int jt = K - 1 - lane;  // ascending index of the target eigenvalue
  // first evaluation at the guess; every lane's (x, count) sample brackets every target
  double lo = gl - 2.0 * kEps * tnorm - pivmin, hi = gu + 2.0 * kEps * tnorm + pivmin;
  double x = lane < K ? fmin(fmax(gs[lane], lo), hi) : 0.5 * (lo + hi);
  double G = 0.0, H = 0.0;
  int cnt = sturm_gh(tb, K, x, pivmin, G, H);
  double* xs = ub;  // the tridiagonalisation's broadcast buffers are free now
  int* cs = (int*)wb;
  xs[lane] = x;
  cs[lane] = cnt;
  lds_order();
  for (int l = 0; l < K; ++l) {
    const double xl = xs[l];
    const int cl = cs[l];
    if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
  }
  double lam = x;
  if (lane < K && (ABL & 1) == 0) {
    int prev = -1;
    double sprev = __builtin_inf();
    for (int it = 0; it < 256; ++it) {
      // Laguerre toward the adjacent root on the target's side: with count(x) == jt the
      // nearest root above x IS lambda_jt, with count(x) == jt + 1 the nearest below is
      // (for a real-rooted polynomial the step never passes it).  A tiny step alone is not
      // convergence: next to a root on the OTHER side the steps are tiny too but grow (~2x);
      // accept only a tiny step that shrank, and extrapolate growing (escaping) steps 8x.
      bool lag = false;
      double xn = 0.0;
      if (cnt == jt || cnt == jt + 1) {
        xn = laguerre_toward(x, G, H, K, cnt == jt);
        double st = fabs(xn - x);
        if (prev == cnt && st >= 1.5 * sprev) {
          xn = fma(8.0, xn - x, x);
          st *= 8.0;
        }
        lag = __builtin_isfinite(xn) && xn >= lo && xn <= hi;
        if (lag && prev == cnt && st <= 1e-9 * fabs(x) && st <= 0.25 * sprev) { x = xn; break; }
        sprev = lag ? st : __builtin_inf();
      }
      if (!lag) { xn = 0.5 * (lo + hi); sprev = __builtin_inf(); }
      if (hi - lo <= 2.0 * kEps * (fabs(lo) + fabs(hi)) + abstol) { x = 0.5 * (lo + hi); break; }
      prev = lag ? cnt : -1;
      x = xn;
      cnt = sturm_gh(tb, K, x, pivmin, G, H);
      if (cnt <= jt) lo = x; else hi = x;
    }
    lam = x;
  }
  if constexpr ((ABL & 2) != 0) {
    if (lane < K) vo[lane] = lam;
    return;
  }
  // ---- 3. eigenvector of T at lam: twisted factorisation ----
  double y[KP];
  if (lane < K) {
    double P[KP], Q[KP];
    double dp = 0.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i < K) {
        const double2 t = tb[i];
        dp = guard_pivot(i == 0 ? t.x - lam : (t.x - lam) - t.y * rcp_nr(dp), pivmin);
        P[i] = dp;
      }
    }
    double dm = 0.0, gmin = 0.0;
    int r = K - 1;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < K) {
        const double a = tb[i].x - lam;
        dm = guard_pivot(i == K - 1 ? a : a - tb[i + 1].y * rcp_nr(dm), pivmin);
        Q[i] = dm;
        const double g = fabs(P[i] + dm - a);
        if (i == K - 1 || g < gmin) { gmin = g; r = i; }
      }
    }
    double cz = 1.0, nrm = 1.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < r) {
        cz = -be[i] * cz * rcp_nr(P[i]);
        nrm = fma(cz, cz, nrm);
      }
      y[i] = i < r ? cz : 0.0;
    }
    cz = 1.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i == r) y[i] = 1.0;
      if (i > r && i < K) {
        cz = -be[i - 1] * cz * rcp_nr(Q[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
    }
    const double sc = rsq_nr(nrm);
#pragma unroll
    for (int i = 0; i < KP; ++i) y[i] *= sc;
  } else {
#pragma unroll
    for (int i = 0; i < KP; ++i) y[i] = 0.0;
  }
  // ---- 4. back-transform y = H_0 ... H_{K-3} z and the bias ratio ----
  // u_s is zero in columns <= s, so steps s in [8g, 8g + 8) run the static column range
  // [8g, KP) (broadcast 16-B pairs of the reflector row)
  auto back = [&](auto J0c, int s_hi) {
    constexpr int J0 = decltype(J0c)::value;
    for (int s = s_hi; s >= J0; --s) {
      if (s + 2 >= K) continue;
      const double tau = ta[s];
      if (tau == 0.0) continue;
      const double* us = A + s * LU;
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        t0 = fma(uu.x, y[j], t0);
        t1 = fma(uu.y, y[j + 1], t1);
      }
      const double f = tau * (t0 + t1);
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        y[j] = fma(-f, uu.x, y[j]);
        y[j + 1] = fma(-f, uu.y, y[j + 1]);
      }
    }
  };
  [&]<int... G>(std::integer_sequence<int, G...>) {
    constexpr int NG = (KP + 7) / 8;
    (back(std::integral_constant<int, 8 * (NG - 1 - G)>{}, 8 * (NG - 1 - G) + 7), ...);
  }(std::make_integer_sequence<int, (KP + 7) / 8>{});
  if (lane < K) {
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < KP; ++j)
      if (j < K) v = fma(dd[j] * dd[j], y[j] * y[j], v);
    vo[lane] = v / lam;
  }
}

size_t bias_tri_lds(int K, int KP) { return ((size_t)K * (KP + 1) + 7 * 64 + 2) * sizeof(double); }

