// A/B-only eigen kernels / launchers (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build
// --ab).  Included by eigen.hip at the position they held in it; the production library never
// compiles them.  Their measurements against the production solvers: profiles/ (r01-r05).
#pragma once
// ---------------- lane-dense tridiagonal bias solver (bias mode 11, K <= 42) ----------------
// mc_bias_tri2_kernel keeps one 42 x 42 problem per wave: 42 of 64 lanes do useful work in every
// phase (34 % of each VALU issue slot idles).  Here a 128-thread workgroup (2 waves) carries
// THREE problems on 126 lanes:
//   lanes 0..41 of wave w  -> slot w, row (or eigenvalue rank) = lane;
//   lanes 42..63 of wave w -> slot 2, row = lane - 42 + 22 w  (rows 0..21 in wave 0, 22..43 in 1).
// Slots 0 / 1 are wave-local; slot 2 spans both waves, so the Householder step publishes its
// column and its partial sums through LDS around 4 workgroup barriers (slot 2's sums: the two
// waves' halves added in a fixed order).  Eigenvalues, eigenvectors and the back-transform are
// per lane, as in mode 5, and use the same arithmetic (sturm_gh_p, 1e-8 Laguerre stop,
// one-Newton reciprocals); only slot 2's wave sums associate differently.
// Per slot LDS: packed reflector rows + tables, zero-initialised (rows / columns beyond K
// read as exact zeros) -> 36.9 KB per workgroup at K = 42: 4 workgroups (8 waves) per CU, each
// wave under a 256-VGPR budget.
constexpr int kT3Slot = 1120 + 8 * 48;  // reflector rows (K = 42, KP = 44) + 8 tables of 48

__device__ __forceinline__ void split_total(double v, bool hi_lane, double& lo, double& hi) {
  const double a = row16_sum(hi_lane ? 0.0 : v);
  const double b = row16_sum(hi_lane ? v : 0.0);
  lo = (readlane(a, 0) + readlane(a, 16)) + readlane(a, 32);
  hi = readlane(b, 32) + readlane(b, 48);
}

template <int ABL = 0>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void
mc_bias_tri3_kernel(const double* __restrict__ D0, int K, int M, int DM,
                    const double* __restrict__ Cz, const int* __restrict__ dvalid,
                    double* __restrict__ vout) {
  constexpr int KP = 44;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const bool hiL = l >= 42;
  const int slot = hiL ? 2 : w;
  const int r = hiL ? l - 42 + 22 * w : l;
  const bool live = r < K;
  const int q = blockIdx.x * 3 + slot;
  const bool qok = q < DM;
  const int d = qok ? q / M : 0, m = qok ? q % M : 0;
  const bool dok = qok && dvalid[d] != 0;
  for (int e = tid; e < 3 * kT3Slot + 8; e += 128) sm[e] = 0.0;
  double* S = sm + slot * kT3Slot;
  double* R = S;                        // packed reflector rows (tri2 layout)
  double* wb = S + 1120;                // [48] broadcast w
  double2* tb = (double2*)(wb + 48);    // [48] {alpha_i, beta_{i-1}^2}
  double* be = (double*)(tb + 48);      // [48] beta_i
  double* ta = be + 48;                 // [48] tau_s
  double* dd = ta + 48;                 // [48] sqrt(D0)
  double* gs = dd + 48;                 // [48] sorted diagonal; Laguerre x later
  double* xc = gs + 48;                 // [48] column s of the step; Sturm counts later
  double* part = sm + 3 * kT3Slot;      // [2] slot-2 sig halves, [2] slot-2 kk halves
  __syncthreads();
  const double* d0 = D0 + (size_t)d * K;
  const double di = (dok && live) ? sqrt(fmax(d0[r], 0.0)) : 0.0;
  if (live) dd[r] = di;
  __syncthreads();
  double a[KP];
  const double* c = Cz + (size_t)m * K * K;
  const int ri = live ? r : 0;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    a[j] = (j < K && dok && live) ? di * c[j * K + ri] * dd[j] : 0.0;
    if ((j & 7) == 7) lds_batch();
  }
  {
    const double g = (dok && live) ? di * c[ri * K + ri] * di : 0.0;
    if (live) wb[r] = g;
    __syncthreads();
    if (live) {
      int rank = 0;
      for (int j = 0; j < K; ++j) {
        const double h = wb[j];
        rank += (h > g) || (h == g && j < r);
      }
      gs[rank] = g;
    }
    __syncthreads();
  }
  // ---- 1. Householder tridiagonalisation, 3 problems in lock step ----
  auto steps = [&](auto J0c) {
    constexpr int J0 = decltype(J0c)::value;
    for (int s = J0; s < J0 + 8 && s < K; ++s) {
      double xs = a[J0];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (J0 + k < KP) {
          double t = a[J0 + k];
          asm volatile("" : "+v"(t));
          xs = s == J0 + k ? t : xs;
        }
      const bool act = live && r > s;
      const double x = act ? xs : 0.0;
      if (live) xc[r] = xs;
      double slo, shi;
      split_total(live && r > s + 1 ? x * x : 0.0, hiL, slo, shi);
      if (l == 0) part[w] = shi;
      __syncthreads();  // B1: column s and slot 2's partial norms
      const double x0 = s + 1 < K ? xc[s + 1] : 0.0;
      const double alpha = xc[s];
      const double sig = hiL ? part[0] + part[1] : slo;
      double u = 0.0, tau = 0.0, beta = x0;
      if (sig != 0.0) {
        const double n2 = fma(x0, x0, sig);
        const double nrm = n2 * rsq_nr(n2);
        beta = x0 >= 0.0 ? -nrm : nrm;
        tau = rcp_nr(nrm * (nrm + fabs(x0)));
        u = act ? (r == s + 1 ? x0 - beta : x) : 0.0;
      }
      double* us = R + tri2_row_off<KP>(s) - J0;
      if (s + 2 < K && live && r >= J0 && r < KP) us[r] = u;
      if (r == 0) {
        tb[s] = double2{alpha, s > 0 ? be[s - 1] * be[s - 1] : 0.0};
        be[s] = beta;
        ta[s] = tau;
      }
      __syncthreads();  // B2: u_s of every slot
      double p0 = 0.0, p1 = 0.0;
      if (s + 2 >= K) us = R + tri2_row_off<KP>(J0) - J0;
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 uu = *(const double2*)(us + j);
        p0 = fma(a[j], uu.x, p0);
        p1 = fma(a[j + 1], uu.y, p1);
        if (((j - J0) & 7) == 6) lds_batch();
      }
      const double p = act ? tau * (p0 + p1) : 0.0;
      double klo, khi;
      split_total(u * p, hiL, klo, khi);
      if (l == 0) part[2 + w] = khi;
      __syncthreads();  // B3: slot 2's partial u^T p
      const double kk = 0.5 * tau * (hiL ? part[2] + part[3] : klo);
      const double wv = p - kk * u;
      if (live) wb[r] = wv;
      __syncthreads();  // B4: w of every slot
#pragma unroll
      for (int j = J0; j < KP; j += 2) {
        const double2 ww = *(const double2*)(wb + j), uu = *(const double2*)(us + j);
        a[j] = fma(-u, ww.x, fma(-wv, uu.x, a[j]));
        a[j + 1] = fma(-u, ww.y, fma(-wv, uu.y, a[j + 1]));
        if (((j - J0) & 7) == 6) lds_batch();
      }
    }
  };
  [&]<int... G>(std::integer_sequence<int, G...>) {
    (steps(std::integral_constant<int, 8 * G>{}), ...);
  }(std::make_integer_sequence<int, (KP + 7) / 8>{});
  __syncthreads();
  // ---- 2. eigenvalue of rank r (descending), as mode 5; Gershgorin bounds from the tables ----
  double gl = __builtin_inf(), gu = -__builtin_inf(), b2max = 0.0;
  for (int i = 0; i < K; ++i) {
    const double ad = tb[i].x;
    const double rr = (i > 0 ? fabs(be[i - 1]) : 0.0) + (i + 1 < K ? fabs(be[i]) : 0.0);
    gl = fmin(gl, ad - rr);
    gu = fmax(gu, ad + rr);
    b2max = fmax(b2max, tb[i].y);
  }
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, b2max);
  constexpr double kEps = 2.220446049250313e-16;
  const double abstol = 1e-22 * tnorm + pivmin;
  const int jt = K - 1 - r;
  double lo = gl - 2.0 * kEps * tnorm - pivmin, hi = gu + 2.0 * kEps * tnorm + pivmin;
  double x = live ? fmin(fmax(gs[r], lo), hi) : 0.5 * (lo + hi);
  double G = 0.0, H = 0.0;
  int cnt = sturm_gh_p(tb, K, x, G, H);
  __syncthreads();  // every lane has read its gs slot
  int* csv = (int*)xc;
  if (live) {
    gs[r] = x;
    csv[r] = cnt;
  }
  __syncthreads();
  for (int i = 0; i < K; ++i) {
    const double xl = gs[i];
    const int cl = csv[i];
    if (cl <= jt) lo = fmax(lo, xl); else hi = fmin(hi, xl);
  }
  double lam = x;
  if (live && dok && (ABL & 1) == 0) {
    int prev = -1;
    double sprev = __builtin_inf();
    for (int it = 0; it < 256; ++it) {
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
        if (lag && prev == cnt && st <= 1e-8 * fabs(x) && st <= 0.25 * sprev) { x = xn; break; }
        sprev = lag ? st : __builtin_inf();
      }
      if (!lag) { xn = 0.5 * (lo + hi); sprev = __builtin_inf(); }
      if (hi - lo <= 2.0 * kEps * (fabs(lo) + fabs(hi)) + abstol) { x = 0.5 * (lo + hi); break; }
      prev = lag ? cnt : -1;
      x = xn;
      cnt = sturm_gh_p(tb, K, x, G, H);
      if (cnt <= jt) lo = x; else hi = x;
    }
    lam = x;
  }
  // ---- 3. eigenvector of T at lam (twisted factorisation), as mode 5 ----
  double y[KP];
  if (live && dok && (ABL & 2) == 0) {
    double dp = 0.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i < K) {
        const double2 t = tb[i];
        dp = guard_pivot(i == 0 ? t.x - lam : (t.x - lam) - t.y * rcp_nr1(dp), pivmin);
      }
      y[i] = i < K ? dp : 0.0;
    }
    double dm = 0.0, gmin = 0.0;
    int rt = K - 1;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < K) {
        const double ai = tb[i].x - lam;
        dm = guard_pivot(i == K - 1 ? ai : ai - tb[i + 1].y * rcp_nr1(dm), pivmin);
        const double g = fabs(y[i] + dm - ai);
        if (i == K - 1 || g < gmin) { gmin = g; rt = i; }
      }
    }
    double cz = 1.0, nrm = 1.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < rt) {
        cz = -be[i] * cz * rcp_nr1(y[i]);
        nrm = fma(cz, cz, nrm);
        y[i] = cz;
      }
    }
    dm = 0.0;
#pragma unroll
    for (int i = KP - 1; i >= 0; --i) {
      if (i < K && i > rt) {
        const double ai = tb[i].x - lam;
        dm = guard_pivot(i == K - 1 ? ai : ai - tb[i + 1].y * rcp_nr1(dm), pivmin);
        y[i] = dm;
      }
    }
    cz = 1.0;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i == rt) y[i] = 1.0;
      if (i > rt && i < K) {
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
  // ---- 4. back-transform and the bias ratio ----
  if ((ABL & 2) == 0) {
    auto back = [&](auto J0c, int s_hi) {
      constexpr int J0 = decltype(J0c)::value;
      for (int s = s_hi; s >= J0; --s) {
        if (s + 2 >= K) continue;
        const double tau = ta[s];
        if (tau == 0.0) continue;
        const double* us = R + tri2_row_off<KP>(s) - J0;
        double t0 = 0.0, t1 = 0.0;
#pragma unroll
        for (int j = J0; j < KP; j += 2) {
          const double2 uu = *(const double2*)(us + j);
          t0 = fma(uu.x, y[j], t0);
          t1 = fma(uu.y, y[j + 1], t1);
          if (((j - J0) & 7) == 6) lds_batch();
        }
        const double f = tau * (t0 + t1);
#pragma unroll
        for (int j = J0; j < KP; j += 2) {
          const double2 uu = *(const double2*)(us + j);
          y[j] = fma(-f, uu.x, y[j]);
          y[j + 1] = fma(-f, uu.y, y[j + 1]);
          if (((j - J0) & 7) == 6) lds_batch();
        }
      }
    };
    [&]<int... G>(std::integer_sequence<int, G...>) {
      constexpr int NG = (KP + 7) / 8;
      (back(std::integral_constant<int, 8 * (NG - 1 - G)>{}, 8 * (NG - 1 - G) + 7), ...);
    }(std::make_integer_sequence<int, (KP + 7) / 8>{});
  }
  if (!qok || !live) return;
  double* vo = vout + (size_t)q * K;
  if (!dok) {
    vo[r] = qnan();
    return;
  }
  double v = 0.0;
#pragma unroll
  for (int j = 0; j < KP; ++j)
    if (j < K) v = fma(dd[j] * dd[j], y[j] * y[j], v);
  vo[r] = (ABL & 2) ? lam : v / lam;
}


size_t bias_tri3_lds() { return (3 * (size_t)kT3Slot + 8) * sizeof(double); }
