// Device helpers of the Householder-tridiagonal eigen solvers (csrc/eigen.hip: one wave per
// problem, K <= 64; csrc/eigen_wide.hip: one workgroup of 2-3 waves per problem, K <= 160):
// Newton-refined reciprocals / inverse square roots, the pivot and division-free Sturm
// recurrences with their Laguerre step, LDS ordering fences and the packed reflector-row layout.
#pragma once
#include "common.h"

namespace mfa {

__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
// one Newton step: <= 2.2e-15 relative on random doubles (tools/probes/rcp64_probe.hip; the
// v_rcp_f64 seed alone is 4.6e-8) -- enough for the Sturm / Laguerre pivot recurrence
__device__ __forceinline__ double rcp_nr1(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = fma(0.5 * y, fma(-x * y, y, 1.0), y);
  return fma(0.5 * y, fma(-x * y, y, 1.0), y);
}

__device__ __forceinline__ double guard_pivot(double q, double pivmin) {
  return fabs(q) < pivmin ? -pivmin : q;
}

// LDL^T pivots q_i of T - x I (T: tb[i] = {alpha_i, beta_{i-1}^2}): returns the Sturm count
// #{eigenvalues < x}, with G = f'/f = sum 1/(x - lambda) and H = sum 1/(x - lambda)^2 for
// f = det(T - x I) (from q_i' and q_i'' carried through the same recurrence).
__device__ __forceinline__ int sturm_gh(const double2* tb, int K, double x, double pivmin,
                                        double& G, double& H) {
  double q = guard_pivot(tb[0].x - x, pivmin), dq = -1.0, d2q = 0.0, g = 0.0, h = 0.0;
  int cnt = q < 0.0;
  auto step = [&](const double2 t) {
    const double r = rcp_nr1(q);
    const double e = dq * r;
    g += e;
    h = fma(e, e, fma(-d2q, r, h));
    const double br = t.y * r;
    d2q = br * r * fma(-2.0 * dq, e, d2q);
    dq = fma(br, e, -1.0);
    q = guard_pivot((t.x - x) - br, pivmin);
    cnt += q < 0.0;
  };
  // the recurrence is one long dependent chain: load the coefficients 4 steps ahead so the
  // LDS latency is not exposed on every step
  int i = 1;
  for (; i + 3 < K; i += 4) {
    const double2 t0 = tb[i], t1 = tb[i + 1], t2 = tb[i + 2], t3 = tb[i + 3];
    step(t0);
    step(t1);
    step(t2);
    step(t3);
  }
  for (; i < K; ++i) step(tb[i]);
  const double r = rcp_nr1(q);
  const double e = dq * r;
  G = g + e;
  H = fma(e, e, fma(-d2q, r, h));
  return cnt;
}

// Laguerre step for a degree-n real-rooted polynomial: the two candidates lie between x and
// its adjacent roots; returns the one on the requested side (NaN if neither is finite).
// FAST: Newton-refined v_rsq / v_rcp instead of the IEEE square root and divisions (~10
// dependent instructions each on the iteration's critical path); the iteration is guarded by
// Sturm counts, so ~1-ulp steps only move where it lands within the stopping tolerance.
template <bool FAST = false>
__device__ __forceinline__ double laguerre_toward(double x, double G, double H, int n, bool right) {
  const double q = (double)(n - 1) * fma((double)n, H, -G * G);
  const double rad = FAST ? (q > 0.0 ? q * rsq_nr(q) : 0.0) : sqrt(fmax(0.0, q));
  const double c1 = FAST ? x - (double)n * rcp_nr(G + rad) : x - (double)n / (G + rad);
  const double c2 = FAST ? x - (double)n * rcp_nr(G - rad) : x - (double)n / (G - rad);
  const bool f1 = __builtin_isfinite(c1), f2 = __builtin_isfinite(c2);
  if (f1 && f2) return right ? fmax(c1, c2) : fmin(c1, c2);
  return f1 ? c1 : (f2 ? c2 : qnan());
}

// Division-free Sturm evaluation (bias mode 5): the determinant recurrence of the leading
// minors f_i(x) = det(T_i - x I) = (a_{i-1} - x) f_{i-1} - b_{i-2}^2 f_{i-2}, with f' and f''
// carried by the differentiated recurrences.  Same outputs as sturm_gh (Sturm count = sign
// changes of f_0 .. f_K = #eigenvalues < x, G = f'/f, H = G^2 - f''/f), but every step is
// fmas off the previous two values (no reciprocal in the dependent chain: ~1/4 of the q-form's
// chain latency).  The three sequences are rescaled together by a power of two every 4 steps
// (exact), so they stay in range; they are homogeneous, so G and H are unaffected.
template <bool FAST = false>
__device__ __forceinline__ int sturm_gh_p(const double2* tb, int K, double x, double& G,
                                          double& H) {
  double f2 = 1.0, f1 = tb[0].x - x;   // f_0, f_1
  double g2 = 0.0, g1 = -1.0;          // f'_0, f'_1
  double h2 = 0.0, h1 = 0.0;           // f''_0, f''_1
  int cnt = f1 < 0.0;
  auto step = [&](const double2 t) {
    const double d = t.x - x, b2 = t.y;
    const double f0 = fma(d, f1, -b2 * f2);
    const double g0 = fma(d, g1, -fma(b2, g2, f1));
    const double h0 = fma(d, h1, -fma(b2, h2, 2.0 * g1));
    cnt += (f0 < 0.0) != (f1 < 0.0);
    f2 = f1; f1 = f0; g2 = g1; g1 = g0; h2 = h1; h1 = h0;
  };
  auto rescale = [&]() {
    int e;
    frexp(fmax(fabs(f1), fabs(f2)), &e);
    const double sc = ldexp(1.0, -e);
    f1 *= sc; f2 *= sc; g1 *= sc; g2 *= sc; h1 *= sc; h2 *= sc;
  };
  int i = 1;
  for (; i + 3 < K; i += 4) {
    const double2 t0 = tb[i], t1 = tb[i + 1], t2 = tb[i + 2], t3 = tb[i + 3];
    step(t0);
    step(t1);
    step(t2);
    step(t3);
    rescale();
  }
  for (; i < K; ++i) step(tb[i]);
  const double r = FAST ? rcp_nr(f1) : 1.0 / f1;
  G = g1 * r;
  H = fma(G, G, -h1 * r);
  return cnt;
}

// Single-wave workgroups: LDS executes one wave's DS instructions in issue order (they also
// return in order), so a lane reading what another lane of the SAME wave wrote needs only the
// compiler to keep program order -- no s_waitcnt / barrier round trip (wsync) per exchange.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }


// LDS reads of an unrolled broadcast loop are issued in batches of 4 x 16 B: without the fence
// hipcc hoists all ~22 of them (88 VGPRs) above the FMAs, which set the kernel's register peak
__device__ __forceinline__ void lds_batch() { asm volatile("" ::: "memory"); }



template <int KP, int GS = 8>
__host__ __device__ constexpr int tri2_rows_doubles(int K) {
  // rows s = 0 .. K-3, row s holds columns [GS floor(s/GS), KP) (GS-step groups)
  int n = 0;
  for (int s = 0; s + 2 < K; ++s) n += KP - GS * (s / GS);
  return n;
}
template <int KP, int GS = 8>
__device__ __forceinline__ int tri2_row_off(int s) {
  // sum over earlier full groups g' < g of GS (KP - GS g') + (s - GS g)(KP - GS g)
  const int g = s / GS;
  return GS * (g * KP - GS * g * (g - 1) / 2) + (s - GS * g) * (KP - GS * g);
}


}  // namespace mfa
