// Accuracy of v_rcp_f64 / v_rsq_f64 seeds and of one / two Newton steps on random doubles
// (decides how many refinement steps the Sturm / twisted-factorisation recurrences need).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

__global__ void probe(const double* x, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  const double r0 = __builtin_amdgcn_rcp(v);
  const double r1 = fma(r0, fma(-v, r0, 1.0), r0);
  const double r2 = fma(r1, fma(-v, r1, 1.0), r1);
  const double ex = 1.0 / v;
  out[3 * i + 0] = fabs(r0 - ex) / fabs(ex);
  out[3 * i + 1] = fabs(r1 - ex) / fabs(ex);
  out[3 * i + 2] = fabs(r2 - ex) / fabs(ex);
}

int main() {
  const int n = 1 << 20;
  std::vector<double> h(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double m = 1.0 + (double)(s >> 11) * (1.0 / 9007199254740992.0);
    const int e = (int)((s >> 3) % 120) - 60;
    h[i] = ((s & 1) ? -1.0 : 1.0) * std::ldexp(m, e);
  }
  double *dx, *dout;
  if (hipMalloc(&dx, n * sizeof(double)) != hipSuccess || hipMalloc(&dout, 3 * n * sizeof(double)) != hipSuccess) return 1;
  (void)hipMemcpy(dx, h.data(), n * sizeof(double), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, dx, n, dout);
  std::vector<double> o(3 * n);
  (void)hipMemcpy(o.data(), dout, 3 * n * sizeof(double), hipMemcpyDeviceToHost);
  double mx[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) mx[k] = std::fmax(mx[k], o[3 * i + k]);
  std::printf("{\"rcp_seed_max_rel\": %.3e, \"one_newton\": %.3e, \"two_newton\": %.3e}\n", mx[0], mx[1], mx[2]);
  (void)hipFree(dx);
  (void)hipFree(dout);
  return 0;
}
