// Probe: sustained rate of v_mfma_f64_16x16x4f64 vs fp64 VALU FMA on gfx950 (MI355X).
// Each wave runs 4 independent MFMA accumulator chains (or 16 VALU FMA chains) for ITER steps.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;
__global__ __launch_bounds__(256) void mfma_k(double* out, double a0) {
  double a = a0 + threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
  v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < ITER; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ __launch_bounds__(256) void valu_k(double* out, double a0) {
  double a = a0 + threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
  double c[16];
  for (int k = 0; k < 16; ++k) c[k] = k;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = fma(a, b, c[k]);
  double s = 0;
  for (int k = 0; k < 16; ++k) s += c[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  double* d;
  const int nb = 256 * 8;
  hipMalloc(&d, (size_t)nb * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_k, nb, 256, 0, 0, d, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double fl = (double)nb * 4 * ITER * 4 * 2048;
    printf("mfma_f64_16x16x4: %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(valu_k, nb, 256, 0, 0, d, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double fv = (double)nb * 256 * ITER * 16 * 2;
    printf("valu fma_f64: %.3f ms  %.1f TFLOP/s\n", ms, fv / ms / 1e9);
  }
  return 0;
}
