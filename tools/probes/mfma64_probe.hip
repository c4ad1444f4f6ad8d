// Probe: register layout of v_mfma_f64_16x16x4f64 on gfx950.
// A[i][k] = 100*i + k (from lane l: i = l%16, k = l/16), B = identity-ish picks.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void k(double* out) {
  const int l = threadIdx.x;
  // A: lane l holds A[l%16][l/16]; B: lane l holds B[l/16][l%16]
  const int ai = l % 16, ak = l / 16;
  const double a = 100.0 * ai + ak;
  const int bk = l / 16, bj = l % 16;
  const double b = (bj < 4 && bk == bj) ? 1.0 : (bj == 4 + bk ? 1000.0 : 0.0);
  v4d c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
  double* d;
  hipMalloc(&d, 256 * 8);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  double h[256];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  // D = A*B: D[i][j] = A[i][j] for j<4 ; D[i][4+k] = 1000*A[i][k]
  int ok = 1;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * (l / 16) + r, j = l % 16;
      double exp = j < 4 ? 100.0 * i + j : (j < 8 ? 1000.0 * (100.0 * i + (j - 4)) : 0.0);
      if (h[l * 4 + r] != exp) {
        if (ok) printf("mismatch lane %d r %d: got %g expect %g\n", l, r, h[l * 4 + r], exp);
        ok = 0;
      }
    }
  printf("layout D[i=4*(l/16)+r][j=l%%16]: %s\n", ok ? "CONFIRMED" : "WRONG");
  for (int l = 0; l < 20; ++l) printf("lane %d: %g %g %g %g\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  return 0;
}
