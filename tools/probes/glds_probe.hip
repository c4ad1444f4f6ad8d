#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;
__global__ void k(const float* g, float* out) {
  __shared__ float s[1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // each wave loads 256 floats (1 KiB): lane l -> floats [4l, 4l+4)
  __builtin_amdgcn_global_load_lds((gbl_void*)(g + w * 256 + lane * 4), (lds_void*)(s + w * 256), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) out[i] = s[i];
}
int main() {
  float *g, *o; hipMalloc(&g, 4096); hipMalloc(&o, 4096);
  float h[1024]; for (int i = 0; i < 1024; ++i) h[i] = i;
  hipMemcpy(g, h, 4096, hipMemcpyHostToDevice);
  k<<<1, 256>>>(g, o);
  hipMemcpy(h, o, 4096, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 1024; ++i) bad += h[i] != i;
  printf("bad=%d  h[5]=%f h[300]=%f h[1023]=%f\n", bad, h[5], h[300], h[1023]);
  return 0;
}
