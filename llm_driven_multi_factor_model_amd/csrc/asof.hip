// Device-side point-in-time as-of join (K12) and the matched-column gather.
//
// Reference: Barra_factor_cal/load_data.py:41-62 (robust_merge_asof) — per ts_code, a pandas
// merge_asof(direction='backward') of daily rows (trade_date) onto statement rows (f_ann_date),
// looping over stocks in Python.  The host path is csrc_host/asof.cpp (threaded two-pointer
// sweep); this is the GPU path for panels that already live in HBM.
//
// Both sides are (int32 group, int64 key) arrays sorted lexicographically by (group, key).
// One lane per left row: a branch-light binary search over the WHOLE right array for the upper
// bound of (g, key) — the last right row with (rg, rk) <= (g, key) — then a group check.  Left
// rows arrive sorted, so the 64 lanes of a wave search neighbouring right ranges and the probes
// share L2 lines (each XCD's L2 sees a contiguous slab of left rows: blockIdx -> contiguous rows).
// Ties among right rows resolve to the last one, as pandas merge_asof does.
//
// mfa_asof_gather then writes out[i, c] = right_vals[idx[i], c] (NaN when idx[i] < 0) for C
// fp32 columns: one lane per (row, column), row-major so consecutive lanes store contiguously.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void asof_search_kernel(const int32_t* __restrict__ lg,
                                                          const int64_t* __restrict__ lk, int64_t nl,
                                                          const int32_t* __restrict__ rg,
                                                          const int64_t* __restrict__ rk, int64_t nr,
                                                          int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nl) return;
  const int32_t g = lg[i];
  const int64_t k = lk[i];
  // count of right rows with (rg, rk) <= (g, k)
  int64_t lo = 0, n = nr;
  while (n > 0) {
    const int64_t half = n >> 1;
    const int64_t m = lo + half;
    const int32_t gm = rg[m];
    const bool le = (gm < g) || (gm == g && rk[m] <= k);
    lo = le ? m + 1 : lo;
    n = le ? n - half - 1 : half;
  }
  const int64_t j = lo - 1;
  out[i] = (j >= 0 && rg[j] == g) ? j : -1;
}

__global__ __launch_bounds__(256) void asof_gather_kernel(const float* __restrict__ rv, int64_t nr,
                                                          const int64_t* __restrict__ idx, int64_t nl,
                                                          int C, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nl * (int64_t)C) return;
  const int64_t i = t / C;
  const int c = (int)(t - i * C);
  const int64_t j = idx[i];
  out[t] = (j >= 0 && j < nr) ? rv[j * C + c] : __builtin_nanf("");
}

}  // namespace

MFA_API int mfa_asof_search(const int32_t* lg, const int64_t* lk, int64_t nl, const int32_t* rg,
                            const int64_t* rk, int64_t nr, int64_t* out, void* stream) {
  if (nl <= 0) return 0;
  if (nr < 0) return (int)hipErrorInvalidValue;
  const int64_t blocks = (nl + 255) / 256;
  if (blocks > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(asof_search_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     lg, lk, nl, rg, rk, nr, out);
  return (int)hipGetLastError();
}

MFA_API int mfa_asof_gather(const float* rv, int64_t nr, const int64_t* idx, int64_t nl, int C,
                            float* out, void* stream) {
  if (nl <= 0 || C <= 0) return 0;
  const int64_t total = nl * (int64_t)C;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(asof_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     rv, nr, idx, nl, C, out);
  return (int)hipGetLastError();
}
