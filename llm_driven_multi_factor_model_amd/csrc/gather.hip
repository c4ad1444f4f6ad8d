// Zero-copy row-range gather from pinned host columns into HBM (date-sharded e2e job).
//
// A rank of the date-sharded job (models/e2e.py, DeviceFactorEngine.from_host_shard) needs, per
// stock, one contiguous range of the loader's rows (its dates + halo).  Gathering those ranges
// on the host (a threaded memcpy into staging buffers) and uploading them costs two passes over
// the bytes, the upload through a pageable bounce buffer.  Here the GPU reads the ranges
// straight out of the reader's pinned buffers over PCIe: one workgroup per range, consecutive
// lanes on consecutive rows (coalesced PCIe reads), every column of the range in one launch, and
// only the rank's bytes cross the link.  Host pointers are translated with
// hipHostGetDevicePointer; memory that is not pinned makes the call fail (the caller then takes
// the host gather).
#include "common.h"

namespace {

constexpr int kMaxCols = 24;

struct GatherCols {
  const void* src[kMaxCols];
  void* dst[kMaxCols];
  int elem[kMaxCols];  // 4 or 8 bytes
  int n;
};

__global__ __launch_bounds__(256) void gather_ranges_kernel(GatherCols cols,
                                                            const int64_t* __restrict__ ranges,
                                                            const int64_t* __restrict__ offs,
                                                            int64_t nr) {
  for (int64_t k = blockIdx.x; k < nr; k += gridDim.x) {
    const int64_t a = ranges[2 * k], len = ranges[2 * k + 1] - a, o = offs[k];
    for (int c = 0; c < cols.n; ++c) {
      if (cols.elem[c] == 8) {
        const int64_t* s = (const int64_t*)cols.src[c] + a;
        int64_t* d = (int64_t*)cols.dst[c] + o;
        for (int64_t i = threadIdx.x; i < len; i += 256) d[i] = s[i];
      } else {
        const int32_t* s = (const int32_t*)cols.src[c] + a;
        int32_t* d = (int32_t*)cols.dst[c] + o;
        for (int64_t i = threadIdx.x; i < len; i += 256) d[i] = s[i];
      }
    }
  }
}

}  // namespace

// host_src[ncols]: pinned host column pointers; dst[ncols]: device buffers of sum(len) elements;
// elem[ncols]: 4 or 8; ranges [nr][2] (start, stop) and offs [nr] (output offset of each range)
// on the device.  Returns hipErrorInvalidValue for a non-pinned source or a bad element size.
MFA_API int mfa_gather_host_ranges(const void* const* host_src, void* const* dst, const int* elem,
                                   int ncols, const int64_t* ranges, const int64_t* offs,
                                   int64_t nr, void* stream) {
  if (nr <= 0 || ncols <= 0) return 0;
  if (ncols > kMaxCols) return (int)hipErrorInvalidValue;
  GatherCols g{};
  g.n = ncols;
  for (int c = 0; c < ncols; ++c) {
    if (elem[c] != 4 && elem[c] != 8) return (int)hipErrorInvalidValue;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, const_cast<void*>(host_src[c]), 0) != hipSuccess || !dp)
      return (int)hipErrorInvalidValue;
    g.src[c] = dp;
    g.dst[c] = dst[c];
    g.elem[c] = elem[c];
  }
  const int grid = (int)(nr < 8192 ? nr : 8192);
  hipLaunchKernelGGL(gather_ranges_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, g,
                     ranges, offs, nr);
  return (int)hipGetLastError();
}
