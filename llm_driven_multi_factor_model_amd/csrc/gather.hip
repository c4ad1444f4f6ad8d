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

// ---------------------------------------------------------------------------------------------
// Rows <-> grid as an LDS-tiled transpose.  The rows are sorted by (stock, date), the grid is
// date-major, so a per-element scatter writes one 4-byte word per 128-byte line.  Here a
// 256-thread block
// owns a tile of 64 dates x 64 stocks: each stock's rows of those dates are one contiguous range
// (toff[s][tb] .. toff[s][tb + 1], from the sorted (stock, date) key), read along the rows
// (coalesced), placed in an LDS tile at their local date, and written out along the stocks
// (coalesced); grid cells without a row get `fill`.  The gather is the same walk backwards.
// (A plain per-element 1:1 scatter kernel measured no faster than torch's index_put: 5.6 ms for
// 20 columns of 12.4 M rows, profiles/r05/r05s.)
// X: C columns of R rows (column stride xs); did [R] the rows' date (< Dg); toff [Ng][NTB + 1]
// with NTB = ceil(Dg / 64); grid cell (c, d, s) at c * gs + d * ds + s.
namespace {

constexpr int kTT = 64;  // tile edge (dates and stocks)

template <bool SCATTER, typename E>
__global__ __launch_bounds__(256) void tile_transpose_kernel(
    E* __restrict__ X, int64_t xs, const int* __restrict__ did, const int64_t* __restrict__ toff,
    int Dg, int Ng, int C, E* __restrict__ G, int64_t gs, int64_t ds, double fill_d) {
  __shared__ E tile[kTT][kTT + 1];
  const E fill = (E)fill_d;
  const int ntb = (Dg + kTT - 1) / kTT;
  const int tb = blockIdx.x, sb = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int d0 = tb * kTT, s0 = sb * kTT;
  // this lane's rows: stock j = wv * 16 + k (k < 16), row toff[s][tb] + lane when inside
  int64_t row[16];
  int ldate[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int s = s0 + wv * 16 + k;
    row[k] = -1;
    ldate[k] = 0;
    if (s < Ng) {
      const int64_t a = toff[(int64_t)s * (ntb + 1) + tb], b = toff[(int64_t)s * (ntb + 1) + tb + 1];
      if (a + lane < b) {
        row[k] = a + lane;
        ldate[k] = did[a + lane] - d0;
      }
    }
  }
  for (int c = 0; c < C; ++c) {
    E* Xc = X + (int64_t)c * xs;
    E* Gc = G + (int64_t)c * gs;
    if constexpr (SCATTER) {
      for (int e = t; e < kTT * kTT; e += 256) tile[e / kTT][e % kTT] = fill;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (row[k] >= 0) tile[ldate[k]][wv * 16 + k] = Xc[row[k]];
      __syncthreads();
      for (int e = t; e < kTT * kTT; e += 256) {
        const int dl = e / kTT, sl = e % kTT;
        if (d0 + dl < Dg && s0 + sl < Ng) Gc[(int64_t)(d0 + dl) * ds + s0 + sl] = tile[dl][sl];
      }
      __syncthreads();
    } else {
      for (int e = t; e < kTT * kTT; e += 256) {
        const int dl = e / kTT, sl = e % kTT;
        if (d0 + dl < Dg && s0 + sl < Ng) tile[dl][sl] = Gc[(int64_t)(d0 + dl) * ds + s0 + sl];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (row[k] >= 0) Xc[row[k]] = tile[ldate[k]][wv * 16 + k];
      __syncthreads();
    }
  }
}

}  // namespace

// scatter (dir = 1: rows -> grid, `fill` in empty cells) or gather (dir = 0: grid -> rows) of C
// columns of 4- or 8-byte floats; see tile_transpose_kernel.  Every stock has <= 64 rows per
// 64-date block (dates distinct within a stock), which the sorted (stock, date) key guarantees.
MFA_API int mfa_rows_grid(int dir, int elem, void* X, int64_t xs, const int* did,
                          const int64_t* toff, int Dg, int Ng, int C, void* G, int64_t gs,
                          int64_t ds, double fill, void* stream) {
  if (Dg <= 0 || Ng <= 0 || C <= 0) return 0;
  const dim3 grid((Dg + kTT - 1) / kTT, (Ng + kTT - 1) / kTT);
  hipStream_t s = (hipStream_t)stream;
#define MFA_RG(DIR_, E_)                                                                        \
  hipLaunchKernelGGL((tile_transpose_kernel<DIR_, E_>), grid, dim3(256), 0, s, (E_*)X, xs, did, \
                     toff, Dg, Ng, C, (E_*)G, gs, ds, fill)
  if (elem == 4) {
    if (dir) MFA_RG(true, float); else MFA_RG(false, float);
  } else if (elem == 8) {
    if (dir) MFA_RG(true, double); else MFA_RG(false, double);
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef MFA_RG
  return (int)hipGetLastError();
}
