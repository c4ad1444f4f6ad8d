// A/B-only CS-WLS kernels (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build --ab).
// Included by xs_wls_impl.h at the position they held in it; the production library never
// compiles them.  Measured against the production fused kernel in profiles/ (r02-r05).
#pragma once
// ------------------------------------------------------------------------------------------
// Resident fused CS-WLS.  The fused kernel above re-reads the date's panel
// slice for the residual pass: ~2.35 GB fetched per 2520-date fp64 step for 1.24 GB of panel,
// because ~512 dates are in flight and the re-read misses every cache.  Here ONE 4-wave
// workgroup per CU (waves_per_eu 1: 512 registers per lane, ~150 KB of LDS) streams its date
// with plain loads (lane = stock, `A` tiles in flight per wave) and KEEPS the residual-pass inputs
// of its first tiles on chip until the coefficients exist:
//   * tiles 0 .. TL-1 of each wave in LDS ([r | x_q | industry-or--1] rows, written after the
//     tile's moments),
//   * tiles TL .. TL+TR-1 in AGPRs (v_accvgpr_write after the moments, v_accvgpr_read in the
//     residual pass: 2Q + 3 registers per fp64 tile),
// and only the tiles past TL + TR are re-read (validity from per-tile ballots in LDS, no cap
// row); waves 1..3 issue their first re-read loads while wave 0 solves.  The moments use the
// per-lane order and the wave-ordered reduction of the deterministic fused kernel (same tile
// assignment: tile wid + 4 i of the date), so they are bitwise the same.
// ------------------------------------------------------------------------------------------
template <typename T> struct AgT;
template <> struct AgT<double> {  // one fp64 value in an AGPR pair
  int lo, hi;
  __device__ __forceinline__ void put(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(lo) : "v"((int)b));
    asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(hi) : "v"((int)(b >> 32)));
  }
  __device__ __forceinline__ double get() const {
    int l, h;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(l) : "a"(lo));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(h) : "a"(hi));
    return __builtin_bit_cast(double, ((long long)h << 32) | (long long)(unsigned)l);
  }
};
template <> struct AgT<float> {
  int v;
  __device__ __forceinline__ void put(float f) {
    asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(v) : "v"(__builtin_bit_cast(int, f)));
  }
  __device__ __forceinline__ float get() const {
    int r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(v));
    return __builtin_bit_cast(float, r);
  }
};
struct AgI {
  int v;
  __device__ __forceinline__ void put(int x) { asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(v) : "v"(x)); }
  __device__ __forceinline__ int get() const {
    int r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(v));
    return r;
  }
};

template <int Q, typename T>
struct ResGeo {
  using L = Layout<Q, T>;
  static constexpr int R = 8;                                   // segment replicas (2 per wave)
  static constexpr int TILE_B = (Q + 1) * kWT * (int)sizeof(T) + kWT * 4;  // one stored tile
  static constexpr int RED = 8 * 65 + L::NACC;                  // wg_reduce tile + partial row
  __host__ __device__ static constexpr int seg_region(int Pseg) {  // doubles, even
    const int a = Pseg * L::seg_stride(R), b = 4 * RED;
    return ((a > b ? a : b) + 1) & ~1;
  }
  __host__ __device__ static constexpr int okl_words(int N) { return (N + kWT - 1) / kWT; }
  __host__ __device__ static constexpr size_t lds_bytes(int Pseg, int N, int TL) {
    return ((size_t)seg_region(Pseg) + ((solve_lds_doubles<Q>(Pseg) + 1) & ~(size_t)1) +
            okl_words(N)) * 8 + (size_t)4 * TL * TILE_B;
  }
};

// VAR & 1 / & 2: timing-only ablations (no segment atomics / no style-Gram FMAs)
template <int Q, int TL, int TR, int A, typename T, int VAR = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void xs_resident_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int P, int Pseg, int pivot_mode, double tol,
    double* __restrict__ fout, T* __restrict__ eout, double* __restrict__ r2out,
    double* __restrict__ stats, int* __restrict__ status, double* __restrict__ mom_out,
    unsigned long long* __restrict__ tprof) {
  using L = Layout<Q, T>;
  using G = ResGeo<Q, T>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC, R = G::R;
  constexpr int SJ = L::seg_stride(R);
  constexpr int NRES = TL + TR;
  constexpr int NB = A + 1;  // tile buffers: A in flight + the one being consumed
  extern __shared__ double dyn[];
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red5[4][5];
  __shared__ int st_s;
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int MS = L::msize(Pseg);
  // phase timestamps (tools/xs_resident_phases.py): start, moments, reduction, solve, end
  auto stamp = [&](int k) {
    if (tprof && tid == 0) tprof[(size_t)d * 6 + k] = wall_clock64();
  };
  stamp(0);
  double* seg = dyn;                                   // segment table, then wg_reduce scratch
  double* sm = dyn + G::seg_region(Pseg);              // moments (md) + solve scratch
  unsigned long long* okl =
      (unsigned long long*)(sm + ((solve_lds_doubles<Q>(Pseg) + 1) & ~(size_t)1));
  char* store = (char*)(okl + G::okl_words(N));        // [4 waves][TL tiles][TILE_B]
  for (int i = tid; i < Pseg * SJ; i += 256) seg[i] = 0.0;
  __syncthreads();

  const T* Xd = X + (size_t)d * Q * N;
  const T* cd = cap + (size_t)d * N;
  const T* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;
  const int ntile_all = (N + kWT - 1) / kWT;
  const int ntile = ntile_all > wid ? (ntile_all - wid + 3) >> 2 : 0;  // tiles wid + 4 i
  const unsigned seg_a = lds_addr(seg + wid * (R / 4) + (lane & (R / 4 - 1)));

  struct Tile {
    T c, r, x[Q];
    int j;
  };
  Tile buf[NB];
  // WITHC: the moments pass (cap row too); NT: non-temporal (the tile is never re-read)
  auto ldt = [&](int i, Tile& t, bool withc, bool nt) {
    const int s = (wid + 4 * i) * kWT + lane;
    const bool in = s < N;
    auto ld = [&](const T* p) -> T {
      return in ? (nt ? __builtin_nontemporal_load(p + s) : p[s]) : T(0);
    };
    if (withc) t.c = ld(cd);
    t.r = ld(rd);
#pragma unroll
    for (int q = 0; q < Q; ++q) t.x[q] = ld(Xd + (size_t)q * N);
    t.j = (in && id) ? (int)id[s] : 0;
  };

  double v[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) v[i] = 0.0;
  // moments of one tile (lane = stock); returns the industry of a valid stock, else -1
  auto consume = [&](int i, const Tile& t, bool keep_bits) -> int {
    const int s = (wid + 4 * i) * kWT + lane;
    const int j = t.j;
    bool ok = (s < N) && (j >= 0) && (j < Pseg) && finite_v(t.c) && (t.c >= T(0)) && finite_v(t.r);
#pragma unroll
    for (int q = 0; q < Q; ++q) ok = ok && finite_v(t.x[q]);
    if (keep_bits) {
      const unsigned long long m = __ballot(ok);
      if (lane == 0) okl[wid + 4 * i] = m;
    }
    if (ok) {
      const double c = t.c, r = t.r, w = sqrt(c);
      double x[Q], wx[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) { x[q] = t.x[q]; wx[q] = w * x[q]; }
      if constexpr ((VAR & 2) != 0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) asm volatile("" ::"v"(wx[q]));
      } else {
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
          for (int u = 0; u <= q; ++u) v[q * (q + 1) / 2 + u] = fma(wx[q], x[u], v[q * (q + 1) / 2 + u]);
      }
      double sx = 0.0, sxx = 0.0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        v[NG + q] = fma(wx[q], r, v[NG + q]);
        v[NG + Q + q] = fma(c, x[q], v[NG + Q + q]);
        sx += x[q];
        sxx = fma(x[q], x[q], sxx);
      }
      v[NG + 2 * Q + 0] += c;
      v[NG + 2 * Q + 1] += sx;
      v[NG + 2 * Q + 2] += sxx;
      v[NG + 2 * Q + 3] += 1.0;
      const unsigned a = seg_a + (unsigned)(j * SJ * 8);
      const double wr = w * r;
      if constexpr ((VAR & 1) != 0) {
        asm volatile("" ::"v"(w), "v"(wr));
      } else {
        lds_add_nowait<0>(a, w);
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (lds_add_nowait<8 * R * (1 + I)>(a, wx[I]), ...);
        }(std::make_integer_sequence<int, Q>{});
        lds_add_nowait<8 * R * (Q + 1)>(a, wr);
        lds_add_nowait<8 * R * (Q + 2)>(a, c);
      }
    }
    return ok ? j : -1;
  };

  AgT<T> kr[TR > 0 ? TR : 1], kx[TR > 0 ? TR : 1][Q];
  AgI kj[TR > 0 ? TR : 1];
  auto tile_lds = [&](int i) { return store + (size_t)(wid * TL + i) * G::TILE_B; };

  // ---- moments pass: resident tiles (unrolled: compile-time buffer / AGPR indices) ----
#pragma unroll
  for (int i = 0; i < A; ++i)
    if (i < ntile) ldt(i, buf[i], true, i < NRES);
#pragma unroll
  for (int i = 0; i < NRES; ++i) {
    if (i < ntile) {
      __builtin_amdgcn_sched_barrier(0);
      if (i + A < ntile) ldt(i + A, buf[(i + A) % NB], true, i + A < NRES);
      __builtin_amdgcn_sched_barrier(0);
      const Tile& t = buf[i % NB];
      const int jj = consume(i, t, false);
      if (i < TL) {
        char* b = tile_lds(i);
        ((T*)b)[lane] = t.r;
#pragma unroll
        for (int q = 0; q < Q; ++q) ((T*)(b + (1 + q) * kWT * sizeof(T)))[lane] = t.x[q];
        ((int*)(b + (Q + 1) * kWT * sizeof(T)))[lane] = jj;
      } else if constexpr (TR > 0) {
        const int k = i - TL < TR ? i - TL : 0;  // always i - TL here
        kr[k].put(t.r);
#pragma unroll
        for (int q = 0; q < Q; ++q) kx[k][q].put(t.x[q]);
        kj[k].put(jj);
      }
    }
  }
  // ---- moments pass: tiles past the resident ones (re-read later), NB tiles per trip ----
  for (int i0 = NRES; i0 < ntile; i0 += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = i0 + u;
      if (i < ntile) {
        __builtin_amdgcn_sched_barrier(0);
        if (i + A < ntile) ldt(i + A, buf[(NRES + u + A) % NB], true, false);
        __builtin_amdgcn_sched_barrier(0);
        consume(i, buf[(NRES + u) % NB], true);
      }
    }
  }
  __syncthreads();
  stamp(1);
  // ---- deterministic reduction (as the DET fused kernel) ----
  for (int i = tid; i < Pseg * NS; i += 256) {
    const double* row = seg + (i / NS) * SJ + (i % NS) * R;
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) t += row[r];
    sm[NACC + i] = t;
    if (mom_out) aux_store(mom_out + (size_t)d * MS + NACC + i, t);
  }
  __syncthreads();
  double* wred = seg + wid * G::RED;  // the segment table is consumed: reuse it
  wg_reduce<NACC, true>(v, wred, wred + 8 * 65);
  __syncthreads();
  if (tid < NACC) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += seg[w * G::RED + 8 * 65 + tid];
    sm[tid] = t;
    if (mom_out) aux_store(mom_out + (size_t)d * MS + tid, t);
  }
  __syncthreads();
  stamp(2);

  // ---- solve (wave 0) while waves 1..3 start their re-read loads ----
  auto reread = [&](int i, Tile& t) { ldt(i, t, false, true); };
  auto prologue = [&]() {
#pragma unroll
    for (int k = 0; k < A; ++k)
      if (NRES + k < ntile) reread(NRES + k, buf[(NRES + k) % NB]);
  };
  // row-per-lane Cholesky (ROWL): the in-register triangle would need more VGPRs than the
  // AGPR-resident tiles leave (it spilled the whole kernel to scratch)
  if (wid == 0) solve_body<Q, true>(sm, d, P, Pseg, pivot_mode, tol, fout, cf_s, stats, status, &st_s);
  else prologue();
  __syncthreads();
  stamp(3);
  if (wid == 0) prologue();

  // ---- residual pass: specific returns + R^2 sums ----
  double beta[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) beta[q] = cf_s[q];
  const double cst = cf_s[Q];
  const double* fI = cf_s + Q + 1;
  T* ed = eout ? eout + (size_t)d * N : nullptr;
  double se = 0.0, see = 0.0, sr = 0.0, srr = 0.0, nn = 0.0;
  auto res1 = [&](int i, T rf, const T (&xf)[Q], int jj) {
    const int s = (wid + 4 * i) * kWT + lane;
    double e = (double)rf - cst;
#pragma unroll
    for (int q = 0; q < Q; ++q) e = fma(-beta[q], (double)xf[q], e);
    T eo = (T)qnan();
    if (jj >= 0) {
      if (P > 0) e -= fI[jj];
      se += e;
      see = fma(e, e, see);
      sr += (double)rf;
      srr = fma((double)rf, (double)rf, srr);
      nn += 1.0;
      eo = (T)e;
    }
    if (ed && s < N) {
      if constexpr (MFA_XS_NT_E) __builtin_nontemporal_store(eo, ed + s);
      else ed[s] = eo;
    }
  };
#pragma unroll
  for (int i = 0; i < NRES; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    if (i < ntile) {
      T rf, xf[Q];
      int jj;
      if (i < TL) {
        const char* b = tile_lds(i);
        rf = ((const T*)b)[lane];
#pragma unroll
        for (int q = 0; q < Q; ++q) xf[q] = ((const T*)(b + (1 + q) * kWT * sizeof(T)))[lane];
        jj = ((const int*)(b + (Q + 1) * kWT * sizeof(T)))[lane];
      } else {
        const int k = i - TL < TR ? i - TL : 0;
        rf = kr[k].get();
#pragma unroll
        for (int q = 0; q < Q; ++q) xf[q] = kx[k][q].get();
        jj = kj[k].get();
      }
      res1(i, rf, xf, jj);
    }
  }
  for (int i0 = NRES; i0 < ntile; i0 += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = i0 + u;
      if (i < ntile) {
        __builtin_amdgcn_sched_barrier(0);
        if (i + A < ntile) reread(i + A, buf[(NRES + u + A) % NB]);
        __builtin_amdgcn_sched_barrier(0);
        const Tile& t = buf[(NRES + u) % NB];
        const bool ok = (okl[wid + 4 * i] >> lane) & 1ull;
        res1(i, t.r, t.x, ok ? t.j : -1);
      }
    }
  }
  se = wave_sum(se); see = wave_sum(see); sr = wave_sum(sr); srr = wave_sum(srr); nn = wave_sum(nn);
  if (lane == 0) {
    red5[wid][0] = se; red5[wid][1] = see; red5[wid][2] = sr; red5[wid][3] = srr; red5[wid][4] = nn;
  }
  __syncthreads();
  if (tid == 0) {
    double a = 0, b = 0, c = 0, e2 = 0, n = 0;
    for (int w = 0; w < 4; ++w) {
      a += red5[w][0]; b += red5[w][1]; c += red5[w][2]; e2 += red5[w][3]; n += red5[w][4];
    }
    const double ve = b / n - (a / n) * (a / n);
    const double vr = e2 / n - (c / n) * (c / n);
    r2out[d] = (st_s & XS_BAD) ? qnan() : 1.0 - ve / vr;
  }
  stamp(4);
  if (tprof && tid == 0) tprof[(size_t)d * 6 + 5] = __smid();
}

