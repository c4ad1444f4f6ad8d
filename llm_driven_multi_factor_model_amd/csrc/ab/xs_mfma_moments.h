// A/B-only CS-WLS kernels (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build --ab).
// Included by xs_wls_impl.h at the position they held in it; the production library never
// compiles them.  Measured against the production fused kernel in profiles/ (r02-r05).
#pragma once
// ------------------------------------------------------------------------------------------
// K1 on the matrix cores: the dense moments as ONE 16 x 16 fp64 MFMA accumulator per wave.
//
// Lane l owns Gram channel c = l & 15 and, per k-step, stock k0 + (l >> 4) of its 64-stock
// tile: v_mfma_f64_16x16x4f64 accumulates G[i][j] += sum_k alpha_i(k) beta_j(k) over 4 stocks
// with (for a valid stock, weight w = sqrt(cap); invalid stocks contribute 0):
//   channel  c < Q : alpha = x_c,  beta = w x_c        -> G[p][q] = Swxx,  G[p][Q] = Swxr
//            c = Q : alpha = r,    beta = w r           G[p][Q+1] = Scx (beta = w w = cap)
//          c = Q+1 : alpha = w,    beta = w w           G[Q+2][Q+1] = Sc, G[Q+2][Q+2] = n
//          c = Q+2 : alpha = 1,    beta = 1             G[p][Q+2] summed over p = Sx
//          c = Q+3 : alpha = sum_q x_q^2, beta = 0      G[Q+3][Q+2] = Sxx
// The 79 per-lane fp64 accumulators of the VALU body (158 VGPRs: 2 waves / SIMD) become 8
// VGPRs per lane, so 3-4 workgroups fit on a CU.  A per-stock prep pass (lane = stock) checks
// validity, does the industry segment atomics and writes {w or -1, sum x^2} to a per-wave aux
// row; ring rows are padded (+8 B fp32 / +16 B fp64) so the 16 channel reads of one k-step hit
// distinct LDS banks.  The 4 waves' accumulators are summed in wave order (deterministic).
// ------------------------------------------------------------------------------------------
template <typename T> struct MfGeo;
template <> struct MfGeo<float> {
  static constexpr int ROWP = kWT * 4 + 8;    // padded fp32 row
  static constexpr int NB = 2;                // ring slots per wave
};
template <> struct MfGeo<double> {
  static constexpr int ROWP = kWT * 8 + 16;   // padded fp64 row
  static constexpr int NB = 2;
};

template <int Q, typename T>
struct RingMF {
  static constexpr int ROWP = MfGeo<T>::ROWP;
  static constexpr int NB = MfGeo<T>::NB;
  static constexpr int WSLOT = (Q + 2) * ROWP + kWT * 2;     // rows | int16 ids
  static constexpr int AUX = kWT * 16;                        // {w | -1, sum x^2} per stock
  static constexpr int RED = 256 * 8;                          // this wave's 16x16 tile
  static constexpr int RW0 = NB * WSLOT + AUX;
  static constexpr int RINGW = RW0 > RED ? RW0 : RED;
  static constexpr int BYTES = 4 * RINGW;
};

template <int Q, typename T>
__device__ __forceinline__ constexpr int dma_per_tile_mf(bool has_ind) {
  return Q + 2 + (has_ind ? 1 : 0);  // one (padded) row per instruction
}

template <int Q, int VAR, int R, typename T>
__device__ __forceinline__ void moments_body_mf(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, int d, char* ring, double* dyn,
    double* md, int nb = 0, int ne = -1, double* __restrict__ gout = nullptr) {
  static_assert(Q + 4 <= 16, "one 16x16 MFMA tile: Q <= 12");
  using L = Layout<Q, T>;
  using G = RingMF<Q, T>;
  constexpr int NS = L::NS, NG = L::NG, NACC = L::NACC;
  constexpr int WSLOT = G::WSLOT, RINGW = G::RINGW, NB = G::NB, ROWP = G::ROWP;
  if (ne < 0) ne = N;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nthr >> 6;
  constexpr bool DET = (VAR & 32) != 0;
  const int rep = DET ? wid * (R / 4) + (lane & (R / 4 - 1)) : (lane & (R - 1));
  const unsigned seg_a = lds_addr(dyn + rep);
  for (int i = tid; i < R * Pseg * NS; i += nthr) dyn[i] = 0.0;
  __syncthreads();

  const T* Xd = X + (size_t)d * Q * N;
  const T* cd = cap + (size_t)d * N;
  const T* rd = ret + (size_t)d * N;
  const int16_t* id = ind ? ind + (size_t)d * N : nullptr;

  char* wring = ring + wid * RINGW;
  double2* aux = (double2*)(wring + NB * WSLOT);
  const int nrows = dma_per_tile_mf<Q, T>(id != nullptr);
  const int ntile_all = (ne - nb + kWT - 1) / kWT;
  const int ntile = ntile_all > wid ? (ntile_all - wid + nw - 1) / nw : 0;
  auto issue = [&](int i) {
    char* slot = wring + (i % NB) * WSLOT;
    const int s0 = nb + (wid + i * nw) * kWT;
    if constexpr (sizeof(T) == 4) {
      const bool in = s0 + lane < ne;
      if (in) glds4(cd + s0 + lane, slot);
      if (in) glds4(rd + s0 + lane, slot + ROWP);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (in) glds4(Xd + (size_t)q * N + s0 + lane, slot + (2 + q) * ROWP);
    } else {  // one 512-B fp64 row per instruction (lanes 0-31, 16 B each)
      const int s = s0 + 2 * (lane & 31);
      const bool in = lane < 32 && s < ne;
      if (in) glds16(cd + s, slot);
      if (in) glds16(rd + s, slot + ROWP);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (in) glds16(Xd + (size_t)q * N + s, slot + (2 + q) * ROWP);
    }
    if (id && lane < kWT / 2 && s0 + 2 * lane < ne) glds4(id + s0 + 2 * lane, slot + (Q + 2) * ROWP);
  };
  // this lane's Gram channel: ring row (x_c: 2 + c, r: 1, aux channels: row 0 as a dummy)
  const int ch = lane & 15, kq = lane >> 4;
  const int crow = ch < Q ? 2 + ch : (ch == Q ? 1 : 0);
  v4d acc4[4];  // 4 independent accumulation chains (the f64 MFMA's dependent latency)
#pragma unroll
  for (int a = 0; a < 4; ++a) acc4[a] = v4d{0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < NB - 1 && i < ntile; ++i) issue(i);
  for (int i = 0; i < ntile; ++i) {
    const bool tail = (i + NB - 1 >= ntile);
    wait_vmcnt(tail ? 0 : (NB - 2) * nrows);
    __builtin_amdgcn_wave_barrier();
    if (i + NB - 1 < ntile) issue(i + NB - 1);
    const char* slot = wring + (i % NB) * WSLOT;
    const T* bf = (const T*)slot;
    // ---- prep: lane = stock
    {
      const int s = nb + (wid + i * nw) * kWT + lane;
      const T cf = *(const T*)(slot + lane * sizeof(T));
      const T rf = *(const T*)(slot + ROWP + lane * sizeof(T));
      const int j = id ? (int)((const int16_t*)(slot + (Q + 2) * ROWP))[lane] : 0;
      T xf[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) xf[q] = *(const T*)(slot + (2 + q) * ROWP + lane * sizeof(T));
      bool ok = (s < ne) && (j >= 0) && (j < Pseg) && finite_v(cf) && (cf >= T(0)) && finite_v(rf);
#pragma unroll
      for (int q = 0; q < Q; ++q) ok = ok && finite_v(xf[q]);
      double w = -1.0, s2 = 0.0;
      if (ok) {
        const double c = cf, r = rf;
        w = sqrt(c);
        double wx[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          wx[q] = w * (double)xf[q];
          s2 = fma((double)xf[q], (double)xf[q], s2);
        }
        if (VAR & 1) {  // timing-only ablation: skip the segment atomics
          asm volatile("" ::"v"(w), "v"(r));
        } else {
          const unsigned a = seg_a + (unsigned)(j * NS * R * 8);
          lds_add_nowait<0>(a, w);
          [&]<int... I>(std::integer_sequence<int, I...>) {
            (lds_add_nowait<8 * R * (1 + I)>(a, wx[I]), ...);
          }(std::make_integer_sequence<int, Q>{});
          lds_add_nowait<8 * R * (Q + 1)>(a, w * r);
          lds_add_nowait<8 * R * (Q + 2)>(a, c);
        }
      }
      // aux row: asm store (like the segment atomics) so hipcc's waitcnt pass does not drain
      // the in-flight DMA tile for it; LDS ops of one wave complete in order
      const unsigned aa = lds_addr(aux + lane);
      asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %2 offset:8" ::"v"(aa), "v"(w),
                   "v"(s2) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // ---- matrix cores: 16 k-steps of 4 stocks
    if constexpr ((VAR & 2) == 0) {
      const T* rowp = (const T*)(slot + crow * ROWP);
#pragma unroll
      for (int k0 = 0; k0 < kWT; k0 += 4) {
        const int k = k0 + kq;
        const double2 a2 = aux[k];
        const double raw = (double)rowp[k];
        const bool okk = a2.x >= 0.0;
        const double wp = okk ? a2.x : 0.0;
        double al, be;
        if (ch <= Q) {
          al = okk ? raw : 0.0;
          be = al * wp;
        } else if (ch == Q + 1) {
          al = wp;
          be = wp * wp;
        } else if (ch == Q + 2) {
          al = okk ? 1.0 : 0.0;
          be = al;
        } else {
          al = ch == Q + 3 ? a2.y : 0.0;
          be = 0.0;
        }
        acc4[(k0 >> 2) & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(al, be, acc4[(k0 >> 2) & 3], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const v4d acc = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
  // the 4 waves' 16x16 tiles, summed in wave order
  double* tile = (double*)wring;
#pragma unroll
  for (int r = 0; r < 4; ++r) tile[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
  __syncthreads();
  auto gsum = [&](int i, int j) {
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += ((const double*)(ring + w * RINGW))[i * 16 + j];
    return t;
  };
  double mv = 0.0;
  if (tid < NG) {
    int q = 0;
    while ((q + 1) * (q + 2) / 2 <= tid) ++q;
    mv = gsum(q, tid - q * (q + 1) / 2);
  } else if (tid < NG + Q) {
    mv = gsum(tid - NG, Q);
  } else if (tid < NG + 2 * Q) {
    mv = gsum(tid - NG - Q, Q + 1);
  } else if (tid == NG + 2 * Q) {
    mv = gsum(Q + 2, Q + 1);
  } else if (tid == NG + 2 * Q + 1) {
    for (int q = 0; q < Q; ++q) mv += gsum(q, Q + 2);
  } else if (tid == NG + 2 * Q + 2) {
    mv = gsum(Q + 3, Q + 2);
  } else if (tid == NG + 2 * Q + 3) {
    mv = gsum(Q + 2, Q + 2);
  }
  static_assert(NACC <= 256, "one thread per moment");
  __syncthreads();  // md may alias the ring
  if (tid < NACC) {
    md[tid] = mv;
    if (gout) gout[tid] = mv;
  }
  for (int i = tid; i < Pseg * NS; i += nthr) {
    const double* row = dyn + i * R;  // unpadded [Pseg * NS][R] table (MFMA A/B kernels)
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) t += row[r];
    md[NACC + i] = t;
    if (gout) gout[NACC + i] = t;
  }
  __syncthreads();
}

template <int Q, int VAR, int R, typename T>
__global__ __launch_bounds__(256) void xs_moments_mf_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int Pseg, int S, int C, double* __restrict__ mom) {
  __shared__ __attribute__((aligned(16))) char ring[RingMF<Q, T>::BYTES];
  extern __shared__ double dyn[];
  const int b = blockIdx.x, d = b / S, sc = b - d * S;
  const int nb = sc * C, ne = min(N, nb + C);
  moments_body_mf<Q, VAR, R, T>(X, cap, ret, ind, N, Pseg, d, ring, dyn,
                                mom + (size_t)b * Layout<Q, T>::msize(Pseg), nb, ne);
}

// High-occupancy fused kernel: MFMA moments (few VGPRs, small padded ring) -> wave-0 solve
// -> residual pass with UU iterations in flight; 3-4 workgroups per CU.
template <int Q, typename T>
constexpr int fused_mf_ring_bytes() {
  constexpr int a = RingMF<Q, T>::BYTES;
  constexpr int b = (int)(solve_lds_doubles<Q>(128) * 8);
  return a > b ? a : b;
}

template <int Q, int R, int VAR, typename T, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void xs_fused_mf_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int N, int P, int Pseg, int pivot_mode, double tol,
    double* __restrict__ fout, T* __restrict__ eout, double* __restrict__ r2out,
    double* __restrict__ stats, int* __restrict__ status, double* __restrict__ mom_out) {
  __shared__ __attribute__((aligned(16))) char ring[fused_mf_ring_bytes<Q, T>()];
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red[4][5];
  __shared__ int st_s;
  extern __shared__ double dyn[];
  const int d = blockIdx.x;
  double* sm = (double*)ring;
  moments_body_mf<Q, VAR & 35, R, T>(X, cap, ret, ind, N, Pseg, d, ring, dyn, sm, 0, -1,
                                     mom_out ? mom_out + (size_t)d * Layout<Q, T>::msize(Pseg)
                                             : nullptr);
  if constexpr ((VAR & 8) != 0) {  // timing-only ablation: no solve
    for (int i = threadIdx.x; i < Q + 1 + P; i += blockDim.x) cf_s[i] = sm[i] * 1e-30;
    if (threadIdx.x == 0) st_s = 0;
  } else if (threadIdx.x < 64) {
    solve_body<Q, true>(sm, d, P, Pseg, pivot_mode, tol, fout, cf_s, stats, status, &st_s);
  }
  __syncthreads();
  constexpr int UR = sizeof(T) == 4 ? 2 : 1;
  if constexpr ((VAR & 4) == 0)
    resid_body<Q, T, false, UR>(X, cap, ret, ind, d, N, P, cf_s, (st_s & XS_BAD) != 0, eout,
                                r2out, red);
}

