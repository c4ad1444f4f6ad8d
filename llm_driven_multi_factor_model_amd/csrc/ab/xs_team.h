// A/B-only CS-WLS kernels (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build --ab).
// Included by xs_wls_impl.h at the position they held in it; the production library never
// compiles them.  Measured against the production fused kernel in profiles/ (r02-r05).
#pragma once
// ------------------------------------------------------------------------------------------
// Pipelined team CS-WLS (persistent grid, deferred residuals): C stock chunks per date, each
// chunk's moments and residuals done by the same workgroup, dates solved by their team's last
// arriver, and no workgroup ever idles while its team catches up.
//
// The fused kernel's residual pass re-reads the date's panel slice: one workgroup streams a
// whole 490 KB fp64 date in ~35 us, ~512 dates are in flight, so ~250 MB of other dates pass
// through the 256 MB Infinity Cache between a line's first read and its re-read and most
// re-reads go to HBM (2.46 GB moved per 1.34 GB compulsory, profiles/r02_xs_cluster_ab.md).  A
// one-wave-per-date team that WAITS for its partners (round-3 first try, r03_team_ab.md) pays
// the wait and a redundant solve per member on the 2 workgroup slots of a CU and lost 25-260 %.
// Here a persistent workgroup loops over tickets:
//   1. take a ticket t of its group (blockIdx & 7: the blocks of one XCD), t -> chunk c = t % C
//      of date d = group + 8 (t / C); stream the chunk once (LDS-DMA ring) into raw moments;
//   2. publish the partial row (write-through sc1 stores), arrive on the date's counter; the
//      LAST arriver sums the C partials in chunk order (bitwise-deterministic), solves in wave 0
//      and publishes the residual coefficients + a ready flag carrying the status word;
//   3. `lag` tickets later (the chunk's date has been solved by then), the same workgroup
//      re-reads ITS chunk for the residual pass: ~10-20 us after the first read instead of
//      ~40, so the re-read is an Infinity-Cache hit; partial R^2 sums are combined in chunk
//      order by the last member to finish.
// Progress (no co-residency assumption): tickets are taken in order by running workgroups, and a
// workgroup always finishes step 2 of a ticket it took before it waits on anything, so every
// fully ticketed date gets solved.  A workgroup waits (step 3) only for a date whose ticket it
// took `lag` or more tickets ago; if that date is not fully ticketed, every ticket taken since
// belongs to it, so a waiting workgroup holds lag + 1 of its C tickets: with lag >= 1 and
// C <= 16, all resident workgroups of a group can be waiting at once only if fewer than
// (C - 1) / (lag + 1) + 1 <= 8 of them are resident.  Every poll is bounded anyway
// (XS_COOP_TIMEOUT status bit): the grid always drains.
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table):
// payloads stored sc1, every storing wave waits vmcnt(0), a workgroup barrier, then ONE lane
// adds / stores the counter or flag; readers poll with sc1 loads from one lane, barrier, and
// load the payload with sc1 loads.
// sync = [tickets 8 | arrive[D] | done[D] | ready[D]] ints, zeroed before every launch.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int Q, int R, int VAR, typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(Q <= 10 ? 2 : MFA_XS_WPE_BIGQ, Q <= 10 ? 2 : MFA_XS_WPE_BIGQ))) void xs_pipe_kernel(
    const T* __restrict__ X, const T* __restrict__ cap, const T* __restrict__ ret,
    const int16_t* __restrict__ ind, int D, int N, int P, int Pseg, int C, int Cs, int lag,
    int pivot_mode, double tol, double* __restrict__ fout, T* __restrict__ eout,
    double* __restrict__ r2out, double* __restrict__ stats, int* __restrict__ status,
    double* __restrict__ mom, double* __restrict__ coef, double* __restrict__ sums,
    unsigned long long* __restrict__ okm, int* __restrict__ sync) {
  __shared__ __attribute__((aligned(16))) char ring[fused_ring_bytes<Q, T>()];
  __shared__ double cf_s[Q + 1 + 128];
  __shared__ double red[4][5];
  __shared__ double rs[5];
  __shared__ int tk_s, last_s, st_s, flag_s;
  extern __shared__ double dyn[];
  const int tid = threadIdx.x;
  const int grp = (int)blockIdx.x & (kPipeGroups - 1);
  const int ndg = D > grp ? (D - grp + kPipeGroups - 1) / kPipeGroups : 0;
  const int ntk = ndg * C;  // this group's tickets
  const int MS = Layout<Q, T>::msize(Pseg);
  const int NT = (N + kWT - 1) / kWT;
  const int KC = Q + 1 + P;
  int* tick = sync;
  int* arrive = sync + kPipeGroups;
  int* done = arrive + D;
  int* ready = done + D;
  double* sm = (double*)ring;  // the chunk's moments, then the solve's scratch
  int pend[kPipeMaxLag + 1];   // tickets whose residual pass is pending (oldest first)
  int np = 0;
  bool more = true;
  for (;;) {
    int t = ntk;
    if (more) {
      __syncthreads();  // tk_s of the previous iteration has been read by every thread
      if (tid == 0) tk_s = __hip_atomic_fetch_add(tick + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      t = tk_s;
      more = t < ntk;
    }
    if (t < ntk) {
      // ---- 1 + 2: moments of the chunk, publish, arrive; the last arriver solves the date ----
      const int k = t / C, c = t - k * C, d = grp + kPipeGroups * k;
      const int nb = c * Cs, ne = min(N, nb + Cs);
      moments_body<Q, VAR & 35, R, T>(X, cap, ret, ind, N, Pseg, d, ring, dyn, sm, nb, ne, nullptr,
                                      okm + (size_t)d * NT);
      double* mp = mom + ((size_t)d * C + c) * MS;
      for (int i = tid; i < MS; i += blockDim.x) st_sc1(mp + i, sm[i]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        last_s = __hip_atomic_fetch_add(arrive + d, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == C - 1;
      __syncthreads();
      if (last_s) {
        // the date's moments: the C partials summed in chunk order (all loads of a thread are
        // issued before its first add: a load -> add chain pays the round trip C times)
        const double* md = mom + (size_t)d * C * MS;
        for (int i = tid; i < MS; i += blockDim.x) {
          double v[kCoopMaxC];
#pragma unroll
          for (int kk = 0; kk < kCoopMaxC; ++kk) v[kk] = kk < C ? ld_sc1(md + (size_t)kk * MS + i) : 0.0;
          double s = v[0];
#pragma unroll
          for (int kk = 1; kk < kCoopMaxC; ++kk)
            if (kk < C) s += v[kk];
          sm[i] = s;
        }
        __syncthreads();
        if (tid < 64) solve_body<Q>(sm, d, P, Pseg, pivot_mode, tol, fout, cf_s, stats, status, &st_s);
        __syncthreads();
        double* co = coef + (size_t)d * KC;
        for (int i = tid; i < KC; i += blockDim.x) st_sc1(co + i, cf_s[i]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(ready + d, st_s | kReadyBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int i = 0; i <= kPipeMaxLag; ++i)
        if (i == np) pend[i] = t;
      ++np;
    }
    if (np > 0 && (np > lag || !more)) {
      // ---- 3: residual pass of the oldest pending chunk ----
      const int t2 = pend[0];
#pragma unroll
      for (int i = 0; i < kPipeMaxLag; ++i) pend[i] = pend[i + 1];
      --np;
      const int k2 = t2 / C, c2 = t2 - k2 * C, d2 = grp + kPipeGroups * k2;
      const int nb2 = c2 * Cs, ne2 = min(N, nb2 + Cs);
      if (tid == 0) {
        int v = 0;
        for (int it = 0; it < kCoopSpin; ++it) {
          v = __hip_atomic_load(ready + d2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v) break;
          __builtin_amdgcn_s_sleep(4);
        }
        flag_s = v ? v : (kReadyBit | XS_COOP_TIMEOUT);
      }
      __syncthreads();
      const int st2 = flag_s & ~kReadyBit;
      const double* co2 = coef + (size_t)d2 * KC;
      for (int i = tid; i < KC; i += blockDim.x) cf_s[i] = ld_sc1(co2 + i);
      __syncthreads();
      const bool bad = (st2 & (XS_BAD | XS_COOP_TIMEOUT)) != 0;
      resid_body<Q, T>(X, cap, ret, ind, d2, N, P, cf_s, bad, eout, nullptr, red, ResidPre<Q, T>{}, rs,
                       nb2, ne2, okm + (size_t)d2 * NT);
      // R^2: the last member of the team to finish combines the C chunk sums in chunk order
      if (tid < 64) {
        double* sd = sums + (size_t)d2 * C * 5;
        int lastd = 0;
        if (tid == 0) {
#pragma unroll
          for (int j = 0; j < 5; ++j) st_sc1(sd + c2 * 5 + j, rs[j]);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          lastd = __hip_atomic_fetch_add(done + d2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == C - 1;
          if ((st2 & XS_COOP_TIMEOUT) != 0) atomicOr(status + d2, XS_COOP_TIMEOUT);
        }
        if (__builtin_amdgcn_readfirstlane(lastd)) {
          double v[5];
#pragma unroll
          for (int j = 0; j < 5; ++j) v[j] = tid < C ? ld_sc1(sd + tid * 5 + j) : 0.0;
          double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
          for (int kk = 0; kk < C; ++kk)  // chunk order, wave-uniform
#pragma unroll
            for (int j = 0; j < 5; ++j) a[j] += readlane(v[j], kk);
          if (tid == 0) {
            const double n = a[4];
            const double ve = a[1] / n - (a[0] / n) * (a[0] / n);
            const double vr = a[3] / n - (a[2] / n) * (a[2] / n);
            r2out[d2] = bad ? qnan() : 1.0 - ve / vr;
          }
        }
      }
    } else if (!more) {
      break;
    }
  }
}

