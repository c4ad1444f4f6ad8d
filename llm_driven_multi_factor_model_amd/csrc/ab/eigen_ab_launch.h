// A/B-only eigen kernels / launchers (MFA_AB=1 builds: python -m llm_driven_multi_factor_model_amd._build
// --ab).  Included by eigen.hip at the position they held in it; the production library never
// compiles them.  Their measurements against the production solvers: profiles/ (r01-r05).
#pragma once
// A/B-only solvers and timing ablations (tools builds, MFA_AB=1): mode 4 (lean layout, pivot-form
// Sturm), 3 (round-2 kernel), 11 (lane-dense), 6-20 (mode-5 variants), 41-67 (ablations).
bool launch_bias_tri_ab(const double* D0, int D, int K, int M, const double* Cz, const int* dvalid,
                     double* ws, hipStream_t s) {
  if (g_bias_mode == 4 || g_bias_mode == 5) {
#define MFA_TRI2(KP_)                                                                        \
    if (K <= KP_) {                                                                        \
      if (g_bias_mode == 5) /* padded eigenvector phase at the measured width (K <= 44) */ \
        hipLaunchKernelGGL((mc_bias_tri2_kernel<KP_, true, 0, MFA_TRI2_WPE, false, 8, 8, 2,  \
                                                (KP_ == 44), false, (KP_ == 44)>),         \
                           dim3(D * M), dim3(64),                                          \
                           bias_tri2_lds(K, KP_), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);            \
      else                                                                                 \
        hipLaunchKernelGGL((mc_bias_tri2_kernel<KP_, false>), dim3(D * M), dim3(64),       \
                           bias_tri2_lds(K, KP_), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);            \
      return true;                                                                         \
    }
    MFA_TRI2(8)
    MFA_TRI2(16)
    MFA_TRI2(24)
    MFA_TRI2(32)
    MFA_TRI2(44)
    MFA_TRI2(48)
    MFA_TRI2(64)
#undef MFA_TRI2
    return false;
  }
  if ((g_bias_mode == 11 || g_bias_mode == 111 || g_bias_mode == 112) && K <= 42 &&
      tri2_rows_doubles<44>(K) <= 1120) {  // lane-dense: 3 problems per 2-wave workgroup
    const int DM = D * M, blocks = (DM + 2) / 3;
    if (g_bias_mode == 11)
      hipLaunchKernelGGL((mc_bias_tri3_kernel<0>), dim3(blocks), dim3(128), bias_tri3_lds(), s, D0,
                         K, M, DM, Cz, dvalid, ws);
    else if (g_bias_mode == 111)  // timing: no Laguerre iterations
      hipLaunchKernelGGL((mc_bias_tri3_kernel<1>), dim3(blocks), dim3(128), bias_tri3_lds(), s, D0,
                         K, M, DM, Cz, dvalid, ws);
    else  // timing: no eigenvectors / back-transform
      hipLaunchKernelGGL((mc_bias_tri3_kernel<2>), dim3(blocks), dim3(128), bias_tri3_lds(), s, D0,
                         K, M, DM, Cz, dvalid, ws);
    return true;
  }
  if ((g_bias_mode == 15 || g_bias_mode == 16) && K <= 44) {  // A/B: padded + every reflector
    // row stored, LDS reads fenced every 2 (15) / 1 (16) double2 steps (LB 4 / 2: fewer spills)
    if (g_bias_mode == 15)
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 4, 2, true, true>),
                         dim3(D * M), dim3(64), bias_tri2_lds(K + 2, 44), s, D0, K, M, Cz, dvalid,
                         ws, nullptr, nullptr, D, 0);
    else
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 2, 2, true, true>),
                         dim3(D * M), dim3(64), bias_tri2_lds(K + 2, 44), s, D0, K, M, Cz, dvalid,
                         ws, nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode == 20 && K <= 44) {  // A/B: the default + tau-only back-transform skips
    hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, true, false, true, false, true>),
                       dim3(D * M), dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws,
                       nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode == 19 && K <= 44) {  // A/B: the default + Newton-refined Laguerre arithmetic
    hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, true, false, true, true>),
                       dim3(D * M), dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws,
                       nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode == 18 && K <= 44) {  // A/B: padded, steps s >= K-2 skip the update
    hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, true, false, true>),
                       dim3(D * M), dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws,
                       nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode == 14 && K <= 44) {  // A/B: mode 5 with the unpadded eigenvector phase
    hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 2, false>),
                       dim3(D * M), dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws,
                       nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode == 13 && K <= 44) {  // A/B: four accumulators per matvec / dot product
    hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 8, 4>), dim3(D * M),
                       dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode == 10 && K <= 44) {  // A/B: LDS broadcast reads fenced in batches of 8 x 16 B
    hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 8, 16>), dim3(D * M),
                       dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);
    return true;
  }
  if ((g_bias_mode == 8 || g_bias_mode == 9) && K <= 44) {  // A/B: Laguerre stop at 1e-9 / 1e-7
    if (g_bias_mode == 8)
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 9>), dim3(D * M),
                         dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);
    else
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, MFA_TRI2_WPE, false, 7>), dim3(D * M),
                         dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);
    return true;
  }
  if ((g_bias_mode == 6 || g_bias_mode == 7) && K <= 44) {  // A/B: mode 5 at 4 / 5 waves per SIMD
    if (g_bias_mode == 6)
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, 4>), dim3(D * M), dim3(64),
                         bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);
    else
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, 0, 5>), dim3(D * M), dim3(64),
                         bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, ws, nullptr, nullptr, D, 0);
    return true;
  }
  if (g_bias_mode > 70 && g_bias_mode < 78 && K > 32 && K <= 42) {
    // round 6: phase ablations of the PRODUCTION K = 42 instantiation (KP = 42, 2-step groups,
    // KP-entry tables, 4 waves / SIMD) for the per-phase instruction budget
    // (tools/bias_phase_budget.py): 71 = no Laguerre iterations, 72 = no eigenvectors /
    // back-transform, 74 = no tridiagonalisation, 73 / 75 / 76 / 77 their unions; outputs
    // meaningless
    const int abl = g_bias_mode - 70;
#define MFA_TRI2_ABL42(A_)                                                                   \
    if (abl == A_)                                                                         \
      hipLaunchKernelGGL((mc_bias_tri2_kernel<42, true, A_, 4, false, 8, 8, 2, true, false, true, \
                                              false, false, 1, kTri2GS, true>),             \
                         dim3(D * M), dim3(64), bias_tri2_lds(K, 42, kTri2GS, true), s, D0, K, M, \
                         Cz, dvalid, ws, nullptr, nullptr, D, 0);
    MFA_TRI2_ABL42(1) MFA_TRI2_ABL42(2) MFA_TRI2_ABL42(3) MFA_TRI2_ABL42(4) MFA_TRI2_ABL42(5)
    MFA_TRI2_ABL42(6) MFA_TRI2_ABL42(7)
#undef MFA_TRI2_ABL42
    return true;
  }
  if (g_bias_mode > 60 && g_bias_mode < 69 && K <= 44) {  // timing-only ablations of mode 5
    const int abl = g_bias_mode == 68 ? 32 : g_bias_mode - 60;  // 68: Sturm-evaluation counts
#define MFA_TRI2_ABL(A_)                                                                     \
    if (abl == A_)                                                                         \
      hipLaunchKernelGGL((mc_bias_tri2_kernel<44, true, A_, MFA_TRI2_WPE, false, 8, 8, 2, true, \
                                              false, true>),                                \
                         dim3(D * M), dim3(64), bias_tri2_lds(K, 44), s, D0, K, M, Cz, dvalid, \
                         ws, nullptr, nullptr, D, 0);
    MFA_TRI2_ABL(1) MFA_TRI2_ABL(2) MFA_TRI2_ABL(3) MFA_TRI2_ABL(4) MFA_TRI2_ABL(5)
    MFA_TRI2_ABL(6) MFA_TRI2_ABL(7) MFA_TRI2_ABL(32)
#undef MFA_TRI2_ABL
    return true;
  }
#define MFA_TRI(KP_)                                                                         \
  if (K <= KP_) {                                                                          \
    hipLaunchKernelGGL((mc_bias_tri_kernel<KP_>), dim3(D * M), dim3(64), bias_tri_lds(K, KP_), s, \
                       D0, K, M, Cz, dvalid, ws);                                          \
    return true;                                                                           \
  }
  if (g_bias_mode > 40 && g_bias_mode < 60 && K <= 44) {  // timing-only ablations
    const int abl = g_bias_mode - 40;
#define MFA_TRI_ABL(A_)                                                                      \
    if (abl == A_)                                                                         \
      hipLaunchKernelGGL((mc_bias_tri_kernel<44, A_>), dim3(D * M), dim3(64), bias_tri_lds(K, 44), \
                         s, D0, K, M, Cz, dvalid, ws);
    MFA_TRI_ABL(1) MFA_TRI_ABL(2) MFA_TRI_ABL(3) MFA_TRI_ABL(4) MFA_TRI_ABL(5) MFA_TRI_ABL(6)
    MFA_TRI_ABL(7) MFA_TRI_ABL(8) MFA_TRI_ABL(16)
#undef MFA_TRI_ABL
    return true;
  }
  MFA_TRI(8)
  MFA_TRI(16)
  MFA_TRI(24)
  MFA_TRI(32)
  MFA_TRI(44)
  MFA_TRI(48)
  MFA_TRI(64)
#undef MFA_TRI
  return false;
}

