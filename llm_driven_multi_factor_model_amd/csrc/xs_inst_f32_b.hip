// CS-WLS per-Q instantiations (float panels, Q = 6, 7, 8, 9): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(6, float)
MFA_XS_INSTANTIATE(7, float)
MFA_XS_INSTANTIATE(8, float)
MFA_XS_INSTANTIATE(9, float)
