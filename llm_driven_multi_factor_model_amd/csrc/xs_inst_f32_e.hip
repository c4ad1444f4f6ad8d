// CS-WLS per-Q instantiations (float panels, Q = 14, 15, 16): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(14, float)
MFA_XS_INSTANTIATE(15, float)
MFA_XS_INSTANTIATE(16, float)
