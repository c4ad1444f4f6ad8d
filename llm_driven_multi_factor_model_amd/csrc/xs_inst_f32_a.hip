// CS-WLS per-Q instantiations (float panels, Q = 1, 2, 3, 4, 5): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(1, float)
MFA_XS_INSTANTIATE(2, float)
MFA_XS_INSTANTIATE(3, float)
MFA_XS_INSTANTIATE(4, float)
MFA_XS_INSTANTIATE(5, float)
