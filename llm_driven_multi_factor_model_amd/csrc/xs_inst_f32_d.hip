// CS-WLS per-Q instantiations (float panels, Q = 11, 12, 13): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(11, float)
MFA_XS_INSTANTIATE(12, float)
MFA_XS_INSTANTIATE(13, float)
