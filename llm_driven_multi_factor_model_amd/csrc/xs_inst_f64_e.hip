// CS-WLS per-Q instantiations (double panels, Q = 14, 15, 16): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls_f64.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(14, double)
MFA_XS_INSTANTIATE(15, double)
MFA_XS_INSTANTIATE(16, double)
