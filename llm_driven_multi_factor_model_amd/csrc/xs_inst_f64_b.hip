// CS-WLS per-Q instantiations (double panels, Q = 6, 7, 8, 9): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls_f64.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(6, double)
MFA_XS_INSTANTIATE(7, double)
MFA_XS_INSTANTIATE(8, double)
MFA_XS_INSTANTIATE(9, double)
