// CS-WLS per-Q instantiations (double panels, Q = 1, 2, 3, 4, 5): one translation unit per
// Q group so the build compiles them in parallel (kernels: xs_wls_impl.h; entry points:
// xs_wls_f64.hip).
#include "xs_wls_impl.h"

MFA_XS_INSTANTIATE(1, double)
MFA_XS_INSTANTIATE(2, double)
MFA_XS_INSTANTIATE(3, double)
MFA_XS_INSTANTIATE(4, double)
MFA_XS_INSTANTIATE(5, double)
