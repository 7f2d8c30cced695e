// fmha_bwd.hip — backward instantiations (placeholder until the bwd kernels land).
#include "fmha_launch.h"

#define XFA_CAT2(a, b) a##b
#define XFA_CAT(a, b) XFA_CAT2(a, b)
#define XFA_FN(hd, dt) XFA_CAT(XFA_CAT(XFA_CAT(launch_bwd_hd, hd), _), dt)

namespace xfa {
hipError_t XFA_FN(XFA_HD, XFA_DTN)(const BwdParams&, hipStream_t) { return hipErrorNotSupported; }
}  // namespace xfa
