// 3D double (f64) kernels: the launch.h launchers of this type (launch_impl.h), compiled apart
// from the host shim and from the other types.
#include "launch_impl.h"

namespace zfp_amd {
ZFP_DEFINE3(double)
}  // namespace zfp_amd
