// sspp_inst.hip — one translation unit of kernel instantiations (see sspp_kern.h):
// -DSSPK_D=d -DSSPK_P=p (d in 1,2,3,4,6,7,9; p in 2,3) instantiates the SamplingPathPlanner
// kernels of dof d and spline degree p, -DSSPK_D=0 the TaskSpacePlanner kernel.
#include "sspp_kern.h"

namespace sspk {
#if SSPK_D == 0
SSPK_TSP_DECL()
#else
SSPK_ENTRY_DECL(, SSPK_D, SSPK_P)
#endif
}  // namespace sspk
