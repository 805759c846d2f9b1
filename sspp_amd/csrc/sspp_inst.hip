// sspp_inst.hip — one translation unit of kernel instantiations (see sspp_kern.h):
// -DSSPK_D=d (d in 1,2,3,4,6,7,9) instantiates the SamplingPathPlanner kernels of dof d,
// -DSSPK_D=0 the TaskSpacePlanner kernel.
#include "sspp_kern.h"

namespace sspk {
#if SSPK_D == 0
SSPK_TSP_DECL()
#else
SSPK_ENTRY_DECL(, SSPK_D)
#endif
}  // namespace sspk
