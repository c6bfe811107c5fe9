/* xcsum_csum_f0.hip -- csum_kernel<G, U, K, 0> for every compiled geometry:
 * plain (INPLACE, V4_RFC, AUTO).  One translation unit per feature set (xcsum_csum.h). */
#include "xcsum_csum.h"

namespace xcsum {

hipError_t launch_csum_f0(const CsumArgs &a, Geometry g, int cus, hipStream_t s)
{
#define X(g_, u_, k_) \
	if (g.G == g_ && g.U == u_ && g.K == k_) return launch_t<g_, u_, k_, 0>(a, cus, g.B, s);
	XCSUM_GEOMETRIES(X)
	XCSUM_SWEEP_GEOMETRIES(X)
#undef X
	return hipErrorInvalidValue;
}

} /* namespace xcsum */
