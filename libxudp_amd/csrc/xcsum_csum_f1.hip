/* xcsum_csum_f1.hip -- csum_kernel<G, U, K, 1> for every compiled geometry:
 * + VERIFY (udp->len and udp->check prefetched a step ahead).  One translation unit per feature set (xcsum_csum.h). */
#include "xcsum_csum.h"

namespace xcsum {

hipError_t launch_csum_f1(const CsumArgs &a, Geometry g, int cus, hipStream_t s)
{
#define X(g_, u_, k_) \
	if (g.G == g_ && g.U == u_ && g.K == k_) return launch_t<g_, u_, k_, 1>(a, cus, g.B, s);
	XCSUM_GEOMETRIES(X)
#undef X
	return hipErrorInvalidValue;
}

} /* namespace xcsum */
