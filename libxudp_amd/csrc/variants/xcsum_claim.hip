/* xcsum_claim.hip -- A/B only (`make variant`, not in libxcsum.so): the
 * claimed-tail schedule of the frame-group checksum kernel,
 * csum_kernel_claim<G, U, K, FEAT> (csrc/xcsum_csum.h), per feature set.
 * Measured in round 6 against the static schedule (DESIGN.md 9.4,
 * profiles/r06/tail/): it removes the persistent grid's tail (config 5
 * occupancy loss 5.1 % -> 0.4 %) but gains at most 1.5 % on the full 8M-frame
 * job and loses on one rank's 1M-frame shard (-2 to -4 %) and on config 2
 * (-7 %): the bandwidth the early waves free is taken by the others. */
#include "xcsum_csum.h"

namespace xcsum {

#define CLAIM_LAUNCHER(NAME, FEAT)                                                            \
	hipError_t NAME(const CsumArgs &a, Geometry g, int cus, const ClaimParams &cp,         \
			hipStream_t s)                                                         \
	{                                                                                      \
		CLAIM_DISPATCH(FEAT)                                                           \
		return hipErrorNotSupported;                                                   \
	}
#define X(g_, u_, k_, feat_)                                                                  \
	if (g.G == g_ && g.U == u_ && g.K == k_)                                              \
		return launch_claim_t<g_, u_, k_, feat_>(a, cus, g.B, cp.claim, cp.static_64,  \
							 cp.chunk_steps, s);
#define X0(g_, u_, k_) X(g_, u_, k_, 0)
#define X1(g_, u_, k_) X(g_, u_, k_, 1)
#define X2(g_, u_, k_) X(g_, u_, k_, 2)
#define CLAIM_DISPATCH(FEAT) XCSUM_CLAIM_GEOMETRIES(X##FEAT)

CLAIM_LAUNCHER(launch_csum_claim_f0, 0)
CLAIM_LAUNCHER(launch_csum_claim_f1, 1)
CLAIM_LAUNCHER(launch_csum_claim_f2, 2)

} /* namespace xcsum */
