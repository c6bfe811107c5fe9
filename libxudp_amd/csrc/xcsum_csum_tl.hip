/* xcsum_csum_tl.hip -- in-place A/B (XCSUM_INPLACE_TL=<chunks>):
 * csum_kernel_tl<16, 2, 6, FEAT, TL>, the MTU frame-group kernel with each
 * frame's first TL chunks (those holding udp->check: chunk 0-1 for IPv4,
 * 2-3 for IPv6) loaded temporally, so the in-place store finds its line in
 * the caches.  FEAT 0 (IPv6, no IP header) and 2 (IPv4 + IPHDR). */
#include "xcsum_csum.h"

namespace xcsum {

template <int G, int U, int K, int FEAT, int TL>
__global__ void __launch_bounds__(256) csum_kernel_tl(CsumArgs a)
{
	csum_body<G, U, K, FEAT, TL>(a);
}

template <int G, int U, int K, int FEAT, int TL>
static hipError_t launch_tl_t(const CsumArgs &a, int cus, int bpc, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, csum_kernel_tl<G, U, K, FEAT, TL>, 256,
								 0) != hipSuccess || nb <= 0)
			nb = 4;
		return nb;
	});
	const int per_cu = (bpc > 0 && bpc < occ) ? bpc : occ;
	uint64_t segs = ((uint64_t)a.ord.nlog + U - 1) / U;
	uint64_t blocks = (segs * G + 255) / 256;
	const uint64_t cap = (uint64_t)cus * per_cu;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();
	hipLaunchKernelGGL((csum_kernel_tl<G, U, K, FEAT, TL>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

hipError_t launch_csum_tl(const CsumArgs &a, Geometry g, int tl, int cus, hipStream_t s)
{
	if (!(g.G == 16 && g.U == 2 && g.K == 6) || (a.flags & XCSUM_F_VERIFY))
		return hipErrorInvalidValue;
	const bool iph = (a.flags & XCSUM_F_IPHDR) != 0;
	if (tl == 2)
		return iph ? launch_tl_t<16, 2, 6, 2, 2>(a, cus, g.B, s)
			   : launch_tl_t<16, 2, 6, 0, 2>(a, cus, g.B, s);
	if (tl == 4)
		return iph ? launch_tl_t<16, 2, 6, 2, 4>(a, cus, g.B, s)
			   : launch_tl_t<16, 2, 6, 0, 4>(a, cus, g.B, s);
	return hipErrorInvalidValue;
}

} /* namespace xcsum */
