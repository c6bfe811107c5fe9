/* xcsum_csum_tl.hip -- csum_kernel_tl<16, 2, 6, 0, 4>: the MTU frame-group
 * kernel for XCSUM_F_INPLACE without XCSUM_F_IPHDR (IPv6, or IPv4 with only
 * udp->check), each frame's first 4 chunks -- the one holding udp->check
 * among them (eth+40: chunk 0-1, eth+60: chunk 2-3) -- loaded temporally, so
 * the in-place store finds its line in L2.  Config 4 in place 0.331 / 0.333
 * -> 0.327 / 0.327 ms (same box, two alternating runs,
 * profiles/r04/inplace/r04g_c4_*.log).  With IPHDR the IPv4 header load is
 * temporal already and the extra temporal chunks cost: 0.341 -> 0.362 ms
 * (r04g_c2_tl2_*.log), so that instantiation is not built. */
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

/* the in-place MTU launch without IPHDR (the caller checks the geometry) */
hipError_t launch_csum_inplace_tl(const CsumArgs &a, Geometry g, int cus, hipStream_t s)
{
	if (!(g.G == 16 && g.U == 2 && g.K == 6) || (a.flags & (XCSUM_F_VERIFY | XCSUM_F_IPHDR)))
		return hipErrorInvalidValue;
	return launch_tl_t<16, 2, 6, 0, 4>(a, cus, g.B, s);
}

} /* namespace xcsum */
