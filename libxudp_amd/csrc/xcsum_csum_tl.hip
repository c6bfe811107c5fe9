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

/* B64 (inplace_blocks(), xcsum_csum.h): two waves per SIMD, as the plain
 * kernels -- the copy with IPHDR and the chunk below the grid otherwise
 * allocates 264 registers and runs one */
template <int G, int U, int K, int FEAT, int TL, int B64>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
csum_kernel_b64(CsumArgs a)
{
	csum_body<G, U, K, FEAT, TL, B64>(a);
}

template <int G, int U, int K, int FEAT, int TL, int B64 = 0>
static hipError_t launch_tl_t(const CsumArgs &a, int cus, int bpc, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	auto kern = [] {
		if constexpr (B64 > 0)
			return csum_kernel_b64<G, U, K, FEAT, TL, B64>;
		else
			return csum_kernel_tl<G, U, K, FEAT, TL>;
	}();
	const int occ = occupancy_cached(occ_cache, [&] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, 0) != hipSuccess ||
		    nb <= 0)
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
	hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

/* the in-place MTU launch without IPHDR (the caller checks the geometry) */
hipError_t launch_csum_inplace_tl(const CsumArgs &a, Geometry g, int cus, hipStream_t s)
{
	if (!(g.G == 16 && g.U == 2 && g.K == 6) || (a.flags & (XCSUM_F_VERIFY | XCSUM_F_IPHDR)))
		return hipErrorInvalidValue;
	return launch_tl_t<16, 2, 6, 0, 4>(a, cus, g.B, s);
}

/* the in-place MTU launch with whole 64-byte block stores (inplace_blocks(),
 * xcsum_csum.h), with or without IPHDR; tl: the temporal-first-chunks loads
 * too (without IPHDR only) */
hipError_t launch_csum_inplace_b64(const CsumArgs &a, Geometry g, int cus, int tl, int pre,
				   hipStream_t s)
{
	if (!(g.G == 16 && g.U == 2 && g.K == 6) || !(a.flags & XCSUM_F_INPLACE) ||
	    (a.flags & XCSUM_F_VERIFY))
		return hipErrorInvalidValue;
	if (a.flags & XCSUM_F_IPHDR)
		return pre ? launch_tl_t<16, 2, 6, 2, 0, 2>(a, cus, g.B, s)
			   : launch_tl_t<16, 2, 6, 2, 0, 1>(a, cus, g.B, s);
	if (tl)
		return launch_tl_t<16, 2, 6, 0, 4, 2>(a, cus, g.B, s);
	return launch_tl_t<16, 2, 6, 0, 0, 2>(a, cus, g.B, s);
}

} /* namespace xcsum */
