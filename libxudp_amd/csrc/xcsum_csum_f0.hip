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

#ifdef XCSUM_WAVE_STAMPS
/* the plain kernels' wave stamps (start, end per wave; 0 = no such wave);
 * clear != 0 zeroes them after the copy.  Synchronous. */
extern "C" int xcsum_wave_stamps(uint64_t *host, uint32_t nwaves, int clear)
{
	if (nwaves > xcsum::WAVE_STAMPS_MAX)
		nwaves = xcsum::WAVE_STAMPS_MAX;
	if (hipDeviceSynchronize() != hipSuccess)
		return -1;
	if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(xcsum::g_wave_stamps),
					2 * sizeof(uint64_t) * nwaves) != hipSuccess)
		return -1;
	if (clear) {
		void *p = nullptr;
		if (hipGetSymbolAddress(&p, HIP_SYMBOL(xcsum::g_wave_stamps)) != hipSuccess ||
		    hipMemset(p, 0, sizeof(xcsum::g_wave_stamps)) != hipSuccess)
			return -1;
	}
	return 0;
}
#endif
