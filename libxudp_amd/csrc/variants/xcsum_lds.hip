/*
 * variants/xcsum_lds.hip -- the LDS-DMA staged checksum kernel (A/B only,
 * not in libxcsum.so) and the variant dispatch the product library reaches
 * through its weak hooks.  Register staging measured 3-4 % faster at MTU
 * (profiles/r01/sweep_lds_vs_reg_config{2,4}.log).
 */
#include "xcsum_csum.h"
#include "xcsum_variants.h"

namespace xcsum {
/* ---- LDS-staged variant ---------------------------------------------------
 * Same arithmetic, chunks moved by LDS-DMA (gfx950 global_load_lds_dwordx4:
 * per-lane global address, 1 KiB per wave-instruction landing contiguously
 * in LDS) into a D-deep ring of K-slot stages per wave, read back with
 * ds_read_b128.  In-flight chunks hold LDS instead of VGPRs, so a wave keeps
 * D iterations of loads in flight.  G = 16: a wave's 4 frames per iteration
 * are consecutive, so their descriptors come from wave-uniform scalar loads
 * (lgkmcnt) and the vmcnt queue holds only the DMAs -- the wait for stage d
 * is then exactly vmcnt((D-1)*K).  The compiler does not order ds_read after
 * LDS-DMA, so the waits are explicit and fenced with sched_barrier. */
#define WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | 0x70 | 0xF00)
#define WAIT_LGKM0() __builtin_amdgcn_s_waitcnt(0xC07F)

typedef __attribute__((address_space(3))) void lds_void;

static __device__ __forceinline__ u32x4 load_desc_scalar(const CsumArgs &a, uint32_t p)
{
	uint32_t q = p < a.n ? p : a.n - 1;
	q = __builtin_amdgcn_readfirstlane(q);
	return *((cu32x4 *)(a.desc + q));
}

template <int K, int D>
__global__ void __launch_bounds__(256) csum_lds_kernel(CsumArgs a)
{
	constexpr int G = 16;
	extern __shared__ u32x4 lds_ring[];  /* [4 waves][D][K][64] */
	const uint32_t wave = threadIdx.x >> 6;
	const uint32_t lw = threadIdx.x & 63;
	const uint32_t lane = lw & (G - 1);
	const uint32_t sub = lw >> 4;                  /* frame of the wave: 0..3 */
	const uint32_t nwave = gridDim.x * 4;
	const uint32_t wave_id = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
	u32x4 *ring = lds_ring + (size_t)wave * D * K * 64;
	const uint8_t *zero = (const uint8_t *)g_zero_chunk;
	/* iteration j of this wave covers frames 4*(wave_id + j*nwave) + 0..3 */
	auto frame0 = [&](uint32_t j) { return 4u * (wave_id + j * nwave); };
	auto pick = [&](u32x4 d0, u32x4 d1, u32x4 d2, u32x4 d3) {
		u32x4 d = d0;
		d = sub == 1 ? d1 : d;
		d = sub == 2 ? d2 : d;
		d = sub == 3 ? d3 : d;
		return d;
	};
	auto resolve_j = [&](uint32_t j) {
		uint32_t f = frame0(j);
		u32x4 d = pick(load_desc_scalar(a, f), load_desc_scalar(a, f + 1),
			       load_desc_scalar(a, f + 2), load_desc_scalar(a, f + 3));
		return resolve<Grid<G, K>::DW, 2>(a, d, f + sub < a.n);
	};
	auto issue_stage = [&](const Frame &f, int slot) {
#pragma unroll
		for (int k = 0; k < K; k++) {
			uint32_t c = lane + k * G;
			const uint8_t *src = c < f.nchunks ? f.base + 16u * c : zero;
			__builtin_amdgcn_global_load_lds((gu32x4 *)src,
							 (lds_void *)(ring + (slot * K + k) * 64), 16, 0,
							 2);
		}
	};

	if (frame0(0) >= a.n)
		return;
	Frame fs[D];
#pragma unroll
	for (int d = 0; d < D; d++) {
		fs[d] = resolve_j(d);
		WAIT_LGKM0();
		__builtin_amdgcn_sched_barrier(0);
		issue_stage(fs[d], d);
	}
	for (uint32_t j0 = 0; frame0(j0) < a.n; j0 += D) {
#pragma unroll
		for (int d = 0; d < D; d++) {
			const uint32_t j = j0 + d;
			if (frame0(j) >= a.n)
				break;
			/* next frames of this stage (descriptors: scalar loads) */
			Frame fn = resolve_j(j + D);
			__builtin_amdgcn_sched_barrier(0);
			WAIT_VM((D - 1) * K);                  /* stage d has landed */
			__builtin_amdgcn_sched_barrier(0);
			u32x4 v[K];
#pragma unroll
			for (int k = 0; k < K; k++)
				v[k] = ring[(d * K + k) * 64 + lw];
			WAIT_LGKM0();                          /* reads done: slot reusable */
			__builtin_amdgcn_sched_barrier(0);
			issue_stage(fn, d);
			__builtin_amdgcn_sched_barrier(0);
			const Frame &f = fs[d];
			uint32_t E = 0, O = 0;
			if (__builtin_amdgcn_ballot_w64(f.nchunks > K * G))
				sum_walk<G, Grid<G, K>::DW>(f, lane, E, O);
			else
				sum_frame<G, K, 2, Grid<G, K>::DW>(f, v, lane, E, O);
			uint32_t sum = f.odd ? (O << 8) + E : (E << 8) + O;
			sum = seg_sum<G>(sum);
			if (lane == 0 && f.mode != -2)
				finalize<2>(a, f, frame0(j) + sub, sum);
			fs[d] = fn;
		}
	}
	WAIT_VM(0);  /* drain the DMAs still in flight before the wave exits */
}

template <int K, int D>
static hipError_t launch_lds_t(const CsumArgs &a, int cus, int bpc, hipStream_t s)
{
	const size_t lds = (size_t)4 * D * K * 64 * 16;
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [&] {
		int nb = 0;
		(void)hipFuncSetAttribute((const void *)csum_lds_kernel<K, D>,
					  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, csum_lds_kernel<K, D>, 256,
								 lds) != hipSuccess || nb <= 0)
			nb = 1;
		return nb;
	});
	int per_cu = (bpc > 0 && bpc < occ) ? bpc : occ;
	uint64_t waves = ((uint64_t)a.n + 3) / 4;
	uint64_t blocks = (waves + 3) / 4;
	uint64_t cap = (uint64_t)cus * per_cu;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();  /* clear a stale error (e.g. hipErrorNotReady from
	                           * someone's hipEventQuery) before checking ours */
	hipLaunchKernelGGL((csum_lds_kernel<K, D>), dim3((unsigned)blocks), dim3(256), lds, s, a);
	return hipGetLastError();
}


bool variant_supported(Geometry g)
{
	if (g.G == 16 && ((g.U == 12 || g.U == 13) && g.K == 6))
		return true;
	if (g.G == 16 && ((g.U == 12 || g.U == 14) && g.K == 3))
		return true;
#define X(f_, d_) if (g.G == 64 && g.U == f_ && (g.K == d_ || g.K == 100 + d_)) return true;
	XCSUM_SEG_GEOMETRIES(X)
#undef X
	return false;
}

hipError_t launch_variant(const CsumArgs &a, Geometry g, int cus, hipStream_t s)
{
	/* segmented stream: G = 64 lanes, U = frames per unit, K = rows in flight */
	if (g.G == 64)
		return launch_seg(a, g.U, g.K, cus, g.B, s);
	/* LDS-staged: G = 16, U = 10 + ring depth; identity order */
	CsumArgs b = a;
	b.ord = order_identity(a.n);
	b.dense = b.ord;
	if (g.U == 12 && g.K == 6) return launch_lds_t<6, 2>(b, cus, g.B, s);
	if (g.U == 13 && g.K == 6) return launch_lds_t<6, 3>(b, cus, g.B, s);
	if (g.U == 14 && g.K == 3) return launch_lds_t<3, 4>(b, cus, g.B, s);
	if (g.U == 12 && g.K == 3) return launch_lds_t<3, 2>(b, cus, g.B, s);
	return hipErrorInvalidValue;
}

} /* namespace xcsum */

/* present only in variant libraries: the Python binding adds the A/B
 * geometries to its sweep lists when it finds this symbol */
extern "C" int xcsum_variants_built(void)
{
	return 1;
}
