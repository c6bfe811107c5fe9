/*
 * xcsum_seg.hip -- the checksum kernel for packed batches of large or mixed
 * frames (config 5: payloads U[64, 9000] back to back): a segmented stream.
 *
 * Why a third kernel.  The frame-group kernel gives each frame G lanes x K
 * preloaded chunks; for mixed sizes that grid must fit the largest frame
 * (G = 64, K = 9: 9 KB), so an average 4.5 KB frame leaves half the loaded
 * registers holding zero chunks, and the bytes a CU keeps in flight -- what
 * sets HBM throughput here -- are half what the registers could hold.  The
 * stream kernel (xcsum_kernels.hip) stages a 64-frame region in LDS, which
 * only fits small frames.
 *
 * Here a wave takes 64 consecutive descriptors (a unit; lane = frame) and
 * reads the region their spans occupy as rows of 1 KiB -- 16 aligned bytes
 * per lane, one coalesced load instruction per row -- with D rows in flight
 * in a register ring that runs on across units without draining.  Spans are
 * disjoint and sorted in a packed batch and the gap between two spans (the
 * next frame's Ethernet and IP header bytes up to the addresses) is >= 22
 * bytes, so a 16-byte chunk meets at most one span: every lane adds its
 * chunk's bytes of the current frame to running even/odd byte sums (the
 * same exact v_dot4_u32_u8 sums as the other kernels), unmasked on rows a
 * span covers whole, masked on rows where a span starts or ends.  When a
 * span ends the wave reduces the sums (DPP + permlane swaps) and hands the
 * total to the frame's lane; after the unit's last row every lane finalizes
 * its frame exactly as the other kernels do (finalize<2>).
 *
 * A unit whose spans are not sorted and disjoint, or whose region is not
 * dense (more than 8 MiB), is walked frame by frame from global memory
 * instead (results identical, only slower); a sparse batch (xudp's 4096-byte
 * slots) runs the frame-group kernel (checked once per launch, dense_batch).
 */
#include "xcsum_csum.h"
#include "xcsum_variants.h"

namespace xcsum {

namespace {

constexpr uint64_t SEG_MAX_REGION = 1ull << 23;   /* bytes per unit, else walked */


struct UnitBounds {
	uint64_t base;   /* UMEM offset of the region's first row (16-aligned) */
	uint32_t len;    /* region bytes from base (0: walk the unit) */
	uint32_t rows;   /* 1 KiB rows */
	uint32_t slots;  /* rows rounded up to the ring depth D: every unit starts
			    at ring slot 0, so the row loop indexes the ring
			    statically and unit switches stay outside it */
};

/* Region of a unit from its first frame's offset and its last present
 * frame's end (UMEM offsets).  Both the issue and the consume side compute
 * it, from the same descriptors: the ring stays in step. */
template <int D>
static __device__ __forceinline__ UnitBounds unit_bounds(uint64_t e0, uint64_t el)
{
	UnitBounds b;
	b.base = (e0 + 22u) & ~15ull;
	if (el <= b.base || el - b.base > SEG_MAX_REGION) {
		b.len = 0;
		b.rows = 0;
	} else {
		b.len = (uint32_t)(el - b.base);
		b.rows = (b.len + 1023u) >> 10;
	}
	b.slots = (b.rows + D - 1) / D * D;
	return b;
}

/* bytes [lo, hi) of a 16-byte chunk (both clamped to [0, 16]), the rest 0 */
static __device__ __forceinline__ u32x4 keep_bytes(u32x4 v, int lo, int hi)
{
	lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
	hi = hi < lo ? lo : (hi > 16 ? 16 : hi);
	auto first = [](int n, uint64_t &m0, uint64_t &m1) {   /* bytes [0, n) */
		m0 = n >= 8 ? ~0ull : (1ull << (8 * n)) - 1ull;
		m1 = n <= 8 ? 0ull : (n >= 16 ? ~0ull : (1ull << (8 * (n - 8))) - 1ull);
	};
	uint64_t h0, h1, l0, l1;
	first(hi, h0, h1);
	first(lo, l0, l1);
	const uint64_t k0 = h0 & ~l0, k1 = h1 & ~l1;
	v.x &= (uint32_t)k0;
	v.y &= (uint32_t)(k0 >> 32);
	v.z &= (uint32_t)k1;
	v.w &= (uint32_t)(k1 >> 32);
	return v;
}

} /* namespace */

/* ATOM (round 6): a finished span's per-lane sums go to the frame's word in
 * LDS by one ds_add per lane instead of a wave reduction (DPP + permlane
 * swaps) -- no dependency chain per frame; the unit's words are read back
 * once by their lanes */
template <int D, int F, bool ATOM>
__global__ void __launch_bounds__(256) csum_seg_kernel(CsumArgs a)
{
	__shared__ uint32_t lds_acc[ATOM ? 4 : 1][ATOM ? F : 1];
	if (!dense_batch(a)) {
		/* sparse batch: the frame-group kernel, region order as usual
		 * (K = 2: its registers set this kernel's occupancy; frames over
		 * 2 KiB take its walk) */
		csum_body<64, 1, 2, 2>(a);
		return;
	}
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t nw = gridDim.x * 4u;
	const uint32_t nunits = (uint32_t)(((uint64_t)a.n + F - 1) / F);
	const uint8_t *zero = (const uint8_t *)g_zero_chunk;
	const uint32_t w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
	const uint32_t wv = ATOM ? threadIdx.x >> 6 : 0u;

	/* scalar (wave-uniform) bounds of unit u from two descriptors */
	auto bounds_of = [&](uint32_t u) __attribute__((always_inline)) {
		const uint32_t p0 = (uint32_t)F * u;
		const uint32_t pl = p0 + (F - 1) < a.n ? p0 + (F - 1) : a.n - 1u;
		const u32x4 d0 = *((cu32x4 *)(a.desc + p0));
		const u32x4 dl = *((cu32x4 *)(a.desc + pl));
		const uint64_t e0 = (((uint64_t)d0.y << 32) | d0.x) - a.bias;
		const uint64_t el = (((uint64_t)dl.y << 32) | dl.x) - a.bias + dl.z;
		return unit_bounds<D>(e0, el);
	};

	/* ---- issue side: ring slots in unit order (walked units have none;
	 * slots past a unit's rows load the zero chunk) ---- */
	uint32_t iu = w0, iu2 = w0 + nw;
	uint32_t irow = 0;
	UnitBounds ib = iu < nunits ? bounds_of(iu) : UnitBounds{0, 0, 0, 0};
	UnitBounds ib2 = iu2 < nunits ? bounds_of(iu2) : UnitBounds{0, 0, 0, 0};
	auto issue = [&](u32x4 &v) __attribute__((always_inline)) {
		while (iu < nunits && irow >= ib.slots) {
			iu = iu2;
			ib = ib2;
			irow = 0;
			iu2 = iu + nw;
			if (iu2 < nunits)
				ib2 = bounds_of(iu2);
		}
		const uint32_t off = irow * 1024u + 16u * lane;
		const bool ok = iu < nunits && off < ib.len;
		v = load_chunk(ok ? a.umem + ib.base + off : zero);
		irow++;
	};

	/* ---- consume side ---- */
	uint32_t cu = w0;
	if (cu >= nunits)
		return;
	u32x4 dcur = *((gu32x4 *)(a.desc + (F * cu + lane < a.n ? F * cu + lane : a.n - 1u)));
	u32x4 dnext = dcur;
	Frame f;
	UnitBounds cb = {0, 0, 0, 0};
	uint32_t s_rel = 0, h_rel = 0, acc = 0, E = 0, O = 0;
	uint32_t cf = F;
	uint32_t sc = 0, hc = 0, oddc = 0;
	bool cwalk = false, cvalid = true;

	/* every lane finalizes its frame (the unit's sums are complete) */
	auto finish_unit = [&]() __attribute__((always_inline)) {
		if (cwalk)
			return;
		/* frames never reached by a row (no span in the region) flush 0 */
		const uint32_t p = F * cu + lane;
		if (ATOM && lane < (uint32_t)F)
			acc = lds_acc[wv][lane];
		if (f.mode != -2)
			finalize<2>(a, f, p, acc);
	};
	/* set up unit cu (dcur holds its descriptors); walked units are done here */
	auto start_unit = [&]() __attribute__((always_inline)) {
		const uint32_t p = F * cu + lane;
		const bool present = lane < F && p < a.n;
		f = resolve<false, 2>(a, dcur, present);
		/* the next unit's descriptors, used at its start */
		const uint32_t pn = F * (cu + nw) + lane;
		dnext = *((gu32x4 *)(a.desc + (pn < a.n ? pn : a.n - 1u)));
		/* region bounds from lanes 0 and the last present lane */
		const uint32_t last = a.n - F * cu > (uint32_t)F ? F - 1u : a.n - F * cu - 1u;
		const uint64_t e = (((uint64_t)dcur.y << 32) | dcur.x) - a.bias;
		const uint64_t el_lane = e + dcur.z;
		const uint64_t e0 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(e >> 32), 0) << 32) |
				    (uint32_t)__builtin_amdgcn_readlane((uint32_t)e, 0);
		const uint64_t el =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(el_lane >> 32), last) << 32) |
			(uint32_t)__builtin_amdgcn_readlane((uint32_t)el_lane, last);
		cb = unit_bounds<D>(e0, el);
		/* the lane's span [s_rel, h_rel) relative to the region base; no
		 * span: an empty one at its frame's place (keeps the order) */
		const int64_t eo = (int64_t)(e - cb.base);
		const uint32_t hdr = f.mode == 2 ? 54u : 34u, pre = f.mode == 2 ? 32u : 8u;
		int64_t s64, h64;
		if (f.nchunks && present) {
			s64 = eo + (int64_t)(hdr - pre);
			h64 = s64 + (int64_t)(pre + f.udp_len);
		} else {
			s64 = present ? eo + 22 : (int64_t)cb.len;
			s64 = s64 < 0 ? 0 : (s64 > (int64_t)cb.len ? (int64_t)cb.len : s64);
			h64 = s64;
		}
		/* sorted and disjoint, inside the region */
		const uint32_t prev_h = (uint32_t)__builtin_amdgcn_ds_bpermute(
			(int)((lane ? lane - 1u : 0u) << 2), (int)(uint32_t)(h64 < 0 ? 0 : h64));
		const bool bad = s64 < 0 || h64 > (int64_t)cb.len || h64 < s64 ||
				 (lane > 0 && (uint64_t)s64 < prev_h);
		cwalk = cb.rows == 0 || __builtin_amdgcn_ballot_w64(bad) != 0;
		s_rel = (uint32_t)(s64 < 0 ? 0 : s64);
		h_rel = (uint32_t)(h64 < 0 ? 0 : h64);
		acc = 0;
		if (ATOM && lane < (uint32_t)F)
			lds_acc[wv][lane] = 0u;
		E = 0;
		O = 0;
		cf = 0;
		sc = __builtin_amdgcn_readlane(s_rel, 0);
		hc = __builtin_amdgcn_readlane(h_rel, 0);
		oddc = __builtin_amdgcn_readlane(f.odd, 0);
		if (cwalk) {
			/* the whole wave walks each frame from global memory */
			for (uint32_t i = 0; i < (uint32_t)F; i++) {
				const uint32_t q = F * cu + i;
				if (q >= a.n)
					break;
				const u32x4 di = *((cu32x4 *)(a.desc + q));
				const Frame g = resolve<false, 2>(a, di, true);
				uint32_t Ew = 0, Ow = 0;
				sum_walk<64, false>(g, lane, Ew, Ow);
				uint32_t s = g.odd ? (Ow << 8) + Ew : (Ew << 8) + Ow;
				s = seg_sum<64>(s);
				if (lane == 0)
					finalize<2>(a, g, q, s);
			}
		}
	};
	auto next_unit = [&]() __attribute__((always_inline)) {
		finish_unit();
		cu += nw;
		if (cu >= nunits) {
			cvalid = false;
			return;
		}
		dcur = dnext;
		start_unit();
	};
	/* frame cf's span is complete: its lane takes the wave's total */
	auto flush = [&]() __attribute__((always_inline)) {
		uint32_t s = oddc ? (O << 8) + E : (E << 8) + O;
		if (ATOM) {
			if (s)
				atomicAdd(&lds_acc[wv][cf], s);
		} else {
			s = seg_sum<64>(s);
			acc = lane == cf ? s : acc;
		}
		E = 0;
		O = 0;
		cf++;
		if (cf < (uint32_t)F) {
			sc = __builtin_amdgcn_readlane(s_rel, (int)cf);
			hc = __builtin_amdgcn_readlane(h_rel, (int)cf);
			oddc = __builtin_amdgcn_readlane(f.odd, (int)cf);
		}
	};
	auto process = [&](const u32x4 &v, uint32_t row) __attribute__((always_inline)) {
		const uint32_t rs = row * 1024u, re = rs + 1024u;
		if (cwalk || cf >= (uint32_t)F || row >= cb.rows)
			return;
		if (sc <= rs && hc >= re) {   /* a span covers the whole row */
			accum(v, E, O);
			if (hc == re)
				flush();
			return;
		}
		const int o = (int)(rs + 16u * lane);
		for (;;) {
			if (sc < re && hc > rs)
				accum(keep_bytes(v, (int)sc - o, (int)hc - o), E, O);
			if (hc > re)
				break;             /* the span goes on into the next row */
			flush();
			if (cf >= (uint32_t)F || sc >= re)
				break;
		}
	};

	start_unit();
	while (cvalid && cb.slots == 0)
		next_unit();
	if (!cvalid)
		return;

	u32x4 v[D];
#pragma unroll
	for (int d = 0; d < D; d++)
		issue(v[d]);
	while (cvalid) {
		for (uint32_t r = 0; r < cb.slots; r += D) {
#pragma unroll
			for (int d = 0; d < D; d++) {
				process(v[d], r + d);
				issue(v[d]);
			}
		}
		/* frames of the unit no row reached: empty spans */
		while (!cwalk && cf < (uint32_t)F)
			flush();
		next_unit();
		while (cvalid && cb.slots == 0)
			next_unit();
	}
}

template <int D, int F, bool ATOM>
static hipError_t launch_seg_t(const CsumArgs &a, int cus, int bpc, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, csum_seg_kernel<D, F, ATOM>, 256, 0) !=
			    hipSuccess || nb <= 0)
			nb = 1;
		return nb;
	});
	const int per_cu = (bpc > 0 && bpc < occ) ? bpc : occ;
	/* a wave per F-frame unit; the sparse fallback sizes its own loop from
	 * the same grid (persistent, strided) */
	uint64_t blocks = ((uint64_t)a.n + 4 * F - 1) / (4 * F);
	const uint64_t cap = (uint64_t)cus * per_cu;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();
	hipLaunchKernelGGL((csum_seg_kernel<D, F, ATOM>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

/* segmented stream: Geometry{64, F, D}: F frames per unit (8..64), D rows
 * of 1 KiB in flight per wave */
hipError_t launch_seg(const CsumArgs &a, int F, int D, int cus, int bpc, hipStream_t s)
{
#define XCSUM_SEG(f_, d_) \
	if (F == f_ && D == d_) return launch_seg_t<d_, f_, false>(a, cus, bpc, s); \
	if (F == f_ && D == 100 + d_) return launch_seg_t<d_, f_, true>(a, cus, bpc, s);
	XCSUM_SEG_GEOMETRIES(XCSUM_SEG)
#undef XCSUM_SEG
	return hipErrorInvalidValue;
}

} /* namespace xcsum */
