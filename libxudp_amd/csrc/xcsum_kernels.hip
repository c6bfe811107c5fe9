/*
 * xcsum_kernels.hip -- gfx950 (CDNA4) kernels of the UDP checksum engine.
 *
 * What is computed (reference: cclinuxer/libxudp xudp/checksum.h and
 * xudp/packet.c).  Every frame xudp builds has no IP options / no IPv6
 * extension headers (packet.c:19-21, :99), so a frame's whole checksum input
 * is ONE contiguous span: the pseudo-header addresses sit right before the
 * UDP header.
 *     IPv4: span = [eth+26, eth+len)   (saddr, daddr, UDP header, payload)
 *     IPv6: span = [eth+22, eth+len)   (saddr, daddr, UDP header, payload)
 * Let S be the EXACT integer sum of the span's big-endian 16-bit words (odd
 * tail byte padded as a high byte) plus 17 + (udp_len >> 16) + (udp_len &
 * 0xffff).  S < 2^32 for udp_len <= 65535 and, being an exact integer sum, it
 * is independent of reduction order.  Then
 *     V4_LEGACY (checksum.h:100-104 udp_checksum): r = ~(u16)((S&0xffff)+(S>>16))
 *     V4_RFC / V6 (packet.c:105-117 udp_csum6):   r = ~fold(fold(S)), 0 -> 0xffff
 * and out = htons(r), the value stored into udp->check.  The legacy quirk
 * (the dropped end-around carry) is reproduced because S is exact.
 *
 * How (memory-bound integer reduction, no MFMA):
 *   - G lanes own one frame; each lane loads aligned 16-byte chunks
 *     (global_load_dwordx4, coalesced: the G lanes of a frame read G*16
 *     consecutive bytes per instruction); the bytes outside the span are
 *     taken back out only in the frame's first and last chunk;
 *   - per lane, two exact u32 sums with v_dot4_u32_u8: E = bytes at even
 *     addresses, O = bytes at odd addresses (2 VALU per dword);
 *     lane value = 256*E + O (or 256*O + E when the span starts odd);
 *   - G-lane reduction with DPP row ops and gfx950 v_permlane{16,32}_swap,
 *     lane 0 of the segment finalizes and stores 2 bytes.
 *   - persistent grid (<= 8 blocks/CU), frames strided over segments; each
 *     segment keeps U frames' loads in flight (K chunks per lane per frame
 *     preloaded), the rest of a jumbo frame streams in a tail loop.
 */
#include "xcsum_csum.h"
#include "xcsum_gen.h"
#include <stdlib.h>

namespace xcsum {
/* ---- stream kernel: packed batches of small frames -------------------------
 * A wave takes 64 consecutive descriptors (one per lane) and reads the UMEM
 * region their frames occupy -- [min eth, max end) -- as one coalesced stream:
 * chunk k*64 + lane of the region for k < KC (1 KiB per load instruction, no
 * per-frame chunk grid, no edge masks on the loads).  The chunks go to the
 * wave's LDS stage; then every lane sums ITS frame's span from LDS (16-byte
 * reads, the head/tail bytes taken back out once) and finalizes it.  The
 * frame boundaries are the descriptors, held one per lane: a segmented
 * reduction of the stream, done per lane instead of per chunk.
 * While one region is summed from LDS, the next region's loads are in flight
 * in registers (KC dwordx4 per lane), and the descriptors after it.
 * Header fields the finalize needs (h_proto for AUTO, udp->len / check for
 * VERIFY, the IPv4 header for IPHDR) come from the same LDS copy.
 * A wave whose frames do not fit in KC KiB (irregular batch, jumbo frame)
 * walks them from global memory, one frame per wave; a sparse batch (xudp's
 * 4096-byte slots) runs the frame-group kernel instead (checked once per
 * launch, like resolve_order). */

struct StreamSpan {
	uint64_t eth;       /* UMEM offset of the frame (desc.addr - bias) */
	uint32_t len;
	uint32_t present;   /* frame index < n */
};

/* the 4 LDS bytes at byte offset o (any alignment), little-endian */
static __device__ __forceinline__ uint32_t lds_bytes4(const uint8_t *st, uint32_t o)
{
	const uint32_t *w = (const uint32_t *)(st + (o & ~3u));
	return __builtin_amdgcn_alignbyte(w[1], w[0], o & 3u);
}

template <int KC>
static __device__ __forceinline__ void stream_loop(const CsumArgs &a, u32x4 *stage)
{
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t nw = gridDim.x * 4;
	const uint8_t *zero = (const uint8_t *)g_zero_chunk;
	const uint8_t *st8 = (const uint8_t *)stage;
	const uint32_t ngroups = (uint32_t)(((uint64_t)a.n + 63) >> 6);
	/* wave-iteration wi reads group wi: 64 frames in descriptor order */
	uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));

	auto span_of = [&](uint32_t wi, u32x4 d) {
		StreamSpan sp;
		const uint64_t p = 64ull * wi + lane;
		sp.present = p < a.n;
		sp.eth = ((((uint64_t)d.y << 32) | d.x) - a.bias);
		sp.len = d.z;
		return sp;
	};
	/* Region of a wave-iteration: base (16-aligned ADDRESS) and chunk
	 * count, or ~0u when the frames do not fit the stage.  The bounds are
	 * the first lane's frame start and the last present lane's frame end
	 * (two readlanes -- a packed batch is in UMEM order); every frame must
	 * then lie inside them (one ballot), else the wave walks its frames.
	 * Aligned as addresses, not as UMEM offsets: with a d_umem that is not
	 * 16-byte aligned, a region aligned as offsets would end up to 15 bytes
	 * past the 16-byte block of the last frame byte (another page,
	 * possibly unmapped), and every load would be misaligned. */
	auto region = [&](uint32_t wi, const StreamSpan &sp, uint64_t &base, uint32_t &nch) {
		const uint64_t rem = a.n - 64ull * wi;
		const uint32_t last = rem > 64 ? 63u : (uint32_t)rem - 1u;
		const uint64_t e = (uint64_t)(uintptr_t)(a.umem + sp.eth);
		const uint64_t end = e + sp.len;
		const uint64_t lo =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(e >> 32), 0) << 32) |
			(uint32_t)__builtin_amdgcn_readlane((uint32_t)e, 0);
		const uint64_t hi =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(end >> 32), last) << 32) |
			(uint32_t)__builtin_amdgcn_readlane((uint32_t)end, last);
		base = lo & ~15ull;
		const bool out = sp.present && (e < lo || end > hi);
		nch = (__builtin_amdgcn_ballot_w64(out) || hi < lo || hi - base > (uint64_t)KC * 1024u)
			      ? ~0u : (uint32_t)((hi - base + 15) >> 4);
	};
	auto issue_region = [&](const StreamSpan &sp, uint64_t base, uint32_t nch,
				u32x4 (&v)[KC]) {
		(void)sp;
#ifdef XCSUM_DEBUG_BOUNDS
		/* the 16-byte blocks of the present frames, computed apart from
		 * region(): min start / max end over the lanes */
		uint64_t mn = sp.present ? (uint64_t)(uintptr_t)(a.umem + sp.eth) : ~0ull;
		uint64_t mx = sp.present ? (uint64_t)(uintptr_t)(a.umem + sp.eth) + sp.len : 0ull;
		for (int o = 32; o; o >>= 1) {
			const uint64_t m2 = __shfl_xor(mn, o), x2 = __shfl_xor(mx, o);
			mn = m2 < mn ? m2 : mn;
			mx = x2 > mx ? x2 : mx;
		}
		const uint64_t ok_lo = mn & ~15ull, ok_hi = (mx + 15) & ~15ull;
#endif
#pragma unroll
		for (int k = 0; k < KC; k++) {
			const uint32_t c = (uint32_t)k * 64u + lane;
			v[k] = load_chunk(nch != ~0u && c < nch
						  ? XB_LOAD((const uint8_t *)(uintptr_t)(base + 16u * c), 16,
							    ok_lo, ok_hi, XB_STREAM_REGION, c, zero)
						  : zero);
		}
	};
	auto load_d = [&](uint32_t wi) {
		const uint64_t p = 64ull * wi + lane;
		return *((gu32x4 *)(a.desc + (p < a.n ? p : a.n - 1)));
	};

	if (w >= ngroups)
		return;
	u32x4 d = load_d(w);
	StreamSpan sc = span_of(w, d);
	uint64_t bc;
	uint32_t nc;
	region(w, sc, bc, nc);
	u32x4 v[KC];
	issue_region(sc, bc, nc, v);
	d = load_d(w + nw);
	for (; w < ngroups; w += nw) {
		/* this iteration's region -> LDS (waits for its loads only: the
		 * descriptors issued after them may still be in flight) */
#pragma unroll
		for (int k = 0; k < KC; k++)
			stage[k * 64 + lane] = v[k];
		const StreamSpan cur = sc;
		const uint64_t cbase = bc;
		const uint32_t cnch = nc;
		/* next iteration: its region's loads go out before this one is summed */
		if (w + nw < ngroups) {
			sc = span_of(w + nw, d);
			region(w + nw, sc, bc, nc);
			__builtin_amdgcn_sched_barrier(0);
			issue_region(sc, bc, nc, v);
			d = load_d(w + 2 * nw);
		}
		__builtin_amdgcn_sched_barrier(0);
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

		if (cnch == ~0u) {
			/* does not fit the stage: the whole wave walks each frame */
			for (uint32_t i = 0; i < 64; i++) {
				const uint64_t p64 = 64ull * w + i;
				if (p64 >= a.n)
					break;
				const uint32_t p = (uint32_t)p64;
				const u32x4 di = *((cu32x4 *)(a.desc + p));
				const Frame f = resolve<false, 2>(a, di, true);
				uint32_t E = 0, O = 0;
				sum_walk<64, false>(f, lane, E, O);
				uint32_t s = f.odd ? (O << 8) + E : (E << 8) + O;
				s = seg_sum<64>(s);
				if (lane == 0)
					finalize<2>(a, f, p, s);
			}
		} else if (cur.present) {
			/* lane = frame: everything from the LDS copy of the region */
			/* frame in the stage */
			const uint32_t oe = (uint32_t)((uint64_t)(uintptr_t)(a.umem + cur.eth) - cbase);
			Frame f;
			f.eth = a.umem + cur.eth;
#ifdef XCSUM_DEBUG_BOUNDS
			f.lim = (const uint8_t *)(((uintptr_t)f.eth + cur.len + 15u) & ~(uintptr_t)15);
			f.dlen = cur.len;
#endif
			int mode = (int)a.mode;
			if (mode == XCSUM_MODE_AUTO) {
				const uint32_t pr = lds_bytes4(st8, oe + 12) & 0xffffu;  /* h_proto, LE */
				mode = pr == 0x0008u ? ((a.flags & XCSUM_F_V4_RFC) ? 1 : 0)
				     : pr == 0xDD86u ? 2 : -1;
			}
			const uint32_t hdr = mode == 2 ? 54u : 34u, pre = mode == 2 ? 32u : 8u;
			if (mode < 0 || cur.len < hdr + 8u || cur.len - hdr > 65535u)
				mode = -1;
			f.udp_len = cur.len - hdr;
			f.ck = 0;
			if (mode >= 0 && (a.flags & XCSUM_F_VERIFY)) {
				const uint32_t uw = lds_bytes4(st8, oe + hdr + 4);  /* len, check */
				const uint32_t ul = bswap16(uw);
				f.ck = uw >> 16;
				f.ul = uw & 0xffffu;   /* finalize sees udp_len == ul: no re-cut */
				if (ul != f.udp_len) {
					if (ul < 8u || ul > f.udp_len)
						mode = -3;  /* never verifies */
					else
						f.udp_len = ul;
				}
			}
			f.mode = mode;
			uint32_t E = 0, O = 0;
			const uint32_t lo = oe + hdr - pre, hi = oe + hdr + f.udp_len;
			f.odd = lo & 1u;
			if (mode >= 0) {
				const uint32_t c0 = lo >> 4;
				uint32_t c1 = (hi + 15) >> 4;
				if (!XB_IDX(c1 - 1, (uint32_t)KC * 64u, XB_STREAM_STAGE))
					c1 = c0 + 1;
				for (uint32_t c = c0; c < c1; c++)
					accum(stage[c], E, O);
				drop_prefix(stage[c0], lo & 15u, E, O);
				drop_suffix(stage[c1 - 1], (16u - (hi & 15u)) & 15u, E, O);
				if (a.flags & XCSUM_F_IPHDR) {
					const uint32_t ih = oe + 14;
					f.ihs = ih & 3u;
#pragma unroll
					for (int j = 0; j < 6; j++)
						f.ih[j] = ((const uint32_t *)(st8 + (ih & ~3u)))[j];
				}
			}
			const uint32_t s = f.odd ? (O << 8) + E : (E << 8) + O;
			finalize<2>(a, f, 64u * w + lane, s);
		}
		/* the stage is rewritten next iteration: all reads done first */
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	}
}

template <int KC>
__global__ void __launch_bounds__(256) csum_stream_kernel(CsumArgs a)
{
	extern __shared__ u32x4 stream_stage[];   /* [4 waves][KC * 64] chunks */
	if (!dense_batch(a)) {
		/* sparse batch: the frame-group kernel, region order as usual */
		csum_body<4, 1, 2, 2>(a);
		return;
	}
	stream_loop<KC>(a, stream_stage + (threadIdx.x >> 6) * (KC * 64));
}

template <int KC>
static hipError_t launch_stream_t(const CsumArgs &a, int cus, int bpc, hipStream_t s)
{
	const size_t lds = (size_t)4 * KC * 64 * 16;
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [&] {
		int nb = 0;
		(void)hipFuncSetAttribute((const void *)csum_stream_kernel<KC>,
					  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, csum_stream_kernel<KC>, 256,
								 lds) != hipSuccess || nb <= 0)
			nb = 1;
		return nb;
	});
	const int per_cu = (bpc > 0 && bpc < occ) ? bpc : occ;
	/* a wave per 64 frames; the sparse fallback sizes its own loop from the
	 * same grid (persistent, strided) */
	uint64_t blocks = ((uint64_t)a.n + 255) / 256;
	const uint64_t cap = (uint64_t)cus * per_cu;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();
	hipLaunchKernelGGL((csum_stream_kernel<KC>), dim3((unsigned)blocks), dim3(256), lds, s, a);
	return hipGetLastError();
}

/* Geometry from the typical frame length (bytes): enough lanes x chunks to
 * cover a typical frame in one preload (frames beyond K*G chunks still work,
 * through the jumbo path), as few lanes per frame as that allows (per-frame
 * work is amortised over the 64/G frames a wave handles at once).  Measured
 * on MI355X: tools/sweep.py, profiles/README.md. */
Geometry pick_geometry(uint32_t len_hint)
{
	if (len_hint == 0)
		return Geometry{16, 2, 6, 1};
	/* worst-case chunks of a frame of len_hint bytes: span <= len - 22,
	 * plus up to 15 bytes of 16-byte misalignment */
	uint32_t chunks = (len_hint + 8) / 16;
	if (chunks <= 8)
		return Geometry{64, 0, 8, 0};  /* 64-byte payloads: the stream kernel, 3.8 TB/s
						  algorithmic (frame groups (4,1,2): 3.1-3.4) */
	if (chunks <= 16)
		return Geometry{8, 1, 2, 0};
	if (chunks <= 32)
		return Geometry{16, 1, 2, 0};
	if (chunks <= 48)
		return Geometry{16, 1, 3, 0};
	if (chunks <= 96)
		return Geometry{16, 2, 6, 1};  /* MTU frames: 6.4-6.5 TB/s at 1 block/CU */
	return Geometry{64, 1, 9, 2};          /* jumbo / mixed up to 9 KB: 6.2 TB/s */
}

bool geometry_supported(Geometry g)
{
	if (g.G == 64 && g.U == 0 && (g.K == 4 || g.K == 8 || g.K == 16))
		return true;
	if (variant_supported && variant_supported(g))
		return true;
#define X(g_, u_, k_) if (g.G == g_ && g.U == u_ && g.K == k_) return true;
	XCSUM_GEOMETRIES(X)
	XCSUM_SWEEP_GEOMETRIES(X)
#undef X
	return false;
}

hipError_t launch_csum(const CsumArgs &a, Geometry g, int cus, hipStream_t s, const ClaimParams *cp)
{
	if (a.n == 0)
		return hipSuccess;
	/* the claimed-tail schedule, where the geometry has it (A/B builds
	 * only: csrc/variants/xcsum_claim.hip) */
	if (cp && cp->claim && cp->static_64 < 64 && g.U > 0 && launch_csum_claim_f0) {
		const hipError_t e = (a.flags & XCSUM_F_IPHDR)    ? launch_csum_claim_f2(a, g, cus, *cp, s)
				     : (a.flags & XCSUM_F_VERIFY) ? launch_csum_claim_f1(a, g, cus, *cp, s)
								  : launch_csum_claim_f0(a, g, cus, *cp, s);
		if (e != hipErrorNotSupported)
			return e;
	}
	/* stream kernel: G = 64 lanes per 64 frames, U = 0, K = KiB of stage */
	if (g.G == 64 && g.U == 0) {
		if (g.K == 4) return launch_stream_t<4>(a, cus, g.B, s);
		if (g.K == 8) return launch_stream_t<8>(a, cus, g.B, s);
		if (g.K == 16) return launch_stream_t<16>(a, cus, g.B, s);
		return hipErrorInvalidValue;
	}
	/* A/B kernels of a variants build (csrc/variants/, not in libxcsum.so) */
	if (variant_supported && variant_supported(g))
		return launch_variant(a, g, cus, s);
	/* Three instantiations per geometry (FEAT): 0 plain, 1 + VERIFY
	 * (udp->len and udp->check prefetched a pipeline step ahead), 2 + IPHDR
	 * (the IPv4 header prefetched too).  Each keeps only the registers and
	 * code it needs: run in the IPHDR instantiation, VERIFY alone cost
	 * 45 % at MTU (tools/verify_probe.py) */
	return (a.flags & XCSUM_F_IPHDR)    ? launch_csum_f2(a, g, cus, s)
	       : (a.flags & XCSUM_F_VERIFY) ? launch_csum_f1(a, g, cus, s)
					    : launch_csum_f0(a, g, cus, s);
}

/* ---- synthetic frame fill: one wave per frame, dword stores ------------- */

static __device__ uint32_t gen_dword(uint32_t family, uint64_t key, uint32_t len, uint32_t hdr,
				     long o0)
{
	/* 4 frame bytes starting at frame offset o0 (all inside the frame) */
	if (o0 >= (long)hdr) {
		uint64_t q = (uint64_t)(o0 - hdr);
		uint64_t w0 = xg_payload_word(key, q >> 3);
		uint64_t w1 = ((q + 3) >> 3) != (q >> 3) ? xg_payload_word(key, (q >> 3) + 1) : w0;
		uint32_t v = 0;
		for (int k = 0; k < 4; k++) {
			uint64_t qq = q + k;
			uint64_t w = (qq >> 3) == (q >> 3) ? w0 : w1;
			v |= (uint32_t)xg_byte_of(w, (uint32_t)(qq & 7)) << (8 * k);
		}
		return v;
	}
	uint32_t v = 0;
	for (int k = 0; k < 4; k++)
		v |= (uint32_t)xg_frame_byte(family, key, len, (uint32_t)(o0 + k)) << (8 * k);
	return v;
}

__global__ void __launch_bounds__(256) gen_kernel(uint8_t *umem, const struct xcsum_desc *desc,
						  uint32_t n, uint32_t family, uint64_t seed,
						  uint64_t first)
{
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t nw = gridDim.x * 4;
	const uint32_t hdr = family == 6 ? XG_HDR6 : XG_HDR4;
	for (uint32_t p = (blockIdx.x * 256 + threadIdx.x) / 64; p < n; p += nw) {
		const struct xcsum_desc d = desc[p];
		uint8_t *eth = umem + d.addr;
		const uint64_t key = xg_key(seed, first + p);
		const uintptr_t e = (uintptr_t)eth + d.len;
		for (uintptr_t w = ((uintptr_t)eth & ~(uintptr_t)3) + 4 * lane; w < e; w += 256) {
			long o0 = (long)(w - (uintptr_t)eth);
			if (w >= (uintptr_t)eth && w + 4 <= e) {
				if (XB_STORE(w, 4, eth, e, XB_GEN_STORE, p))
					*reinterpret_cast<uint32_t *>(w) = gen_dword(family, key, d.len, hdr, o0);
			} else {
				for (int k = 0; k < 4; k++) {
					long o = o0 + k;
					if (o >= 0 && o < (long)d.len)
						eth[o] = xg_frame_byte(family, key, d.len, (uint32_t)o);
				}
			}
		}
	}
}

hipError_t launch_gen(uint8_t *d_umem, const struct xcsum_desc *d_desc, uint32_t n,
		      uint32_t family, uint64_t seed, uint64_t first_index, int max_blocks,
		      hipStream_t s)
{
	if (n == 0)
		return hipSuccess;
	uint64_t blocks = ((uint64_t)n + 3) / 4;
	if (blocks > (uint64_t)max_blocks)
		blocks = max_blocks;
	(void)hipGetLastError();  /* clear a stale error (e.g. hipErrorNotReady from
	                           * someone's hipEventQuery) before checking ours */
	hipLaunchKernelGGL(gen_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_umem, d_desc, n,
			   family, seed, first_index);
	return hipGetLastError();
}

#ifdef XCSUM_DEBUG_BOUNDS
/* positive control of the debug build: one check that must fail, so a test
 * can see the log -> xcsum_debug_bounds() path report it (nothing is
 * accessed) */
__global__ void bounds_selftest_kernel(uint32_t index)
{
	if (threadIdx.x == 0)
		(void)XB_IN((const void *)0x1000, 16, (const void *)0x2000, (const void *)0x3000,
			    XB_GEN_STORE, index);
}
#endif

} /* namespace xcsum */

#ifdef XCSUM_DEBUG_BOUNDS
extern "C" int xcsum_debug_bounds_selftest(uint32_t index)
{
	hipLaunchKernelGGL(xcsum::bounds_selftest_kernel, dim3(1), dim3(64), 0, nullptr, index);
	return hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif
