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
#include "xcsum_internal.h"
#include "xcsum_device.h"
#include "xcsum_frame.h"
#include "xcsum_gen.h"
#include <stdlib.h>

namespace xcsum {

/* Descriptor of frame p (clamped so the load is unconditional; validity is
 * decided by p < n).  With one frame per wave (UNIFORM) it is a scalar load
 * (s_load_dwordx4, counted on lgkmcnt): the compiler moves uniform values to
 * SGPRs right after a vector load, which would make every prefetched
 * descriptor wait stall on the in-order vmcnt of the chunk loads. */
/* Automatic order (ord.sparse_only): keep the prepared region order only when
 * the batch is sparse in the UMEM -- the first and last descriptors span more
 * than twice the bytes of n frames of their mean length.  xudp's TX UMEM (one
 * ~1.5 KB frame per 4096-B chunk, every frame at the same in-chunk offset)
 * is the case: visited in descriptor order, the frames in flight hit a
 * narrow set of HBM channels (tools/slot_probe.py).  Wave-uniform scalar
 * loads; the result never depends on the order. */
static __device__ __forceinline__ void resolve_order(CsumArgs &a)
{
	if (!a.ord.sparse_only)
		return;
	bool sparse = false;
	if (a.n >= 2) {
		const u32x4 d0 = *((cu32x4 *)(a.desc));
		const u32x4 dl = *((cu32x4 *)(a.desc + (a.n - 1)));
		const uint64_t a0 = ((uint64_t)d0.y << 32) | d0.x;
		const uint64_t al = ((uint64_t)dl.y << 32) | dl.x;
		const uint64_t mean = ((uint64_t)d0.z + dl.z) / 2 + 1;
		sparse = al > a0 && al + dl.z - a0 > 2ull * a.n * mean;
	}
	if (!sparse)
		a.ord = order_identity(a.n);
}

template <bool UNIFORM>
static __device__ __forceinline__ u32x4 load_desc(const CsumArgs &a, uint32_t p)
{
	uint32_t q = p < a.n ? p : a.n - 1;
	if (UNIFORM)
		return *((cu32x4 *)(a.desc + q));
	return *((gu32x4 *)(a.desc + q));
}

template <bool DW, int FEAT>
static __device__ __forceinline__ Frame resolve(const CsumArgs &a, u32x4 d, bool present)
{
	Frame f;
	/* d.w (xdp_desc.options) is unused; keeping it "used" here stops the
	 * register allocator from recycling that VGPR as a temporary right after
	 * the prefetch is issued, which would force a full vmcnt(0) drain of the
	 * software pipeline every iteration */
	asm volatile("" ::"v"(d.w));
	uint64_t addr = (((uint64_t)d.y << 32) | d.x) - a.bias;
	uint32_t len = d.z;
	int mode = (int)a.mode;
	f.eth = a.umem + addr;
	if (present && mode == XCSUM_MODE_AUTO) {
		uint32_t proto = ((uint32_t)f.eth[12] << 8) | f.eth[13];
		mode = proto == 0x0800u ? ((a.flags & XCSUM_F_V4_RFC) ? 1 : 0)
		     : proto == 0x86DDu ? 2 : -1;
	}
	uint32_t hdr = mode == 2 ? 54u : 34u;
	uint32_t pre = mode == 2 ? 32u : 8u;
	if (mode < 0 || len < hdr + 8u || len - hdr > 65535u)
		mode = -1;
	uintptr_t lo = (uintptr_t)f.eth + hdr - pre;
	f.udp_len = len - hdr;
	set_span<DW>(f, lo, lo + (len + pre - hdr));
	if (mode < 0 || !present)
		f.nchunks = 0;
	f.mode = present ? mode : -2;
	/* VERIFY needs the check field: load it with this frame's chunks, one
	 * pipeline step before finalize() reads it (loaded there, it was a
	 * dependent round trip on every frame).  Unconditional and unused
	 * until then: any branch or arithmetic on it here makes the compiler
	 * wait for the load on the spot. */
	f.ck = 0;
	f.ul = 0;
	if (FEAT >= 1 && (a.flags & XCSUM_F_VERIFY)) { /* wave-uniform: no load otherwise */
		/* udp->len too: a received frame may carry Ethernet padding, so
		 * the span ends at udp + ntohs(udp->len), not at the frame end */
		/* Two 2-byte loads whose addresses differ by no constant (the
		 * absent-frame fallbacks are 8 bytes apart), so the compiler
		 * cannot merge them: merged, they were one dword load at eth + 38
		 * (2 mod 4 in every xudp frame), and that misaligned load cost the
		 * MTU kernel 45 % (tools/verify_probe.py).  An empty asm to keep
		 * them apart cost every mode 20 %: it coarsened the waitcnts. */
		const uint8_t *z = (const uint8_t *)g_zero_chunk;
		const uint32_t lo = mode == 2 ? 58u : 38u;
		f.ul = *(const uint16_t *)(f.nchunks ? f.eth + lo : z);
		f.ck = *(const uint16_t *)(f.nchunks ? f.eth + lo + 2 : z + 8);
	}
	/* IPHDR: the IPv4 header too (six dwords, same reasoning) */
	if (FEAT == 2 && (a.flags & XCSUM_F_IPHDR)) {
		const uint8_t *ih = f.nchunks && mode != 2 ? f.eth + 14
							   : (const uint8_t *)g_zero_chunk;
		f.ihs = (uint32_t)(uintptr_t)ih & 3u;
		const uint32_t *w = (const uint32_t *)((uintptr_t)ih & ~(uintptr_t)3);
#pragma unroll
		for (int j = 0; j < 6; j++)
			f.ih[j] = w[j];
	}
	return f;
}


/* IPv4 header checksum (RFC 1071 over the 20-byte header) with the check
 * field as 0 -- equals xudp_checksum_half() (packet.c:43-66) on every header
 * iph_build() writes (ihl is always 5 there, packet.c:21, and the
 * frame-layout contract of xcsum.h) -- or, to VERIFY a received header, with
 * the check field included (0 = valid).  Returns the memory-order value. */
static __device__ uint16_t ip_header_csum_mem(const uint8_t *iph, bool verify)
{
	uint32_t sum = 0;
#pragma unroll
	for (uint32_t i = 0; i < 20; i += 2)
		if (verify || i != 10)
			sum += ((uint32_t)iph[i] << 8) | iph[i + 1];
	sum = (sum & 0xffffu) + (sum >> 16);
	sum = (sum & 0xffffu) + (sum >> 16);
	return bswap16(~sum & 0xffffu);
}

/* IPH: from the dwords resolve() prefetched; else from memory (a dependent
 * round trip -- the kernels are instantiated with FEAT 2 whenever IPHDR is set,
 * the fallback only keeps results independent of the instantiation) */
template <bool IPH>
static __device__ uint16_t ip_header_csum(const Frame &f, bool verify)
{
	if (!IPH)
		return ip_header_csum_mem(f.eth + 14, verify);
	/* the header from the dwords resolve() prefetched, opaque until here
	 * (or the compiler computes on them early and waits for the loads) */
	uint32_t w[6];
#pragma unroll
	for (int j = 0; j < 6; j++) {
		w[j] = f.ih[j];
		asm volatile("" : "+v"(w[j]));
	}
	uint32_t sum = 0;
#pragma unroll
	for (int j = 0; j < 5; j++) {
		/* header bytes 4j..4j+3, little-endian; BE words = 256*even + odd */
		const uint32_t d = __builtin_amdgcn_alignbyte(w[j + 1], w[j], f.ihs);
		sum += (dot_even(d, 0u) << 8) + dot_odd(d, 0u);
		if (j == 2 && !verify)   /* bytes 10-11: the check field itself */
			sum -= ((d >> 8) & 0xff00u) | (d >> 24);
	}
	sum = (sum & 0xffffu) + (sum >> 16);
	sum = (sum & 0xffffu) + (sum >> 16);
	return bswap16(~sum & 0xffffu);
}

template <int FEAT>
static __device__ __forceinline__ void finalize(const CsumArgs &a, const Frame &f, uint32_t p,
						uint32_t s)
{
	uint16_t wire = 0;
	if (f.mode >= 0) {
		uint32_t udp_len = f.udp_len;
		bool bad_len = false;
		if (FEAT >= 1 && (a.flags & XCSUM_F_VERIFY)) {
			/* A received frame may carry Ethernet padding or trailing
			 * bytes: the datagram ends at udp + ntohs(udp->len) (RFC 768;
			 * xudp_fill_msg reads it the same way, channel.c:86).  Rare,
			 * so handled here by this one lane, re-summing the span from
			 * memory; tested in the pipelined loop it cost 36 % at MTU
			 * (one wave per SIMD has nothing to hide the check behind).
			 * f.ul was loaded with the frame's chunks, opaque until here. */
			uint32_t ul = f.ul;
			asm volatile("" : "+v"(ul));
			ul = bswap16(ul);
			if (ul != udp_len) {
				bad_len = ul < 8u || ul > udp_len;   /* never verifies */
				if (!bad_len) {
					Frame g = f;
					const uint32_t pre = f.mode == 2 ? 32u : 8u;
					const uintptr_t lo = (uintptr_t)f.eth + (f.mode == 2 ? 54u : 34u) - pre;
					set_span<false>(g, lo, lo + pre + ul);
					uint32_t E = 0, O = 0;
					sum_walk<1, false>(g, 0, E, O);
					s = g.odd ? (O << 8) + E : (E << 8) + O;
					udp_len = ul;
				}
			}
		}
		uint32_t S = s + 17u + (udp_len >> 16) + (udp_len & 0xffffu);
		uint32_t r;
		if (FEAT >= 1 && (a.flags & XCSUM_F_VERIFY)) {
			/* the frame's check field was summed with everything else:
			 * a valid RFC checksum folds to 0xffff, i.e. r == 0 */
			uint32_t t = (S & 0xffffu) + (S >> 16);
			t = (t & 0xffffu) + (t >> 16);
			r = ~t & 0xffffu;
			/* opaque until here, or the compiler hoists the test into
			 * resolve() and waits for the load there */
			uint32_t ck = f.ck;
			asm volatile("" : "+v"(ck));
			if ((ck & 0xffffu) == 0)  /* no checksum: IPv4 ok, IPv6 invalid */
				r = f.mode == 2 ? 0xffffu : 0u;
			if (bad_len)
				r = 0xffffu;
			wire = bswap16(r);
			if ((a.flags & XCSUM_F_IPHDR) && f.mode != 2) {
				uint16_t ipr = ip_header_csum<FEAT == 2>(f, true);
				if (a.out_ip)
					a.out_ip[p] = ipr;
				if (wire == 0)
					wire = ipr;  /* 0 only if both verify */
			}
			if (a.out)
				a.out[p] = wire;
			return;
		}
		if (f.mode == 0) {
			/* checksum.h:100-104: one fold, carry dropped by the u16 cast */
			r = ~((S & 0xffffu) + (S >> 16)) & 0xffffu;
		} else {
			uint32_t t = (S & 0xffffu) + (S >> 16);
			t = (t & 0xffffu) + (t >> 16);
			r = ~t & 0xffffu;
			if (r == 0)
				r = 0xffffu; /* CSUM_MANGLED_0, packet.c:23, :115-116 */
		}
		wire = bswap16(r);
		if (a.flags & XCSUM_F_INPLACE)
			store_u16(f.eth + (f.mode == 2 ? 60 : 40), wire);
		if ((a.flags & XCSUM_F_IPHDR) && f.mode != 2) {
			uint16_t ipc = ip_header_csum<FEAT == 2>(f, false);
			if (a.flags & XCSUM_F_INPLACE)
				store_u16(f.eth + 24, ipc);
			if (a.out_ip)
				a.out_ip[p] = ipc;
		}
	} else {
		if (f.mode != -3)        /* -3: UDP length does not fit (VERIFY) */
			atomicAdd(a.err, 1ull);
		if (a.flags & XCSUM_F_VERIFY)
			wire = 0xffffu;  /* a malformed frame never verifies */
	}
	if (a.out)
		a.out[p] = wire;
	if (a.out_ip && !((a.flags & XCSUM_F_IPHDR) && f.mode >= 0 && f.mode != 2))
		a.out_ip[p] = 0;
}

/* accumulate, reduce and finalize the U frames of one iteration */
template <bool ORD>
static __device__ __forceinline__ uint32_t fidx(const CsumArgs &a, uint32_t p)
{
	return ORD ? frame_of(a.ord, p) : p;
}

template <int G, int U, int K, bool TAIL, bool ORD, int FEAT>
static __device__ __forceinline__ void consume(const CsumArgs &a, const Frame (&fc)[U],
					       const u32x4 (&vc)[U][K], uint32_t lane,
					       uint32_t p0, uint32_t nseg)
{
#pragma unroll
	for (int u = 0; u < U; u++) {
		const Frame &f = fc[u];
		uint32_t E = 0, O = 0;
		if (!TAIL || f.nchunks <= K * G)
			sum_frame<G, K, U, Grid<G, K>::DW>(f, vc[u], lane, E, O);
		else
			sum_walk<G, Grid<G, K>::DW>(f, lane, E, O);   /* jumbo frame */
		uint32_t s = f.odd ? (O << 8) + E : (E << 8) + O;
		s = seg_sum<G>(s);
		if (lane == 0 && f.mode != -2)
			finalize<FEAT>(a, f, fidx<ORD>(a, p0 + u * nseg), s);
	}
}

/* XCSUM_PINGPONG=0 builds the previous loop shape (A/B only): "next" copied
 * into "current" at the loop latch */
#ifndef XCSUM_PINGPONG
#define XCSUM_PINGPONG 1
#endif

/* wave-uniform split: the jumbo path lives in its own copy of the body, so
 * its drains never merge into the common path's vmcnt bookkeeping */
template <int G, int U, int K, bool ORD, int FEAT>
static __device__ __forceinline__ void consume_any(const CsumArgs &a, const Frame (&fc)[U],
						   const u32x4 (&vc)[U][K], uint32_t lane,
						   uint32_t p0, uint32_t nseg)
{
	bool big = false;
#pragma unroll
	for (int u = 0; u < U; u++)
		big |= fc[u].nchunks > K * G;
	if (__builtin_amdgcn_ballot_w64(big))
		consume<G, U, K, true, ORD, FEAT>(a, fc, vc, lane, p0, nseg);
	else
		consume<G, U, K, false, ORD, FEAT>(a, fc, vc, lane, p0, nseg);
}

/*
 * Persistent grid; segment s (G lanes) owns frames s, s + nseg, ... and
 * handles U of them per step.  Two-stage software pipeline written as a
 * ping-pong over two register sets (A, B): while step i's chunks are
 * reduced, step i+1's chunks are in flight and step i+2's descriptors are
 * loading.  Descriptor loads are issued BEFORE the chunk loads of the same
 * step, so the in-order vmcnt wait for them never waits on chunk data.
 * The ping-pong matters: with one "current" set refilled from a "next" set
 * at the loop latch, that copy needs the next step's loads to have landed,
 * and the ISA showed a vmcnt(0) there -- one step in flight, not two.
 */
template <int G, int U, int K, bool ORD, int FEAT>
static __device__ __forceinline__ void csum_loop(const CsumArgs &a)
{
	const uint32_t lane = threadIdx.x & (G - 1);
	uint32_t seg = (blockIdx.x * 256u + threadIdx.x) / G;
	const uint32_t nseg = gridDim.x * (256u / G);
	if (G == 64)
		seg = __builtin_amdgcn_readfirstlane(seg);
	const uint32_t step = nseg * U;
	const uint32_t limit = ORD ? a.ord.nlog : a.n;
	/* logical index q names a frame only below the logical range end (past
	 * it, frame_of() would alias real frames) */
	auto has = [&](uint32_t q) { return q < limit && fidx<ORD>(a, q) < a.n; };

	u32x4 d[U];
	Frame fa[U];
	u32x4 va[U][K];
#pragma unroll
	for (int u = 0; u < U; u++)
		d[u] = load_desc<G == 64>(a, fidx<ORD>(a, seg + u * nseg));
#pragma unroll
	for (int u = 0; u < U; u++)
		fa[u] = resolve<Grid<G, K>::DW, FEAT>(a, d[u], has(seg + u * nseg));
#pragma unroll
	for (int u = 0; u < U; u++)
		d[u] = load_desc<G == 64>(a, fidx<ORD>(a, seg + step + u * nseg));
	/* keep every descriptor load older than the chunk loads it shares a
	 * vmcnt queue with: the next wait for the descriptors then leaves all
	 * chunk loads in flight */
	__builtin_amdgcn_sched_barrier(0);
	issue<G, U, K>(fa, lane, va);

#if XCSUM_PINGPONG
	Frame fb[U];
	u32x4 vb[U][K];
	for (uint32_t p0 = seg; p0 < limit; p0 += 2 * step) {
#pragma unroll
		for (int u = 0; u < U; u++)
			fb[u] = resolve<Grid<G, K>::DW, FEAT>(a, d[u], has(p0 + step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 2 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K>(fb, lane, vb);
		consume_any<G, U, K, ORD, FEAT>(a, fa, va, lane, p0, nseg);

#pragma unroll
		for (int u = 0; u < U; u++)
			fa[u] = resolve<Grid<G, K>::DW, FEAT>(a, d[u],
							has(p0 + 2 * step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 3 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K>(fa, lane, va);
		consume_any<G, U, K, ORD, FEAT>(a, fb, vb, lane, p0 + step, nseg);
	}
#else
	for (uint32_t p0 = seg; p0 < limit; p0 += step) {
		Frame fn[U];
		u32x4 vn[U][K];
#pragma unroll
		for (int u = 0; u < U; u++)
			fn[u] = resolve<Grid<G, K>::DW, FEAT>(a, d[u], has(p0 + step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 2 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K>(fn, lane, vn);
		consume_any<G, U, K, ORD, FEAT>(a, fa, va, lane, p0, nseg);
#pragma unroll
		for (int u = 0; u < U; u++) {
			fa[u] = fn[u];
#pragma unroll
			for (int k = 0; k < K; k++)
				va[u][k] = vn[u][k];
		}
	}
#endif
}

/* The identity order gets its own copy of the loop, so descriptor-order
 * batches pay nothing for the region order; which copy runs is decided once
 * per launch (uniform branch, after resolve_order). */
template <int G, int U, int K, int FEAT>
static __device__ __forceinline__ void csum_body(CsumArgs &a)
{
	resolve_order(a);
	if (a.ord.rshift == 0)
		csum_loop<G, U, K, false, FEAT>(a);
	else
		csum_loop<G, U, K, true, FEAT>(a);
}

template <int G, int U, int K, int FEAT>
__global__ void __launch_bounds__(256) csum_kernel(CsumArgs a)
{
	csum_body<G, U, K, FEAT>(a);
}

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
							 XCSUM_NT ? 2 : 0);
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

/* dense batch: the first and last descriptors span at most twice the bytes
 * of n frames of their mean length (the converse of resolve_order) */
static __device__ __forceinline__ bool dense_batch(const CsumArgs &a)
{
	if (a.n < 2)
		return true;
	const u32x4 d0 = *((cu32x4 *)(a.desc));
	const u32x4 dl = *((cu32x4 *)(a.desc + (a.n - 1)));
	const uint64_t a0 = ((uint64_t)d0.y << 32) | d0.x;
	const uint64_t al = ((uint64_t)dl.y << 32) | dl.x;
	const uint64_t mean = ((uint64_t)d0.z + dl.z) / 2 + 1;
	return !(al > a0 && al + dl.z - a0 > 2ull * a.n * mean);
}

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
	uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));

	auto span_of = [&](uint32_t wi, u32x4 d) {
		StreamSpan sp;
		const uint32_t p = 64u * wi + lane;
		sp.present = p < a.n;
		sp.eth = ((((uint64_t)d.y << 32) | d.x) - a.bias);
		sp.len = d.z;
		return sp;
	};
	/* Region of a wave-iteration: base (16-aligned UMEM offset) and chunk
	 * count, or ~0u when the frames do not fit the stage.  The bounds are
	 * the first lane's frame start and the last present lane's frame end
	 * (two readlanes -- a packed batch is in UMEM order); every frame must
	 * then lie inside them (one ballot), else the wave walks its frames. */
	auto region = [&](uint32_t wi, const StreamSpan &sp, uint64_t &base, uint32_t &nch) {
		const uint64_t rem = a.n - 64ull * wi;
		const uint32_t last = rem > 64 ? 63u : (uint32_t)rem - 1u;
		const uint64_t end = sp.eth + sp.len;
		const uint64_t lo =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(sp.eth >> 32), 0) << 32) |
			__builtin_amdgcn_readlane((uint32_t)sp.eth, 0);
		const uint64_t hi =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(end >> 32), last) << 32) |
			__builtin_amdgcn_readlane((uint32_t)end, last);
		base = lo & ~15ull;
		const bool out = sp.present && (sp.eth < lo || end > hi);
		nch = (__builtin_amdgcn_ballot_w64(out) || hi < lo || hi - base > (uint64_t)KC * 1024u)
			      ? ~0u : (uint32_t)((hi - base + 15) >> 4);
	};
	auto issue_region = [&](uint64_t base, uint32_t nch, u32x4 (&v)[KC]) {
#pragma unroll
		for (int k = 0; k < KC; k++) {
			const uint32_t c = (uint32_t)k * 64u + lane;
			v[k] = load_chunk(nch != ~0u && c < nch ? a.umem + base + 16u * c : zero);
		}
	};
	auto load_d = [&](uint32_t wi) {
		const uint32_t p = 64u * wi + lane;
		return *((gu32x4 *)(a.desc + (p < a.n ? p : a.n - 1)));
	};

	if (64ull * w >= a.n)
		return;
	u32x4 d = load_d(w);
	StreamSpan sc = span_of(w, d);
	uint64_t bc;
	uint32_t nc;
	region(w, sc, bc, nc);
	u32x4 v[KC];
	issue_region(bc, nc, v);
	d = load_d(w + nw);
	for (; 64ull * w < a.n; w += nw) {
		/* this iteration's region -> LDS (waits for its loads only: the
		 * descriptors issued after them may still be in flight) */
#pragma unroll
		for (int k = 0; k < KC; k++)
			stage[k * 64 + lane] = v[k];
		const StreamSpan cur = sc;
		const uint64_t cbase = bc;
		const uint32_t cnch = nc;
		/* next iteration: its region's loads go out before this one is summed */
		if (64ull * (w + nw) < a.n) {
			sc = span_of(w + nw, d);
			region(w + nw, sc, bc, nc);
			__builtin_amdgcn_sched_barrier(0);
			issue_region(bc, nc, v);
			d = load_d(w + 2 * nw);
		}
		__builtin_amdgcn_sched_barrier(0);
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

		if (cnch == ~0u) {
			/* does not fit the stage: the whole wave walks each frame */
			for (uint32_t i = 0; i < 64; i++) {
				const uint32_t p = 64u * w + i;
				if (p >= a.n)
					break;
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
			const uint32_t oe = (uint32_t)(cur.eth - cbase);   /* frame in the stage */
			Frame f;
			f.eth = a.umem + cur.eth;
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
				const uint32_t c0 = lo >> 4, c1 = (hi + 15) >> 4;
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

/* XCSUM_STREAM_WPE=N builds a variant capped for N waves per SIMD (A/B) */
#if defined(XCSUM_STREAM_WPE) && XCSUM_STREAM_WPE > 0
#define STREAM_ATTR __attribute__((amdgpu_waves_per_eu(XCSUM_STREAM_WPE)))
#else
#define STREAM_ATTR
#endif

template <int KC>
__global__ void __launch_bounds__(256) STREAM_ATTR csum_stream_kernel(CsumArgs a)
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

template <int G, int U, int K, int FEAT>
static hipError_t launch_t(const CsumArgs &a, int cus, int bpc, hipStream_t s)
{
	/* persistent grid: at most what the device keeps resident, so no second
	 * wave of late blocks; fewer per CU when that streams better (Geometry.B) */
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, csum_kernel<G, U, K, FEAT>, 256, 0) !=
			    hipSuccess || nb <= 0)
			nb = 4;
		return nb;
	});
	int per_cu = (bpc > 0 && bpc < occ) ? bpc : occ;
	uint64_t segs = ((uint64_t)a.ord.nlog + U - 1) / U;
	uint64_t blocks = (segs * G + 255) / 256;
	uint64_t cap = (uint64_t)cus * per_cu;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();  /* clear a stale error (e.g. hipErrorNotReady from
	                           * someone's hipEventQuery) before checking ours */
	hipLaunchKernelGGL((csum_kernel<G, U, K, FEAT>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

#define XCSUM_GEOMETRIES(X) \
	X(64, 1, 2) X(64, 1, 9) X(32, 1, 3) X(32, 1, 6) \
	X(16, 1, 2) X(16, 1, 3) X(16, 1, 6) X(16, 2, 6) X(16, 1, 12) \
	X(8, 1, 2) X(8, 2, 1) X(8, 1, 12) X(4, 2, 2) X(4, 4, 2) X(4, 1, 2) \
	X(2, 1, 4) X(2, 2, 4) X(1, 1, 6) X(1, 1, 8) X(1, 2, 6)

bool geometry_supported(Geometry g)
{
	if (g.G == 64 && g.U == 0 && (g.K == 4 || g.K == 8 || g.K == 16))
		return true;
	if (g.G == 16 && ((g.U == 12 || g.U == 13) && g.K == 6))
		return true;
	if (g.G == 16 && ((g.U == 12 || g.U == 14) && g.K == 3))
		return true;
#define X(g_, u_, k_) if (g.G == g_ && g.U == u_ && g.K == k_) return true;
	XCSUM_GEOMETRIES(X)
#undef X
	return false;
}

hipError_t launch_csum(const CsumArgs &a, Geometry g, int cus, hipStream_t s)
{
	if (a.n == 0)
		return hipSuccess;
	/* LDS-staged variant: G = 16, U = 10 + ring depth; identity order */
	/* stream kernel: G = 64 lanes per 64 frames, U = 0, K = KiB of stage */
	if (g.G == 64 && g.U == 0) {
		if (g.K == 4) return launch_stream_t<4>(a, cus, g.B, s);
		if (g.K == 8) return launch_stream_t<8>(a, cus, g.B, s);
		if (g.K == 16) return launch_stream_t<16>(a, cus, g.B, s);
		return hipErrorInvalidValue;
	}
	CsumArgs b = a;
	b.ord = order_identity(a.n);
	if (g.G == 16 && g.U == 12 && g.K == 6) return launch_lds_t<6, 2>(b, cus, g.B, s);
	if (g.G == 16 && g.U == 13 && g.K == 6) return launch_lds_t<6, 3>(b, cus, g.B, s);
	if (g.G == 16 && g.U == 14 && g.K == 3) return launch_lds_t<3, 4>(b, cus, g.B, s);
	if (g.G == 16 && g.U == 12 && g.K == 3) return launch_lds_t<3, 2>(b, cus, g.B, s);
	/* Three instantiations per geometry (FEAT): 0 plain, 1 + VERIFY
	 * (udp->len and udp->check prefetched a pipeline step ahead), 2 + IPHDR
	 * (the IPv4 header prefetched too).  Each keeps only the registers and
	 * code it needs: run in the IPHDR instantiation, VERIFY alone cost
	 * 45 % at MTU (tools/verify_probe.py) */
#define X(g_, u_, k_)                                                                  \
	if (g.G == g_ && g.U == u_ && g.K == k_)                                        \
		return (a.flags & XCSUM_F_IPHDR)    ? launch_t<g_, u_, k_, 2>(a, cus, g.B, s) \
		       : (a.flags & XCSUM_F_VERIFY) ? launch_t<g_, u_, k_, 1>(a, cus, g.B, s) \
						    : launch_t<g_, u_, k_, 0>(a, cus, g.B, s);
	XCSUM_GEOMETRIES(X)
#undef X
	return hipErrorInvalidValue;
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

} /* namespace xcsum */
