/* xcsum_csum.h -- the frame-group checksum kernel csum_kernel<G, U, K, FEAT>
 * (see xcsum_kernels.hip for what it computes and how), its launcher and the
 * table of compiled geometries.  Instantiated per feature set in its own
 * translation unit (xcsum_csum_f{0,1,2}.hip) so the three compile in
 * parallel; static/template code only. */
#ifndef XCSUM_CSUM_H
#define XCSUM_CSUM_H

#include "xcsum_internal.h"
#include "xcsum_device.h"
#include "xcsum_frame.h"

namespace xcsum {

/* Descriptor of frame p (clamped so the load is unconditional; validity is
 * decided by p < n).  With one frame per wave (UNIFORM) it is a scalar load
 * (s_load_dwordx4, counted on lgkmcnt): the compiler moves uniform values to
 * SGPRs right after a vector load, which would make every prefetched
 * descriptor wait stall on the in-order vmcnt of the chunk loads. */
/* Automatic order (ord.sparse_only): keep the prepared region order when the
 * batch is sparse in the UMEM -- the first and last descriptors span more
 * than twice the bytes of n frames of their mean length -- else take the
 * dense batch's order (a.dense).  xudp's TX UMEM (one ~1.5 KB frame per
 * 4096-B chunk, every frame at the same in-chunk offset) is the sparse case:
 * visited in descriptor order, the frames in flight hit a narrow set of HBM
 * channels (tools/slot_probe.py).  Wave-uniform scalar loads; the result
 * never depends on the order. */
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
		a.ord = a.dense;
}

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

/* descriptor hooks of the plain argument type (never called: kChecked is
 * false); a checked type brings its own overloads */
static __device__ __forceinline__ bool desc_ok(const CsumArgs &, u32x4)
{
	return true;
}
static __device__ __forceinline__ void desc_bad(const CsumArgs &, uint32_t) {}

template <bool UNIFORM, class A>
static __device__ __forceinline__ u32x4 load_desc(const A &a, uint32_t p)
{
	uint32_t q = p < a.n ? p : a.n - 1;
	if constexpr (A::kChecked) {
		if (a.inl)   /* descriptors that came with the request (LDS) */
			return desc_inline(a, q);
	}
	if (UNIFORM)
		return *((cu32x4 *)(a.desc + q));
	return *((gu32x4 *)(a.desc + q));
}

template <bool DW, int FEAT, class A = CsumArgs>
static __device__ __forceinline__ Frame resolve(const A &a, u32x4 d, bool present)
{
	Frame f;
	/* a checked argument type: a descriptor outside its bounds is an absent
	 * frame (no load of it) marked -4, reported by consume() */
	bool bad = false;
	if constexpr (A::kChecked) {
		bad = present && !desc_ok(a, d);
		present = present && !bad;
	}
	/* d.w (xdp_desc.options) is unused; keeping it "used" here stops the
	 * register allocator from recycling that VGPR as a temporary right after
	 * the prefetch is issued, which would force a full vmcnt(0) drain of the
	 * software pipeline every iteration */
	asm volatile("" ::"v"(d.w));
	uint64_t addr = (((uint64_t)d.y << 32) | d.x) - a.bias;
	uint32_t len = d.z;
	int mode = (int)a.mode;
	f.eth = a.umem + addr;
#ifdef XCSUM_DEBUG_BOUNDS
	f.lim = (const uint8_t *)(((uintptr_t)f.eth + len + 15u) & ~(uintptr_t)15);
	f.dlen = len;
	/* a zero-copy frame must lie in its registered region, 16-byte blocks
	 * included: else it is not read at all */
	if constexpr (!A::kChecked) {
		if (present && a.reg_hi &&
		    !XB_IN((uintptr_t)f.eth & ~(uintptr_t)15, (uintptr_t)f.lim - ((uintptr_t)f.eth & ~(uintptr_t)15),
			   a.reg_lo, a.reg_hi, XB_CSUM_REGION, addr))
			present = false;
	}
#endif
	if (present && mode == XCSUM_MODE_AUTO) {
		/* h_proto only inside the frame: a descriptor shorter than the
		 * Ethernet header is malformed whatever its next bytes hold */
		uint32_t proto = 0;
		if (len >= 14 && XB_IN(f.eth + 12, 2, f.eth, f.eth + len, XB_CSUM_HDR, 12))
			proto = ((uint32_t)ld_g<uint8_t>(f.eth + 12) << 8) | ld_g<uint8_t>(f.eth + 13);
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
	f.mode = present ? mode : bad ? -4 : -2;
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
		f.ul = ld_g<uint16_t>(f.nchunks ? XB_LOAD(f.eth + lo, 2, f.eth, f.eth + len,
							   XB_CSUM_HDR, lo, z)
						: z);
		f.ck = ld_g<uint16_t>(f.nchunks ? XB_LOAD(f.eth + lo + 2, 2, f.eth, f.eth + len,
							   XB_CSUM_HDR, lo + 2, z + 8)
						: z + 8);
	}
	/* IPHDR: the IPv4 header too (six dwords, same reasoning) */
	if (FEAT == 2 && (a.flags & XCSUM_F_IPHDR)) {
		const uint8_t *ih = f.nchunks && mode != 2 ? f.eth + 14
							   : (const uint8_t *)g_zero_chunk;
		f.ihs = (uint32_t)(uintptr_t)ih & 3u;
		/* global loads: the integer round trip loses the address space,
		 * and as flat loads (counted on lgkmcnt too) they ran config 2 in
		 * place 0.3419 ms instead of 0.3381 (same box, alternating,
		 * profiles/r04/inplace/r04n_ab_flat_b64.txt) */
		typedef __attribute__((address_space(1))) const uint32_t gu32;
		gu32 *w = (gu32 *)((uintptr_t)ih & ~(uintptr_t)3);
		if (ih != (const uint8_t *)g_zero_chunk &&
		    !XB_IN(w, 24, (uintptr_t)f.eth & ~(uintptr_t)3, f.lim, XB_CSUM_HDR, 14))
			w = (gu32 *)g_zero_chunk;
		/* plain (temporal) loads: with XCSUM_F_INPLACE the line they bring
		 * into L2 takes the iph->check store; nontemporal, the in-place
		 * pass ran 0.391 ms instead of 0.341 (config 2, same box, round 4
		 * A/B, profiles/r04/inplace/r04g_c2_ihnt_*.log) */
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
				if (a.out_ip && XB_IDX(p, a.n, XB_CSUM_OUT))
					st_res(a.out_ip + p, ipr);
				if (wire == 0)
					wire = ipr;  /* 0 only if both verify */
			}
			if (a.out && XB_IDX(p, a.n, XB_CSUM_OUT))
				st_res(a.out + p, wire);
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
		/* In place: 2-byte stores from lane 0.  Round 4 A/B (same box,
		 * alternating, profiles/r04/inplace/r04i_cs16.bundle.txt): the lane holding
		 * the field's 16-byte chunk storing the whole chunk, patched, ran
		 * config 2 0.365 ms vs 0.342, config 4 0.397 vs 0.325, xudp's slots
		 * 0.369 vs 0.358 -- deleted.  The four lanes holding the 64-byte
		 * block around the field storing it whole (a complete block, no
		 * merge beyond L2; the chunk below the grid loaded for it): config 4
		 * 0.338 vs 0.3265, config 2 0.358 vs 0.338 (r04n_ab_flat_b64.txt,
		 * commit d8dab61) -- deleted.
		 * frame end: eth + hdr + udp_len (udp_len is not re-cut without VERIFY) */
		const uint8_t *fend = f.eth + (f.mode == 2 ? 54u : 34u) + f.udp_len;
		(void)fend;
		if ((a.flags & XCSUM_F_INPLACE) &&
		    XB_STORE(f.eth + (f.mode == 2 ? 60 : 40), 2, f.eth, fend, XB_CSUM_INPLACE, p))
			store_u16(f.eth + (f.mode == 2 ? 60 : 40), wire);
		if ((a.flags & XCSUM_F_IPHDR) && f.mode != 2) {
			uint16_t ipc = ip_header_csum<FEAT == 2>(f, false);
			if ((a.flags & XCSUM_F_INPLACE) &&
			    XB_STORE(f.eth + 24, 2, f.eth, fend, XB_CSUM_INPLACE, p))
				store_u16(f.eth + 24, ipc);
			if (a.out_ip && XB_IDX(p, a.n, XB_CSUM_OUT))
				st_res(a.out_ip + p, ipc);
		}
	} else {
		if (f.mode != -3)        /* -3: UDP length does not fit (VERIFY) */
			atomicAdd(a.err, 1ull);
		if (a.flags & XCSUM_F_VERIFY)
			wire = 0xffffu;  /* a malformed frame never verifies */
	}
	if (a.out && XB_IDX(p, a.n, XB_CSUM_OUT))
		st_res(a.out + p, wire);
	if (a.out_ip && !((a.flags & XCSUM_F_IPHDR) && f.mode >= 0 && f.mode != 2) &&
	    XB_IDX(p, a.n, XB_CSUM_OUT))
		st_res(a.out_ip + p, (uint16_t)0);
}

/* accumulate, reduce and finalize the U frames of one iteration */
template <bool ORD>
static __device__ __forceinline__ uint32_t fidx(const CsumArgs &a, uint32_t p)
{
	return ORD ? frame_of(a.ord, p) : p;
}

template <int G, int U, int K, bool TAIL, bool ORD, int FEAT, class A>
static __device__ __forceinline__ void consume(const A &a, const Frame (&fc)[U],
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
		if (lane == 0 && f.mode != -2) {
			if constexpr (A::kChecked) {
				if (f.mode == -4)
					desc_bad(a, fidx<ORD>(a, p0 + u * nseg));
				else
					finalize<FEAT>(a, f, fidx<ORD>(a, p0 + u * nseg), s);
			} else {
				finalize<FEAT>(a, f, fidx<ORD>(a, p0 + u * nseg), s);
			}
		}
	}
}

/* wave-uniform split: the jumbo path lives in its own copy of the body, so
 * its drains never merge into the common path's vmcnt bookkeeping */
template <int G, int U, int K, bool ORD, int FEAT, class A>
static __device__ __forceinline__ void consume_any(const A &a, const Frame (&fc)[U],
						   const u32x4 (&vc)[U][K], uint32_t lane,
						   uint32_t p0, uint32_t nseg)
{
	bool big = false;
#pragma unroll
	for (int u = 0; u < U; u++)
		big |= fc[u].nchunks > K * G;
	if (__builtin_amdgcn_ballot_w64(big))
		consume<G, U, K, true, ORD, FEAT, A>(a, fc, vc, lane, p0, nseg);
	else
		consume<G, U, K, false, ORD, FEAT, A>(a, fc, vc, lane, p0, nseg);
}

#ifdef XCSUM_WAVE_STAMPS
/* `make variant NAME=stamps DEFS=-DXCSUM_WAVE_STAMPS` only (tools/wave_tail.py,
 * DESIGN.md 9.4): every wave's start and end on the 100 MHz constant clock,
 * to see the persistent grid's tail.  Not in libxcsum.so. */
constexpr uint32_t WAVE_STAMPS_MAX = 65536;
static __device__ uint64_t g_wave_stamps[2 * WAVE_STAMPS_MAX];
#endif

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
template <int G, int U, int K, bool ORD, int FEAT, class A, int TL = 0>
static __device__ __forceinline__ void csum_loop(const A &a)
{
#ifdef XCSUM_WAVE_STAMPS
	const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
	__builtin_amdgcn_s_waitcnt(0xC07F);
#endif
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
		fa[u] = resolve<Grid<G, K>::DW, FEAT, A>(a, d[u], has(seg + u * nseg));
#pragma unroll
	for (int u = 0; u < U; u++)
		d[u] = load_desc<G == 64>(a, fidx<ORD>(a, seg + step + u * nseg));
	/* keep every descriptor load older than the chunk loads it shares a
	 * vmcnt queue with: the next wait for the descriptors then leaves all
	 * chunk loads in flight */
	__builtin_amdgcn_sched_barrier(0);
	issue<G, U, K, TL>(fa, lane, va);

	Frame fb[U];
	u32x4 vb[U][K];
	for (uint32_t p0 = seg; p0 < limit; p0 += 2 * step) {
#pragma unroll
		for (int u = 0; u < U; u++)
			fb[u] = resolve<Grid<G, K>::DW, FEAT, A>(a, d[u], has(p0 + step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 2 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K, TL>(fb, lane, vb);
		consume_any<G, U, K, ORD, FEAT, A>(a, fa, va, lane, p0, nseg);

#pragma unroll
		for (int u = 0; u < U; u++)
			fa[u] = resolve<Grid<G, K>::DW, FEAT, A>(a, d[u],
							has(p0 + 2 * step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 3 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K, TL>(fa, lane, va);
		consume_any<G, U, K, ORD, FEAT, A>(a, fb, vb, lane, p0 + step, nseg);
	}
#ifdef XCSUM_WAVE_STAMPS
	const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
	__builtin_amdgcn_s_waitcnt(0xC07F);
	const uint32_t wv = (blockIdx.x * 256u + threadIdx.x) >> 6;
	if ((threadIdx.x & 63u) == 0u && wv < WAVE_STAMPS_MAX) {
		g_wave_stamps[2 * wv] = t_start;
		g_wave_stamps[2 * wv + 1] = t_end;
	}
#endif
}

/* The identity order gets its own copy of the loop, so descriptor-order
 * batches pay nothing for the region order; which copy runs is decided once
 * per launch (uniform branch, after resolve_order). */
template <int G, int U, int K, int FEAT, int TL = 0>
static __device__ __forceinline__ void csum_body(CsumArgs &a)
{
	resolve_order(a);
	if (a.ord.rshift == 0)
		csum_loop<G, U, K, false, FEAT, CsumArgs, TL>(a);
	else
		csum_loop<G, U, K, true, FEAT, CsumArgs, TL>(a);
}

template <int G, int U, int K, int FEAT>
__global__ void __launch_bounds__(256) csum_kernel(CsumArgs a)
{
	csum_body<G, U, K, FEAT>(a);
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

/* ---- claimed tail (xcsum_ctx_set_tuning XCSUM_TUNE_CLAIM, A/B) -----------
 * csum_kernel's static schedule gives every segment the same number of
 * frames; with mixed frame sizes (config 5) and unequal bandwidth between
 * CUs the waves end at different times, and the last ones run alone
 * (tools/wave_tail.py).  csum_kernel_claim runs the same pipeline over the
 * first `from` logical frames statically, then every wave claims chunks of
 * `chunk` logical frames from a device counter (one returning atomic per
 * chunk, wave-uniform), so the waves that are ahead take the tail.  The
 * counter pair lives in a ring of the context (claim[0] next offset,
 * claim[1] waves done); the last wave to finish resets both, so the next
 * launch that gets this slot finds them zero. */
struct ClaimArgs {
	CsumArgs a;
	uint32_t *claim;
	uint32_t from;                 /* multiple of the static step */
	uint32_t chunk;                /* multiple of (64 / G) * U */
};

/* csum_loop's pipeline over the logical range of one segment: frames seg,
 * seg + nseg, ... below limit (nseg = spacing of the U slots of a step) */
template <int G, int U, int K, bool ORD, int FEAT>
static __device__ __forceinline__ void csum_range(const CsumArgs &a, uint32_t seg, uint32_t nseg,
						  uint32_t limit)
{
	const uint32_t lane = threadIdx.x & (G - 1);
	const uint32_t step = nseg * U;
	if (G == 64)
		seg = __builtin_amdgcn_readfirstlane(seg);
	auto has = [&](uint32_t q) { return q < limit && fidx<ORD>(a, q) < a.n; };
	u32x4 d[U];
	Frame fa[U];
	u32x4 va[U][K];
#pragma unroll
	for (int u = 0; u < U; u++)
		d[u] = load_desc<G == 64>(a, fidx<ORD>(a, seg + u * nseg));
#pragma unroll
	for (int u = 0; u < U; u++)
		fa[u] = resolve<Grid<G, K>::DW, FEAT, CsumArgs>(a, d[u], has(seg + u * nseg));
#pragma unroll
	for (int u = 0; u < U; u++)
		d[u] = load_desc<G == 64>(a, fidx<ORD>(a, seg + step + u * nseg));
	__builtin_amdgcn_sched_barrier(0);
	issue<G, U, K, 0>(fa, lane, va);
	Frame fb[U];
	u32x4 vb[U][K];
	for (uint32_t p0 = seg; p0 < limit; p0 += 2 * step) {
#pragma unroll
		for (int u = 0; u < U; u++)
			fb[u] = resolve<Grid<G, K>::DW, FEAT, CsumArgs>(a, d[u], has(p0 + step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 2 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K, 0>(fb, lane, vb);
		consume_any<G, U, K, ORD, FEAT, CsumArgs>(a, fa, va, lane, p0, nseg);
#pragma unroll
		for (int u = 0; u < U; u++)
			fa[u] = resolve<Grid<G, K>::DW, FEAT, CsumArgs>(a, d[u],
								has(p0 + 2 * step + u * nseg));
#pragma unroll
		for (int u = 0; u < U; u++)
			d[u] = load_desc<G == 64>(a, fidx<ORD>(a, p0 + 3 * step + u * nseg));
		__builtin_amdgcn_sched_barrier(0);
		issue<G, U, K, 0>(fa, lane, va);
		consume_any<G, U, K, ORD, FEAT, CsumArgs>(a, fb, vb, lane, p0 + step, nseg);
	}
}

template <int G, int U, int K, bool ORD, int FEAT>
static __device__ __forceinline__ void claim_loop(const ClaimArgs &c, const CsumArgs &a)
{
#ifdef XCSUM_WAVE_STAMPS
	const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
	__builtin_amdgcn_s_waitcnt(0xC07F);
#endif
	constexpr uint32_t W = 64u / G;      /* segments per wave */
	const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * 256u + threadIdx.x) >> 6);
	const uint32_t j = (threadIdx.x & 63u) / G;
	const uint32_t nwaves = gridDim.x * 4u;
	const uint32_t limit = ORD ? a.ord.nlog : a.n;
	/* the static part: csum_kernel's schedule below `from` */
	csum_range<G, U, K, ORD, FEAT>(a, wave * W + j, nwaves * W, c.from < limit ? c.from : limit);
	/* the claimed part: chunks of consecutive logical frames, the wave's
	 * segment j taking frames base + j + u * W + i * W * U */
	for (;;) {
		uint32_t got = 0;
		if ((threadIdx.x & 63u) == 0u)
			got = atomicAdd(&c.claim[0], c.chunk);
		const uint32_t base = __builtin_amdgcn_readfirstlane(got) + c.from;
		if (base >= limit || base < c.from)
			break;
		const uint32_t end = limit - base > c.chunk ? base + c.chunk : limit;
		csum_range<G, U, K, ORD, FEAT>(a, base + j, W, end);
	}
	/* the last wave out resets the slot for the launch that reuses it */
	if ((threadIdx.x & 63u) == 0u && atomicAdd(&c.claim[1], 1u) == nwaves - 1u) {
		atomicExch(&c.claim[0], 0u);
		atomicExch(&c.claim[1], 0u);
	}
#ifdef XCSUM_WAVE_STAMPS
	const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
	__builtin_amdgcn_s_waitcnt(0xC07F);
	const uint32_t wv = (blockIdx.x * 256u + threadIdx.x) >> 6;
	if ((threadIdx.x & 63u) == 0u && wv < WAVE_STAMPS_MAX) {
		g_wave_stamps[2 * wv] = t_start;
		g_wave_stamps[2 * wv + 1] = t_end;
	}
#endif
}

template <int G, int U, int K, int FEAT>
__global__ void __launch_bounds__(256) csum_kernel_claim(ClaimArgs c)
{
	CsumArgs a = c.a;
	resolve_order(a);
	if (a.ord.rshift == 0)
		claim_loop<G, U, K, false, FEAT>(c, a);
	else
		claim_loop<G, U, K, true, FEAT>(c, a);
}

/* static_64: the static share in 64ths of the logical range; chunk_steps:
 * wave steps per claim */
template <int G, int U, int K, int FEAT>
static hipError_t launch_claim_t(const CsumArgs &a, int cus, int bpc, uint32_t *claim,
				 uint32_t static_64, uint32_t chunk_steps, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, csum_kernel_claim<G, U, K, FEAT>,
								 256, 0) != hipSuccess || nb <= 0)
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
	ClaimArgs c;
	c.a = a;
	c.claim = claim;
	/* the static step of the grid: every segment's U frames */
	const uint64_t step = blocks * (256u / G) * U;
	const uint64_t nlog = a.ord.nlog;   /* >= n; the dense order may differ, which
					       only moves the split point */
	c.from = (uint32_t)((nlog * static_64 / 64u) / step * step);
	c.chunk = (uint32_t)(chunk_steps * (64u / G) * U);
	(void)hipGetLastError();
	hipLaunchKernelGGL((csum_kernel_claim<G, U, K, FEAT>), dim3((unsigned)blocks), dim3(256), 0,
			   s, c);
	return hipGetLastError();
}

/* the geometries with a claimed-tail kernel */
#define XCSUM_CLAIM_GEOMETRIES(X) X(64, 1, 9) X(64, 1, 2) X(16, 2, 6)

#define XCSUM_GEOMETRIES(X) \
	X(64, 1, 2) X(64, 1, 9) X(32, 1, 3) X(32, 1, 6) \
	X(16, 1, 2) X(16, 1, 3) X(16, 1, 6) X(16, 2, 6) X(16, 1, 12) \
	X(8, 1, 2) X(8, 2, 1) X(8, 1, 12) X(4, 2, 2) X(4, 4, 2) X(4, 1, 2) \
	X(2, 1, 4) X(2, 2, 4) X(1, 1, 6) X(1, 1, 8) X(1, 2, 6)

/* extra geometries for tuning sweeps only (make variant DEFS=-DXCSUM_SWEEP_GEOMS):
 * plain instantiation, not in the tested table */
#ifdef XCSUM_SWEEP_GEOMS
#define XCSUM_SWEEP_GEOMETRIES(X) X(16, 3, 6) X(16, 4, 6) X(32, 2, 3) X(32, 3, 3) X(16, 3, 5) X(8, 4, 12) \
	X(64, 2, 9) X(64, 1, 12) X(64, 2, 6) X(32, 2, 9) X(64, 3, 6)
#else
#define XCSUM_SWEEP_GEOMETRIES(X)
#endif

} /* namespace xcsum */

#endif
