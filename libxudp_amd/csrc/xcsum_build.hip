/*
 * xcsum_build.hip -- xudp_frame_send's per-frame work on the GPU.
 *
 * For message i (payload bytes + a UMEM frame slot) build, in one pass over
 * the payload, the frame xudp_packet_udp() builds (cclinuxer/libxudp
 * xudp/packet.c:156-194): eth + IPv4/IPv6 + UDP headers in front of the
 * payload, iph->check (xudp_checksum_half, packet.c:43-66), udp->check
 * (IPv6 udp_csum6, packet.c:105-117; IPv4 0 as packet.c:125, RFC on request),
 * copying the payload into the slot first unless it is already there (the
 * memcpy of xudp_packet_udp_payload, packet.c:196-203, fused with the
 * checksum: every payload byte is read once, written once, summed from
 * registers), then the xdp_desc the frame is published with (tx.c:450-452).
 *
 * The batch shares one route (xudp_tx_info_prepare, tx.c:690), so the host
 * passes a 64-byte header template holding every constant header byte
 * (addresses, ports, MACs, version/TTL/protocol/DF); the kernel patches the
 * per-frame length fields and both checksums.  All checksum arithmetic is
 * here, none on the host.
 *
 * Memory-bound: payload read + frame write (+ 16-byte message, 16-byte
 * descriptor) per frame.  G lanes per frame, K 16-byte chunks per lane
 * preloaded, longer payloads stream through a tail loop.
 */
#include "xcsum_internal.h"
#include "xcsum_device.h"
#include <stdio.h>
#include <stdlib.h>

namespace xcsum {

static __device__ __forceinline__ u32x4 ld16(const uint8_t *p)
{
	return __builtin_nontemporal_load((gu32x4 *)p);
}

static __device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int n)
{
	/* bytes [0, n) of a dword, n clamped to [0, 4] */
	return n >= 4 ? w : (n <= 0 ? 0u : (w & (0xffffffffu >> (32 - 8 * n))));
}

/* One build message resolved: where its payload comes from (src, 16-byte
 * aligned block base `blk` and phase `sh`), where its frame goes. */
struct Msg {
	const uint8_t *blk;     /* src & ~15 */
	uint8_t *data;          /* frame slot data pointer (16-aligned) */
	uint64_t data_off;      /* umem offset of data */
	uint32_t len, sh;
	bool ok, present;
#ifdef XCSUM_DEBUG_BOUNDS
	const uint8_t *slot, *slot_end;   /* the frame slot: every store stays inside */
	const uint8_t *blk_end;           /* src rounded up to 16 past the payload */
#endif
};

static __device__ __forceinline__ Msg resolve_msg(const BuildArgs &a, u32x4 m, bool present,
						  bool inplace)
{
	Msg g;
	const uint64_t srcoff = ((uint64_t)m.y << 32) | m.x;
	asm volatile("" ::"v"(m.w), "v"(m.z));
	g.len = m.z;
	g.data_off = (uint64_t)m.w * a.frame_size + a.data_off;
	g.data = a.umem + g.data_off;
	g.ok = present && m.z <= 65527u && (uint64_t)a.data_off + m.z <= a.frame_size;
	g.present = present;
	const uint8_t *src = inplace ? (const uint8_t *)g.data : a.src + srcoff;
	g.sh = (uint32_t)(uintptr_t)src & 15u;
	g.blk = (const uint8_t *)((uintptr_t)src & ~(uintptr_t)15);
	if (!g.ok)
		g.len = 0;
#ifdef XCSUM_DEBUG_BOUNDS
	g.slot = a.umem + (uint64_t)m.w * a.frame_size;
	g.slot_end = g.slot + a.frame_size;
	g.blk_end = (const uint8_t *)(((uintptr_t)src + g.len + 15u) & ~(uintptr_t)15);
#endif
	return g;
}

__device__ u32x4 g_zero_block[4];

/* The payload's aligned 16-byte blocks, block c = lane + k*G in v[k]; with
 * TWO (unaligned sources) also block K*G in lane 0's `vx`: chunk c of the
 * payload straddles blocks c and c + 1.  Blocks holding no payload byte load
 * zeros instead (nothing is read past the payload's last aligned block). */
template <int G, int K, bool TWO>
static __device__ __forceinline__ void issue_blocks(const Msg &g, uint32_t lane, u32x4 (&v)[K],
						    u32x4 &vx)
{
	const uint8_t *zero = (const uint8_t *)g_zero_block;
	const uint32_t end = g.len + g.sh;          /* block offsets below hold payload */
#pragma unroll
	for (int k = 0; k < K; k++) {
		const uint32_t off = 16u * (lane + k * G);
		v[k] = ld16(off < end ? XB_LOAD(g.blk + off, 16, g.blk, g.blk_end, XB_BUILD_SRC, off, zero)
				      : zero);
	}
	if (TWO)
		vx = ld16(lane == 0 && 16u * K * G < end
				  ? XB_LOAD(g.blk + 16u * K * G, 16, g.blk, g.blk_end, XB_BUILD_SRC,
					    16u * K * G, zero)
				  : zero);
}

/* a where the lane's bit of `lanes` is clear, b where it is set: v_cndmask
 * through inline asm, so the compiler cannot fold a select chain back into a
 * runtime-indexed (scratch) array read */
static __device__ __forceinline__ uint32_t pick(uint32_t a, uint32_t b, uint64_t lanes)
{
	uint32_t r;
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(lanes));
	return r;
}

/* the chunk's 16 payload bytes from its two blocks (byte shift by sh), bytes
 * past the payload cleared */
static __device__ __forceinline__ u32x4 shift_chunk(u32x4 v0, u32x4 v1, uint32_t sh, uint32_t rem)
{
	u32x4 r;
	if (sh == 0) {
		r = v0;
	} else {
		const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
		const uint32_t q = sh >> 2, s8 = sh & 3u;
		const uint64_t m1 = __builtin_amdgcn_ballot_w64(q == 1);
		const uint64_t m2 = __builtin_amdgcn_ballot_w64(q == 2);
		const uint64_t m3 = __builtin_amdgcn_ballot_w64(q == 3);
		uint32_t o[5];
#pragma unroll
		for (int j = 0; j < 5; j++)
			o[j] = pick(pick(pick(w[j], w[j + 1], m1), w[j + 2], m2), w[j + 3], m3);
		r.x = __builtin_amdgcn_alignbyte(o[1], o[0], s8);
		r.y = __builtin_amdgcn_alignbyte(o[2], o[1], s8);
		r.z = __builtin_amdgcn_alignbyte(o[3], o[2], s8);
		r.w = __builtin_amdgcn_alignbyte(o[4], o[3], s8);
	}
	if (rem < 16) {
		r.x = keep_bytes(r.x, (int)rem);
		r.y = keep_bytes(r.y, (int)rem - 4);
		r.z = keep_bytes(r.z, (int)rem - 8);
		r.w = keep_bytes(r.w, (int)rem - 12);
	}
	return r;
}

/* slow path for payloads longer than K*G chunks: plain walk */
static __device__ __forceinline__ u32x4 load_payload(const uint8_t *blk, uint32_t sh, uint32_t off,
						     uint32_t rem)
{
	u32x4 v0 = ld16(blk + off);
	u32x4 v1 = (sh != 0 && 16u - sh < rem) ? ld16(blk + off + 16) : u32x4{0, 0, 0, 0};
	return shift_chunk(v0, v1, sh, rem);
}

/* the chunk's first min(rem, 16) bytes to d (16-byte aligned): a full chunk
 * is one non-temporal 16-byte store; a payload's last, partial chunk is up
 * to three dword stores, a short and a byte -- all at static offsets (the
 * byte-by-byte loop this replaces held ~100 VGPRs of addresses) */
static __device__ __forceinline__ void store_payload(uint8_t *d, u32x4 v, uint32_t rem)
{
	if (rem >= 16) {
		__builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4 *)d);
		return;
	}
	const uint32_t nd = rem >> 2, t = rem & 3u;
	if (nd >= 1)
		*reinterpret_cast<uint32_t *>(d) = v.x;
	if (nd >= 2)
		*reinterpret_cast<uint32_t *>(d + 4) = v.y;
	if (nd >= 3)
		*reinterpret_cast<uint32_t *>(d + 8) = v.z;
	if (t) {
		const uint32_t w = nd == 0 ? v.x : (nd == 1 ? v.y : (nd == 2 ? v.z : v.w));
		uint8_t *q = d + 4 * nd;
		if (t & 2u)
			*reinterpret_cast<uint16_t *>(q) = (uint16_t)w;
		if (t & 1u)
			q[t & 2u] = (uint8_t)(w >> (8 * (t & 2u)));
	}
}

/* header bytes + descriptor + result for one built frame (s = payload sum,
 * in every lane of the segment).  The header is written as the four 16-byte
 * pieces of [data - 64, data) (data is 16-byte aligned): piece i comes from
 * the batch's header image in LDS (template right-aligned at byte 64 - hdr),
 * the per-frame length and check halfwords are patched in at their static
 * positions, and lanes 0..3 store one piece each -- full pieces with one
 * 16-byte store, the piece holding the header's first bytes with a short,
 * (a dword,) and a dwordx2.  (A halfword-per-store loop cost ~10 store
 * instructions per frame.) */
template <int G>
static __device__ __forceinline__ void finish_frame(const BuildArgs &a, const Msg &g, uint32_t p,
						    uint32_t s, uint32_t lane, const u32x4 *img,
						    bool v6, uint32_t hdr, uint32_t sconst,
						    uint32_t ipconst)
{
	if (!g.ok) {
		if (lane == 0 && XB_IDX(p, a.n, XB_BUILD_OUT)) {
			struct xcsum_desc d0 = {g.data_off, 0u, 0u};
			a.desc_out[p] = d0;
			if (a.out)
				a.out[p] = 0;
			atomicAdd(a.err, 1ull);
		}
		return;
	}
	const uint32_t ulen = 8u + g.len;
	/* S = payload + addresses + ports + 17 + udp_len (pseudo) + udp_len
	 * (header); the header's check field is 0 */
	uint32_t S = s + sconst + 2u * ulen;
	uint32_t t = (S & 0xffffu) + (S >> 16);
	t = (t & 0xffffu) + (t >> 16);
	uint32_t r = ~t & 0xffffu;
	if (r == 0)
		r = 0xffffu;                               /* CSUM_MANGLED_0 */
	uint32_t ucheck = (v6 || (a.flags & XCSUM_F_V4_RFC)) ? bswap16(r) : 0u;
	uint32_t ipcheck = 0;
	if (!v6) {
		uint32_t ip = ipconst + 20u + ulen;        /* + tot_len */
		ip = (ip & 0xffffu) + (ip >> 16);
		ip = (ip & 0xffffu) + (ip >> 16);
		ipcheck = bswap16(~ip & 0xffffu);
	}
	if (lane < 4) {
		u32x4 w = img[lane];
		/* image byte of header byte b: 64 - hdr + b.  IPv4 (at 22):
		 * tot_len 38, check 46, udp len 60, udp check 62.  IPv6 (at 2):
		 * payload_len 20, udp len 60, udp check 62. */
		if (v6) {
			if (lane == 1)
				w.y = (w.y & 0xffff0000u) | bswap16(ulen);
		} else if (lane == 2) {
			w.y = (w.y & 0x0000ffffu) | (bswap16(20u + ulen) << 16);
			w.w = (w.w & 0x0000ffffu) | (ipcheck << 16);
		}
		if (lane == 3)
			w.w = bswap16(ulen) | (ucheck << 16);
		uint8_t *pb = g.data - 64 + 16 * lane;
		const uint32_t first = v6 ? 0u : 1u;      /* piece holding header byte 0 */
		/* the header's pieces: [data - hdr, data) */
		if (lane >= first &&
		    !XB_STORE(lane > first ? pb : g.data - hdr,
			      lane > first ? 16u : 16u * (lane + 1) - (64u - hdr), g.slot, g.slot_end,
			      XB_BUILD_DATA, 64u - 16u * lane)) {
			/* outside the slot: not written (debug build only) */
		} else if (lane > first) {
			*reinterpret_cast<u32x4 *>(pb) = w;
		} else if (lane == first) {
			if (v6) {                          /* bytes 2..15 */
				*reinterpret_cast<uint16_t *>(pb + 2) = (uint16_t)(w.x >> 16);
				*reinterpret_cast<uint32_t *>(pb + 4) = w.y;
			} else {                           /* bytes 6..15 */
				*reinterpret_cast<uint16_t *>(pb + 6) = (uint16_t)(w.y >> 16);
			}
			typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
			*reinterpret_cast<u32x2 *>(pb + 8) = u32x2{w.z, w.w};
		}
	}
	if (lane == 0 && XB_IDX(p, a.n, XB_BUILD_OUT)) {
		struct xcsum_desc d0 = {g.data_off - hdr, hdr + g.len, 0u};
		a.desc_out[p] = d0;
		if (a.out)
			a.out[p] = (uint16_t)ucheck;
	}
}

/* Dwords of the LDS stage per group (TWO): K*G + 1 blocks and one block of
 * slack for the fifth dword the last chunk reads. */
template <int G, int K>
struct Stage {
	static constexpr uint32_t DW = 4 * (K * G + 2);
};

/* Copy (unless in place), sum, header and descriptor of one message whose
 * payload blocks v[] have landed.  Group-uniform; every lane calls it.
 * Unaligned sources (TWO) are realigned through the group's LDS stage: the
 * blocks go in as they are, and chunk c comes back as the five dwords from
 * byte sh + 16c, byte-shifted with v_alignbyte.  One load and no dword
 * selects per chunk; loading both straddled blocks and selecting in
 * registers took two loads, 15 v_cndmask and twice the registers. */
template <int G, int K, bool TWO>
static __device__ __forceinline__ void build_msg(const BuildArgs &a, const Msg &gc,
						 const u32x4 (&vc)[K], const u32x4 &vx, uint32_t ic,
						 uint32_t lane, bool inplace, const u32x4 *img,
						 bool v6, uint32_t hdr, uint32_t sconst,
						 uint32_t ipconst, uint32_t *st)
{
	uint32_t E = 0, O = 0;
	if (__builtin_amdgcn_ballot_w64(gc.len > 16u * K * G)) {
		/* jumbo payloads: plain walk (own copy of the body) */
		for (uint32_t off = 16u * lane; off < gc.len; off += 16u * G) {
			u32x4 v = XB_IN(gc.blk + off, (gc.sh && 16u - gc.sh < gc.len - off) ? 32u : 16u,
					gc.blk, gc.blk_end, XB_BUILD_SRC, off)
					  ? load_payload(gc.blk, gc.sh, off, gc.len - off)
					  : u32x4{0u, 0u, 0u, 0u};
			if (!inplace && XB_STORE(gc.data + off, gc.len - off < 16u ? gc.len - off : 16u,
						 gc.slot, gc.slot_end, XB_BUILD_DATA, off))
				store_payload(gc.data + off, v, gc.len - off);
			accum(v, E, O);
		}
	} else if (TWO) {
		/* the stage was last read by this group's previous message */
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
		for (int k = 0; k < K; k++)
			*((u32x4 *)(st + 4 * (lane + k * G))) = vc[k];
		if (lane == 0)
			*((u32x4 *)(st + 4 * K * G)) = vx;
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		const uint32_t s8 = gc.sh & 3u;
#pragma unroll
		for (int k = 0; k < K; k++) {
			const uint32_t off = 16u * (lane + k * G);
			if (off < gc.len) {
				const uint32_t *q = st + (gc.sh >> 2) + 4 * (lane + k * G);
				const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
				u32x4 v = {__builtin_amdgcn_alignbyte(d1, d0, s8),
					   __builtin_amdgcn_alignbyte(d2, d1, s8),
					   __builtin_amdgcn_alignbyte(d3, d2, s8),
					   __builtin_amdgcn_alignbyte(d4, d3, s8)};
				v = shift_chunk(v, v, 0u, gc.len - off);     /* clear past the end */
				if (!inplace && XB_STORE(gc.data + off, gc.len - off < 16u ? gc.len - off : 16u,
							 gc.slot, gc.slot_end, XB_BUILD_DATA, off))
					store_payload(gc.data + off, v, gc.len - off);
				accum(v, E, O);
			}
		}
	} else {
#pragma unroll
		for (int k = 0; k < K; k++) {
			uint32_t off = 16u * (lane + k * G);
			if (off < gc.len) {
				u32x4 v = shift_chunk(vc[k], vc[k], 0u, gc.len - off);
				if (!inplace && XB_STORE(gc.data + off, gc.len - off < 16u ? gc.len - off : 16u,
							 gc.slot, gc.slot_end, XB_BUILD_DATA, off))
					store_payload(gc.data + off, v, gc.len - off);
				accum(v, E, O);
			}
		}
	}
	/* payload starts 16-aligned (even address): E holds high bytes */
	uint32_t s = seg_sum<G>((E << 8) + O);
	if (gc.present)
		finish_frame<G>(a, gc, ic, s, lane, img, v6, hdr, sconst, ipconst);
}

/*
 * Persistent grid, G lanes per message, the checksum kernel's two-stage
 * pipeline written as a ping-pong over two register sets (A, B): message
 * i+1's payload blocks and message i+2's descriptor are in flight while
 * message i is shifted, stored, summed and headed.  (A "next" set copied into
 * "current" at the loop latch would wait for the in-flight loads there.)
 */
/* The batch's header template in LDS: tmpl = memory-order halfwords (big-
 * endian word j of the header is bswap16(tmpl[j])), img = the template
 * right-aligned in 64 bytes.  Returns the constant parts of the sums: the
 * UDP checksum's pseudo-header addresses and ports (header halfwords 13..18 /
 * 11..28) + protocol 17, and the IPv4 header sum without tot_len and check
 * (halfwords 7..16).  Block-wide (__syncthreads). */
static __device__ __forceinline__ void load_template(const BuildArgs &a, uint16_t *tmpl, u32x4 *img,
						     bool v6, uint32_t hdr, uint32_t &sconst,
						     uint32_t &ipconst)
{
	if (threadIdx.x < 32)
		tmpl[threadIdx.x] = (uint16_t)(a.tmpl[threadIdx.x / 2] >> (16 * (threadIdx.x & 1)));
	if (threadIdx.x < 64) {
		const uint32_t b = threadIdx.x, pad = 64u - hdr;
		const uint8_t v = b < pad ? 0u : (uint8_t)(a.tmpl[(b - pad) >> 2] >> (8 * ((b - pad) & 3)));
		reinterpret_cast<uint8_t *>(img)[b] = v;
	}
	__syncthreads();
	sconst = 17u;
	for (uint32_t j = v6 ? 11u : 13u; j < (v6 ? 29u : 19u); j++)
		sconst += bswap16(tmpl[j]);
	ipconst = 0;
	if (!v6)
		for (uint32_t j = 7; j < 17; j++)
			if (j != 8 && j != 12)
				ipconst += bswap16(tmpl[j]);
}

template <int G, int K, bool TWO>
__global__ void __launch_bounds__(256) build_kernel(BuildArgs a)
{
	__shared__ uint16_t tmpl[32];
	__shared__ __attribute__((aligned(16))) u32x4 img[4];
	const bool v6 = a.family == 6;
	const uint32_t hdr = v6 ? 62u : 42u;
	uint32_t sconst, ipconst;
	load_template(a, tmpl, img, v6, hdr, sconst, ipconst);

	const uint32_t lane = threadIdx.x & (G - 1);
	const uint32_t seg = (blockIdx.x * 256u + threadIdx.x) / G;
	const uint32_t nseg = gridDim.x * (256u / G);
	const bool inplace = (a.flags & XCSUM_F_BUILD_INPLACE) != 0;
	const uint32_t last = a.n - 1;
	/* message index of logical position q in the batch's visiting order
	 * (a.ord); >= n: none (past the logical range frame_of would alias) */
	auto idx = [&](uint32_t q) { return q < a.ord.nlog ? frame_of(a.ord, q) : a.n; };
	auto msg = [&](uint32_t i) { return *((gu32x4 *)(a.msgs + (i < a.n ? i : last))); };

	uint32_t ia = idx(seg);
	u32x4 d = msg(ia);
	Msg ga = resolve_msg(a, d, ia < a.n, inplace);
	uint32_t ib = idx(seg + nseg);
	d = msg(ib);
	__builtin_amdgcn_sched_barrier(0);
	__shared__ __attribute__((aligned(16))) uint32_t stage[TWO ? (256 / G) * Stage<G, K>::DW : 4];
	uint32_t *st = stage + (TWO ? (threadIdx.x / G) * Stage<G, K>::DW : 0u);
	u32x4 va[K], vb[K], xa, xb;
	issue_blocks<G, K, TWO>(ga, lane, va, xa);

	for (uint32_t p = seg; p < a.ord.nlog; p += 2 * nseg) {
		Msg gb = resolve_msg(a, d, ib < a.n, inplace);
		const uint32_t ia2 = idx(p + 2 * nseg);
		d = msg(ia2);
		__builtin_amdgcn_sched_barrier(0);
		issue_blocks<G, K, TWO>(gb, lane, vb, xb);
		__builtin_amdgcn_sched_barrier(0);
		build_msg<G, K, TWO>(a, ga, va, xa, ia, lane, inplace, img, v6, hdr, sconst, ipconst,
				     st);

		ga = resolve_msg(a, d, ia2 < a.n, inplace);
		ia = ia2;
		const uint32_t ib2 = idx(p + 3 * nseg);
		d = msg(ib2);
		__builtin_amdgcn_sched_barrier(0);
		issue_blocks<G, K, TWO>(ga, lane, va, xa);
		__builtin_amdgcn_sched_barrier(0);
		build_msg<G, K, TWO>(a, gb, vb, xb, ib, lane, inplace, img, v6, hdr, sconst, ipconst,
				     st);
		ib = ib2;
	}
}


/*
 * IPv4 in place without XCSUM_F_V4_RFC: libxudp's default IPv4 send on
 * frames whose payload already sits in its slot (the xudp_frame_alloc path,
 * tx.c:760).  The reference computes only iph->check there (iph_build ->
 * xudp_checksum_half, packet.c:43-66, :83) and leaves udp->check 0
 * (packet.c:125), so no payload byte is read: per message the 16-byte
 * message in, the 42 header bytes and the 16-byte descriptor out.  Four lanes
 * per message store the header pieces (finish_frame<4>; lane 0 holds no
 * IPv4 header byte and writes the descriptor); the next message is loaded
 * while this one is written.
 */
__global__ void __launch_bounds__(256) build_hdr_kernel(BuildArgs a)
{
	__shared__ uint16_t tmpl[32];
	__shared__ __attribute__((aligned(16))) u32x4 img[4];
	uint32_t sconst, ipconst;
	load_template(a, tmpl, img, false, 42u, sconst, ipconst);
	const uint32_t lane = threadIdx.x & 3u;
	const uint32_t seg = (blockIdx.x * 256u + threadIdx.x) / 4u;
	const uint32_t nseg = gridDim.x * 64u;
	const uint32_t last = a.n - 1;
	auto idx = [&](uint32_t q) { return q < a.ord.nlog ? frame_of(a.ord, q) : a.n; };
	auto msg = [&](uint32_t i) { return *((gu32x4 *)(a.msgs + (i < a.n ? i : last))); };
	uint32_t i = idx(seg);
	u32x4 d = msg(i);
	for (uint32_t p = seg; p < a.ord.nlog; p += nseg) {
		const uint32_t i2 = idx(p + nseg);
		const u32x4 d2 = msg(i2);
		const Msg g = resolve_msg(a, d, i < a.n, true);
		if (g.present)
			finish_frame<4>(a, g, i, 0u, lane, img, false, 42u, sconst, ipconst);
		i = i2;
		d = d2;
	}
}

static hipError_t launch_build_hdr(const BuildArgs &a, int cus, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, build_hdr_kernel, 256, 0) !=
			    hipSuccess || nb <= 0)
			nb = 8;
		return nb;
	});
	uint64_t blocks = ((uint64_t)a.ord.nlog * 4 + 255) / 256;
	const uint64_t cap = (uint64_t)cus * occ;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();
	hipLaunchKernelGGL(build_hdr_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

template <int G, int K, bool TWO>
static hipError_t launch_build_t(const BuildArgs &a, int cus, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, build_kernel<G, K, TWO>, 256,
								 0) != hipSuccess || nb <= 0)
			nb = 4;
		return nb;
	});
	uint64_t blocks = ((uint64_t)a.ord.nlog * G + 255) / 256;
	uint64_t cap = (uint64_t)cus * occ;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();  /* clear a stale error (e.g. hipErrorNotReady from
	                           * someone's hipEventQuery) before checking ours */
	hipLaunchKernelGGL((build_kernel<G, K, TWO>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

#define XCSUM_BUILD_GEOMETRIES(X) \
	X(4, 1) X(8, 2) X(16, 2) X(16, 3) X(16, 6) X(32, 3) X(64, 2) X(64, 9)

/* t: the context's tuning -- build_hdr false (A/B, tests) sends IPv4 in
 * place through the payload-summing build kernel, as before round 5;
 * build_G/K force a geometry (sweeps) */
hipError_t launch_build(const BuildArgs &a, uint32_t len_hint, int cus, const Tuning &t,
			hipStream_t s)
{
	if (a.n == 0)
		return hipSuccess;
	if (a.family == 4 && (a.flags & XCSUM_F_BUILD_INPLACE) && !(a.flags & XCSUM_F_V4_RFC) &&
	    t.build_hdr)
		return launch_build_hdr(a, cus, s);
	/* payloads read from 16-byte aligned addresses need one block per chunk */
	const bool two = !(a.flags & (XCSUM_F_BUILD_INPLACE | XCSUM_F_SRC_ALIGNED));
	int G = t.build_G, K = t.build_K;
	if (!G) {
		/* lanes x chunks to cover a typical payload in one preload */
		uint32_t chunks = (len_hint + 15) / 16;
		if (chunks <= 4) { G = 4; K = 1; }
		else if (chunks <= 16) { G = 8; K = 2; }
		else if (chunks <= 96) {
			/* MTU payloads, measured (tools/bench_build.py,
			 * profiles/r01/build/pingpong_*.log): 5.1-5.3 TB/s moved at (16,6) */
			G = 16;
			K = 6;
		}
		else { G = 64; K = 9; }
	}
#define X(g_, k_)                                                                       \
	if (G == g_ && K == k_)                                                         \
		return two ? launch_build_t<g_, k_, true>(a, cus, s)                    \
			   : launch_build_t<g_, k_, false>(a, cus, s);
	XCSUM_BUILD_GEOMETRIES(X)
#undef X
	return hipErrorInvalidValue;
}

/* xcsum_ctx_set_tuning(XCSUM_TUNE_BUILD_GEOMETRY): compiled in? */
bool build_geometry_supported(int G, int K)
{
#define X(g_, k_) if (G == g_ && K == k_) return true;
	XCSUM_BUILD_GEOMETRIES(X)
#undef X
	return false;
}

} /* namespace xcsum */
