/* xcsum_frame.h -- the frame-group checksum machinery shared by the checksum
 * kernel (xcsum_kernels.hip) and the receive kernel built on the same
 * pipeline (xcsum_rx.hip): a frame's chunk grid, chunk loads, edge masks,
 * the per-frame sums.  Static device functions: each translation unit gets
 * its own copy of the code, one source. */
#ifndef XCSUM_FRAME_H
#define XCSUM_FRAME_H

#include "xcsum_internal.h"
#include "xcsum_device.h"

namespace xcsum {

/* Per-frame geometry: the span [lo, hi) is covered by nchunks 16-byte
 * chunks from base, with `head` bytes before lo in the first chunk and
 * `tail` bytes after hi in the last one.  Two chunk grids (template DW):
 *   DW = true: laid back from E4 = hi rounded up to 4 bytes, chunk c =
 *     [E4 - 16*(nchunks - c), ...).  Chunks are dword aligned (16-byte loads
 *     at dword alignment stream at full rate, 2-byte aligned ones do not,
 *     tools/slot_probe.py); head 0..15 (the first chunk starts inside the
 *     frame's headers), tail 0..3; both masked to zero BEFORE summing.
 *   DW = false: 16-byte aligned from lo & ~15; head and tail 0..15, summed
 *     and then taken back out of E/O by the lanes holding the edge chunks.
 * Neither reads past the 16-byte block (DW: the dword) holding hi - 1.
 * DW wins where edge work is a large share (small frames, G = 64); aligned
 * chunks win by ~1% for MTU frames at G = 16 (profiles/r01/ab). */
struct Frame {
	const uint8_t *base;
	uint8_t *eth;
	uint32_t nchunks;       /* 0: nothing to load (malformed / absent) */
	uint32_t head, tail;    /* 0..15 bytes to drop at either end */
	uint32_t udp_len;
	uint32_t odd;           /* span starts at an odd address */
	int mode;               /* 0 legacy, 1 rfc, 2 v6, -1 malformed, -2 absent */
	uint32_t ck;            /* VERIFY: the frame's udp->check (raw 16 bits),
				   loaded a pipeline step ahead */
	uint32_t ul;            /* VERIFY: udp->len (raw 16 bits), same load step */
	uint32_t ih[6];         /* IPHDR: the dwords holding the IPv4 header
				   [eth+14, eth+34), loaded a step ahead */
	uint32_t ihs;           /* byte phase of eth+14 in ih[0] */
#ifdef XCSUM_DEBUG_BOUNDS
	const uint8_t *lim;     /* the frame's end rounded up to 16 bytes: no
				   load may reach past it (nor before eth) */
	uint32_t dlen;          /* descriptor length: stores stay below eth + dlen */
#endif
};

/* 16 zero bytes: lanes past the end of their frame load these, so the
 * accumulation needs no data masking (one select per chunk) */
__device__ u32x4 g_zero_chunk[4];

/* chunk loads are nontemporal: every byte is read exactly once */
static __device__ __forceinline__ u32x4 load_chunk(const uint8_t *p)
{
	return __builtin_nontemporal_load((gu32x4 *)p);
}

typedef __attribute__((address_space(4))) const u32x4 cu32x4;


/* chunk grid of the span [lo, hi) (see the Frame comment) */
template <bool DW>
static __device__ __forceinline__ void set_span(Frame &f, uintptr_t lo, uintptr_t hi)
{
	f.odd = (uint32_t)lo & 1u;
	if (DW) {
		const uintptr_t e4 = (hi + 3) & ~(uintptr_t)3;
		f.nchunks = (uint32_t)(e4 - lo + 15) >> 4;
		const uintptr_t base = e4 - 16u * f.nchunks;
		f.base = (const uint8_t *)base;
		f.head = (uint32_t)(lo - base);
		f.tail = (uint32_t)(e4 - hi);
	} else {
		const uintptr_t base = lo & ~(uintptr_t)15;
		f.nchunks = (uint32_t)(hi - base + 15) >> 4;
		f.base = (const uint8_t *)base;
		f.head = (uint32_t)(lo - base);
		f.tail = (f.nchunks << 4) - (uint32_t)(hi - base);
	}
}

/* Edge masks, applied to the chunks before they are summed: the first
 * chunk keeps bytes [head, 16), the last keeps all but the top `tail` bytes
 * of its last dword.  Built from 64-bit shifts, no branches. */
static __device__ __forceinline__ u32x4 and_head(u32x4 v, uint32_t head)
{
	const uint64_t k0 = head >= 8 ? 0ull : ~0ull << (8 * (head & 7));
	const uint64_t k1 = head <= 8 ? ~0ull : ~0ull << (8 * (head & 7));
	v.x &= (uint32_t)k0;
	v.y &= (uint32_t)(k0 >> 32);
	v.z &= (uint32_t)k1;
	v.w &= (uint32_t)(k1 >> 32);
	return v;
}

static __device__ __forceinline__ uint32_t tail_keep(uint32_t tail)
{
	return 0xffffffffu >> (8 * tail);   /* tail <= 3 */
}

/* chunk c of f, masked, for the walking (jumbo) paths */
static __device__ __forceinline__ u32x4 edge_mask_one(const Frame &f, uint32_t c, u32x4 v)
{
	if (c == 0)
		v = and_head(v, f.head);
	if (c + 1 == f.nchunks)
		v.w &= tail_keep(f.tail);
	return v;
}

/* Edge masks for a frame whose chunks sit in v[0..K) of its G lanes (chunk
 * lane + k*G): lane 0 masks its first chunk, the lane holding the last
 * chunk masks that chunk's last dword.  Every lane runs the same code with
 * all-ones masks where it holds no edge.  A one-chunk frame gets both. */
template <int G, int K>
static __device__ __forceinline__ void edge_mask(const Frame &f, u32x4 (&v)[K], uint32_t lane)
{
	const uint32_t last = f.nchunks - 1;
	v[0] = and_head(v[0], lane == 0 ? f.head : 0u);
	const uint32_t tk = tail_keep(f.tail);
#pragma unroll
	for (int k = 0; k < K; k++)
		v[k].w &= lane + k * G == last ? tk : 0xffffffffu;
}

/* ---- aligned grid (DW = false): take edge bytes back out after summing */
static __device__ __forceinline__ void drop_masked(u32x4 v, uint64_t m0, uint64_t m1,
						   uint32_t &E, uint32_t &O)
{
	const uint32_t w0 = v.x & (uint32_t)m0, w1 = v.y & (uint32_t)(m0 >> 32);
	const uint32_t w2 = v.z & (uint32_t)m1, w3 = v.w & (uint32_t)(m1 >> 32);
	uint32_t e = dot_even(w0, 0u), o = dot_odd(w0, 0u);
	e = dot_even(w1, e); o = dot_odd(w1, o);
	e = dot_even(w2, e); o = dot_odd(w2, o);
	e = dot_even(w3, e); o = dot_odd(w3, o);
	E -= e;
	O -= o;
}

/* the first n / last n bytes of a chunk, n in [0, 15] (0: nothing) */
static __device__ __forceinline__ void drop_prefix(u32x4 v, uint32_t n, uint32_t &E, uint32_t &O)
{
	const uint64_t m0 = n >= 8 ? ~0ull : (1ull << (8 * (n & 7))) - 1;
	const uint64_t m1 = n <= 8 ? 0ull : (1ull << (8 * (n & 7))) - 1;
	drop_masked(v, m0, m1, E, O);
}

static __device__ __forceinline__ void drop_suffix(u32x4 v, uint32_t n, uint32_t &E, uint32_t &O)
{
	const uint64_t m1 = n == 0 ? 0ull : (n >= 8 ? ~0ull : ~0ull << (8 * (8 - n)));
	const uint64_t m0 = n <= 8 ? 0ull : ~0ull << (8 * ((16 - n) & 7));
	drop_masked(v, m0, m1, E, O);
}

/* v_cndmask_b32 through inline asm: a per-lane pick the compiler cannot turn
 * back into a runtime-indexed read of v[] (which it spills to scratch) */
static __device__ __forceinline__ u32x4 pick_if(u32x4 a, u32x4 b, uint64_t lanes)
{
	u32x4 r;
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.x) : "v"(a.x), "v"(b.x), "s"(lanes));
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.y) : "v"(a.y), "v"(b.y), "s"(lanes));
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.z) : "v"(a.z), "v"(b.z), "s"(lanes));
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.w) : "v"(a.w), "v"(b.w), "s"(lanes));
	return r;
}

/* After all K chunks were summed: lane 0 takes the head bytes of its first
 * chunk back out (branch-free, n = 0 elsewhere); the tail comes out of the
 * lane holding the last chunk, in one constant-index block per k -- or, with
 * U > 1 (where the compiler merges those blocks into a runtime-indexed,
 * scratch-spilled read of v[]), from a chunk every lane picks. */
template <int G, int K, int U>
static __device__ __forceinline__ void edge_drop(const Frame &f, const u32x4 (&v)[K],
						 uint32_t lane, uint32_t &E, uint32_t &O)
{
	const uint32_t last = f.nchunks - 1;
	drop_prefix(v[0], lane == 0 && f.nchunks ? f.head : 0u, E, O);
	if (U > 1) {
		u32x4 vl = v[0];
#pragma unroll
		for (int k = 1; k < K; k++)
			vl = pick_if(vl, v[k], __builtin_amdgcn_ballot_w64((last / G) == (uint32_t)k));
		drop_suffix(vl, f.nchunks && lane == (last & (G - 1)) ? f.tail : 0u, E, O);
	} else if (f.tail && f.nchunks && lane == (last & (G - 1))) {
#pragma unroll
		for (int k = 0; k < K; k++)
			if ((last / G) == (uint32_t)k)
				drop_suffix(v[k], f.tail, E, O);
	}
}

static __device__ __forceinline__ void edge_drop_one(const Frame &f, uint32_t c, u32x4 v,
						     uint32_t &E, uint32_t &O)
{
	if (c == 0)
		drop_prefix(v, f.head, E, O);
	if (c + 1 == f.nchunks)
		drop_suffix(v, f.tail, E, O);
}

/* all K chunks of a frame into E/O, edges handled per grid */
template <int G, int K, int U, bool DW>
static __device__ __forceinline__ void sum_frame(const Frame &f, const u32x4 (&vc)[K],
						 uint32_t lane, uint32_t &E, uint32_t &O)
{
	if (DW) {
		u32x4 v[K];
#pragma unroll
		for (int k = 0; k < K; k++)
			v[k] = vc[k];
		edge_mask<G, K>(f, v, lane);
#pragma unroll
		for (int k = 0; k < K; k++)
			accum(v[k], E, O);
	} else {
#pragma unroll
		for (int k = 0; k < K; k++)
			accum(vc[k], E, O);
		edge_drop<G, K, U>(f, vc, lane, E, O);
	}
}

/* walking (jumbo) path: every chunk of f strided over G lanes */
template <int G, bool DW>
static __device__ __forceinline__ void sum_walk(const Frame &f, uint32_t lane, uint32_t &E,
						uint32_t &O)
{
	for (uint32_t c = lane; c < f.nchunks; c += G) {
		u32x4 v = load_chunk(XB_LOAD(f.base + 16u * c, 16, f.eth, f.lim, XB_CSUM_WALK, c,
					     g_zero_chunk));
		if (DW) {
			accum(edge_mask_one(f, c, v), E, O);
		} else {
			accum(v, E, O);
			edge_drop_one(f, c, v, E, O);
		}
	}
}

/* the chunk grid a geometry uses (measured, see the Frame comment) */
template <int G, int K>
struct Grid {
	static constexpr bool DW = !(G == 16 && K >= 6) && !(G == 8 && K >= 12);
};

/* Frame bytes and result arrays are global memory (device memory or a
 * registered host UMEM): accessed through address_space(1) pointers, so a
 * pointer that came from memory (the resident kernel's request words) or
 * from integer arithmetic still gets global, not flat, instructions -- a
 * flat access is counted on lgkmcnt too and the waits around it drain the
 * whole vmcnt queue (csum_kernel<16,2,6,2>, profiles/r04/inplace/
 * r04n_ab_flat_b64.txt). */
template <typename T>
static __device__ __forceinline__ T ld_g(const void *p)
{
	return *(const __attribute__((address_space(1))) T *)p;
}

/* Result and in-place stores are plain (temporal): nontemporal 2-byte stores
 * each became a partial write, config 2 +12 % (profiles/r02) */
template <typename T>
static __device__ __forceinline__ void st_res(T *p, T v)
{
	*(__attribute__((address_space(1))) T *)p = v;
}

/* a 2-byte check field of the frame (in-place writes) */
static __device__ __forceinline__ void store_u16(uint8_t *p, uint16_t v)
{
	if (((uintptr_t)p & 1) == 0) {
		st_res(reinterpret_cast<uint16_t *>(p), v);
	} else {
		st_res(p, (uint8_t)v);
		st_res(p + 1, (uint8_t)(v >> 8));
	}
}

/* TL > 0 (in-place A/B, xcsum_csum_tl.hip): a frame's first TL chunks -- the
 * ones holding udp->check -- are loaded temporally (allocated in the caches),
 * the rest nontemporally, so the in-place store that follows may find its
 * line still cached */
template <int G, int U, int K, int TL = 0>
static __device__ __forceinline__ void issue(const Frame (&f)[U], uint32_t lane,
					     u32x4 (&v)[U][K])
{
	const uint8_t *zero = (const uint8_t *)g_zero_chunk;
#pragma unroll
	for (int u = 0; u < U; u++)
#pragma unroll
		for (int k = 0; k < K; k++) {
			uint32_t c = lane + k * G;
			const uint8_t *q = c < f[u].nchunks ? XB_LOAD(f[u].base + 16u * c, 16, f[u].eth,
								      f[u].lim, XB_CSUM_CHUNK, c, zero)
							    : zero;
			if (TL > 0 && k == 0 && c < (uint32_t)TL)
				v[u][k] = *((gu32x4 *)q);
			else
				v[u][k] = load_chunk(q);
		}
}

} /* namespace xcsum */

#endif
