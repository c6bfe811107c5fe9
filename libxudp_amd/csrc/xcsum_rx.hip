/*
 * xcsum_rx.hip -- the receive path's per-frame work on the GPU: what
 * xudp_nic_recv_channel (cclinuxer/libxudp group/channel.c:211-267) does for
 * each descriptor it dequeues from the RX ring.
 *
 *   packet_parse()       include/packet_parse.h:101-165 (parse_ipv6 :33-99)
 *   stats-request test   channel.c:182-190 (iph->saddr == iph->daddr)
 *   xudp_fill_msg()      channel.c:69-128 (body, size, peer/local address)
 *   + UDP verify         RFC 768/2460 over the UDP header's own length
 *                        (the reference verifies nothing)
 *
 * Design (HBM-bound: frame bytes once, 16-B descriptor in, 64-B record out).
 * The header decides where the checksum span ends (the UDP length, not the
 * frame length: received frames may carry Ethernet padding), so loading the
 * span after parsing would put a dependent HBM round trip on every frame.
 * Instead the kernel loads the WHOLE frame speculatively from the descriptor
 * alone -- the 16-byte aligned blocks from the one holding the EtherType at
 * eth+12 to the one holding the frame's last byte -- with the
 * checksum kernel's two-stage software pipeline (frame i+1's chunks and frame
 * i+2's descriptor in flight while frame i is processed).  When frame i's
 * chunks land:
 *   1. its first 6 chunks (96 bytes: every header byte packet_parse reads
 *      unless IPv6 extension headers follow) are written to a per-frame LDS
 *      stage; the parse reads every field it may need (frame bytes
 *      12..61) in one batch of 14 dword reads and cuts the fields out with
 *      v_alignbyte, so no stage read waits on another;
 *   2. the span [pseudo-header addresses, udp + ulen) is summed from the
 *      chunk registers with v_dot4_u32_u8 (exact even/odd byte sums, as in
 *      xcsum_kernels.hip), every chunk masked to the span with byte masks
 *      from a 17-entry LDS table (no per-chunk branch);
 *   3. G-lane DPP reduction, RFC verify, the record (lanes 0..3 store one
 *      16-byte piece each).
 * Frames the stage cannot describe (IPv6 extension headers; IPv4 options
 * under VERIFY, whose pseudo header is not contiguous with the UDP header)
 * take a wave-uniform slow path that parses from global memory byte by byte
 * exactly as before; jumbo frames (more than K*G chunks) re-walk their
 * chunks from global memory.  Results never depend on the path.
 *
 * rx_wide_kernel (geometries with U = 0, the default for jumbo frames) does
 * the header work one frame per lane, 64 frames per wave, and then sums the
 * spans G lanes per frame (see its comment).
 *
 * d_umem must be 4-byte aligned (the ABI's rule).  The first chunk may start
 * up to 15 bytes before eth+12 and the last end up to 15 bytes after the
 * frame: neither leaves the 16-byte block of a frame byte, so neither can
 * touch an unmapped page.
 */
#include "xcsum_internal.h"
#include "xcsum_device.h"
#include <stdio.h>
#include <stdlib.h>

namespace xcsum {

/* Record stores are nontemporal: written once, never re-read by the kernel.
 * Plain stores left 64 MB of dirty lines per 1M frames in L2 among the
 * streaming frame reads: MTU VERIFY 0.287 -> 0.259 ms (1.21x -> 1.09x the
 * checksum kernel), IPv6 1.17x -> 1.08x, config 5 1.03x -> 1.02x, same
 * call (profiles/r02/session2/rx_ntrec). */
static __device__ __forceinline__ void store_rec(u32x4 *dst, u32x4 v)
{
	__builtin_nontemporal_store(v, dst);
}

static __device__ __forceinline__ uint32_t be16(const uint8_t *p)
{
	return ((uint32_t)p[0] << 8) | p[1];
}

static __device__ __forceinline__ uint32_t fold16(uint32_t s)
{
	s = (s & 0xffffu) + (s >> 16);
	return (s & 0xffffu) + (s >> 16);
}

/* sum of the big-endian 16-bit words of [p, p + nbytes), nbytes even */
static __device__ __forceinline__ uint32_t be_words(const uint8_t *p, uint32_t nbytes)
{
	uint32_t s = 0;
	for (uint32_t i = 0; i < nbytes; i += 2)
		s += be16(p + i);
	return s;
}

/* big-endian 16-bit word sum of the 4 bytes of a little-endian dword */
static __device__ __forceinline__ uint32_t be_words4(uint32_t w)
{
	return (dot_even(w, 0u) << 8) + dot_odd(w, 0u);
}

/* ---- slow path: packet_parse() from global memory ------------------------ */

struct Parsed {
	uint32_t ok, family, l3, l4;
};

/* packet_parse() of include/packet_parse.h:101-165, offsets instead of
 * pointers, quirks kept (see xcsum.h) */
static __device__ Parsed packet_parse(const uint8_t *pkt, uint32_t len)
{
	Parsed r = {0u, 0u, 14u, 0u};
	if (len < 14)
		return r;
	const uint8_t p0 = pkt[12], p1 = pkt[13];
	if (p0 == 0x08 || p1 == 0x00) {
		if (len < 14 + 20 || pkt[14 + 9] != 17)
			return r;
		const uint32_t ihl = pkt[14] & 0xfu;
		const uint32_t udp = 14 + (ihl == 5 ? 20 : (ihl << 2));
		if (udp + 8 > len)
			return r;
		r.ok = 1;
		r.family = 4;
		r.l4 = udp;
		return r;
	}
	if (p0 == 0x86 && p1 == 0xDD) {
		if (len < 14 + 40)
			return r;
		uint32_t pos = 14 + 40;
		uint32_t nexthdr = pkt[14 + 6];
		for (int i = 0; i < 8; i++) {      /* MAX_IPV6_OPT, packet_parse.h:5 */
			if (pos + 2 > len)
				return r;
			uint32_t ol;
			switch (nexthdr) {
			case 17:
				if (14 + 40 + 8 > len)
					return r;
				r.ok = 1;
				r.family = 6;
				r.l4 = 14 + 40;    /* iph6 + 1, whatever was skipped (:62) */
				return r;
			case 51:                   /* AUTH: (hdrlen + 2) << 2 */
				ol = ((uint32_t)pkt[pos + 1] + 2) << 2;
				break;
			case 44:                   /* FRAGMENT */
				ol = 8;
				break;
			case 0: case 43: case 47: case 50: case 60: case 135:
				ol = ((uint32_t)pkt[pos + 1] + 1) << 3;
				break;
			default:                   /* SCTP, ICMP, NONE, TCP, IPV6, unknown */
				return r;
			}
			nexthdr = pkt[pos];
			pos += ol;
		}
	}
	return r;
}

/* chunk c of the dword grid over [lo, hi): masked, for summing */
static __device__ __forceinline__ u32x4 grid_chunk(const uint8_t *base, uint32_t n,
						   uint32_t head, uint32_t tail, uint32_t c,
						   const uint8_t *ok_lo, const uint8_t *ok_hi)
{
	u32x4 v = {0u, 0u, 0u, 0u};
	(void)ok_lo;
	(void)ok_hi;
	if (c < n && XB_IN(base + 16u * c, 16, ok_lo, ok_hi, XB_RX_CHUNK, c)) {
		v = __builtin_nontemporal_load((gu32x4 *)(base + 16u * c));
		if (c == 0) {
			const uint64_t k0 = head >= 8 ? 0ull : ~0ull << (8 * (head & 7));
			const uint64_t k1 = head <= 8 ? ~0ull : ~0ull << (8 * (head & 7));
			v.x &= (uint32_t)k0;
			v.y &= (uint32_t)(k0 >> 32);
			v.z &= (uint32_t)k1;
			v.w &= (uint32_t)(k1 >> 32);
		}
		if (c + 1 == n)
			v.w &= 0xffffffffu >> (8 * tail);
	}
	return v;
}

/* One frame's record fields, whichever path produced them. */
struct Rec {
	uint32_t status, family, l4, ulen, ports;
};

/* The whole per-frame work from global memory (the general case: IPv6
 * extension headers, IPv4 options).  Every lane of the wave runs it (the
 * reductions need them all); only frames flagged slow use the result. */
template <int G>
static __device__ Rec rx_slow(const uint8_t *pkt, uint32_t len, uint32_t lane, bool present,
			      bool verify, bool iphdr)
{
	const Parsed ps = present ? packet_parse(pkt, len) : Parsed{0u, 0u, 14u, 0u};
	Rec r = {XCSUM_RX_PARSE, ps.family, ps.ok ? ps.l4 : 0u, 0u, 0u};
	if (ps.ok) {
		const uint8_t *udp = pkt + ps.l4;
		r.ulen = be16(udp + 4);
		r.ports = (uint32_t)udp[0] | ((uint32_t)udp[1] << 8) | ((uint32_t)udp[2] << 16) |
			  ((uint32_t)udp[3] << 24);
		/* xudp_stats_req_check(): iphdr saddr/daddr fields, both
		 * families (the union, channel.c:241) */
		const uint8_t *ip = pkt + ps.l3;
		const bool stats = ip[12] == ip[16] && ip[13] == ip[17] && ip[14] == ip[18] &&
				   ip[15] == ip[19];
		r.status = stats ? XCSUM_RX_STATS : XCSUM_RX_OK;
	}
	if (verify && r.status == XCSUM_RX_OK) {
		const uint8_t *ip = pkt + ps.l3;
		const uint32_t ihl = ip[0] & 0xfu;
		const uint32_t ulen = r.ulen;
		bool good = ulen >= 8 && ps.l4 + ulen <= len && !(ps.family == 4 && ihl < 5);
		if (good) {
			const uintptr_t lo = (uintptr_t)(pkt + ps.l4);
			const uintptr_t hi = lo + ulen;
			const uintptr_t e4 = (hi + 3) & ~(uintptr_t)3;
			const uint32_t n = (uint32_t)(e4 - lo + 15) >> 4;
			const uint8_t *base = (const uint8_t *)(e4 - 16u * n);
			const uint32_t head = (uint32_t)(lo - (uintptr_t)base);
			const uint32_t tail = (uint32_t)(e4 - hi);
			uint32_t E = 0, O = 0;
			for (uint32_t c = lane; c < n; c += G)   /* one chunk per lane in flight:
								    rare path, few registers */
				accum(grid_chunk(base, n, head, tail, c, pkt,
						 (const uint8_t *)(((uintptr_t)pkt + len + 15u) &
								   ~(uintptr_t)15)),
				      E, O);
			uint32_t s = (lo & 1u) ? (O << 8) + E : (E << 8) + O;
			s = seg_sum<G>(s);
			/* pseudo header (RFC 768 / RFC 2460 8.1) */
			if (ps.family == 4)
				s += be_words(ip + 12, 8);
			else
				s += be_words(ip + 8, 32);
			s += 17u + (ulen >> 16) + (ulen & 0xffffu);
			const bool nocheck = (pkt[ps.l4 + 6] | pkt[ps.l4 + 7]) == 0;
			good = nocheck ? ps.family == 4 : fold16(s) == 0xffffu;
		}
		if (good && iphdr && ps.family == 4) {
			/* RFC 1071 over the 4*ihl-byte header, check included */
			uint32_t h = 0;
			for (uint32_t j = 2 * lane; j < 4 * ihl; j += 2 * G)
				h += be16(ip + j);
			h = seg_sum<G>(h);
			good = fold16(h) == 0xffffu;
		}
		if (!good)
			r.status = XCSUM_RX_CSUM;
	}
	return r;
}

/* ---- fast path ----------------------------------------------------------- */

constexpr uint32_t STAGE_CHUNKS = 6;   /* 96 bytes from the chunk holding eth+12 */

/* A frame's chunk grid: the 16-byte aligned blocks from the one holding
 * eth + 12 to the one holding the last byte.  Chunk c covers frame bytes
 * [g0 + 16c, g0 + 16c + 16) with g0 = 12 - h, h = offset of eth + 12 in chunk 0
 * (0..15), so frame byte x sits at stage byte x - 12 + h.  Everything but the
 * frame pointer is a 32-bit frame-relative offset (registers: two frames are
 * live in the pipeline). */
struct RFrame {
	const uint8_t *eth;
	uint32_t meta;          /* frame length (clamped to 2^31 - 1) | present << 31 */
};

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef __attribute__((address_space(1))) const u32x3 gu32x3;

/* xdp_desc {addr, len}: the unused options word is not loaded */
static __device__ __forceinline__ u32x3 rx_desc(const RxArgs &a, uint32_t q)
{
	return *((gu32x3 *)(a.desc + (q < a.n ? q : a.n - 1)));
}

/* Visiting order of a receive batch (as resolve_order in xcsum_csum.h): the
 * prepared region order only when the batch is sparse in the UMEM -- the
 * first and last descriptors span more than twice the bytes of n frames of
 * their mean length, as the frames of an AF_XDP RX ring are, one per 2-4 KB
 * chunk -- else descriptor order.  Wave-uniform scalar loads. */
typedef __attribute__((address_space(4))) const u32x3 cu32x3;

static __device__ __forceinline__ void rx_resolve_order(RxArgs &a)
{
	if (!a.ord.sparse_only)
		return;
	bool sparse = false;
	if (a.n >= 2) {
		const u32x3 d0 = *((cu32x3 *)(a.desc));
		const u32x3 dl = *((cu32x3 *)(a.desc + (a.n - 1)));
		const uint64_t a0 = ((uint64_t)d0.y << 32) | d0.x;
		const uint64_t al = ((uint64_t)dl.y << 32) | dl.x;
		const uint64_t mean = ((uint64_t)d0.z + dl.z) / 2 + 1;
		sparse = al > a0 && al + dl.z - a0 > 2ull * a.n * mean;
	}
	if (!sparse)
		a.ord = a.dense;
}

static __device__ __forceinline__ RFrame rx_resolve(const RxArgs &a, u32x3 d, bool present)
{
	RFrame f;
	f.eth = a.umem + (((uint64_t)d.y << 32) | d.x);
	f.meta = (d.z > 0x7fffffffu ? 0x7fffffffu : d.z) | (present ? 0x80000000u : 0u);
	return f;
}

static __device__ __forceinline__ bool rx_present(const RFrame &f)
{
	return (f.meta >> 31) != 0;
}

static __device__ __forceinline__ uint32_t rx_len(const RFrame &f)
{
	return f.meta & 0x7fffffffu;
}

/* chunk count and h (registers are scarce: recomputed where needed): the
 * 16-byte blocks from the one holding eth + 12 to the one holding the
 * frame's last byte.  Aligned chunks: the dword grid laid back from the
 * frame end that this replaced made every load straddle two 16-byte blocks
 * when the end was not 16-byte aligned, and cost 3-8 % at MTU
 * (profiles/r02/rx/ab_grid16/). */
static __device__ __forceinline__ uint32_t rx_nchunks(const RFrame &f)
{
	const uint32_t len = rx_len(f);
	const uint32_t e = (uint32_t)(uintptr_t)f.eth;
	const uint32_t span = ((e + len + 15u) & ~15u) - ((e + 12u) & ~15u);
	return (rx_present(f) && len >= 14) ? span >> 4 : 0u;
}

static __device__ __forceinline__ uint32_t rx_h(const RFrame &f, uint32_t nchunks)
{
	return nchunks ? ((uint32_t)(uintptr_t)f.eth + 12u) & 15u : 0u;
}

/* frame-relative offset of chunk c's first byte */
static __device__ __forceinline__ int rx_chunk_off(uint32_t h, uint32_t c)
{
	return 12 - (int)h + 16 * (int)c;
}

/* what a frame's chunk loads may touch (bounds checks of the debug build):
 * the 16-byte blocks from the one holding eth + 12 to the one holding the
 * last byte */
__attribute__((unused)) static __device__ __forceinline__ const uint8_t *rx_ok_lo(const RFrame &f)
{
	return (const uint8_t *)(((uintptr_t)f.eth + 12u) & ~(uintptr_t)15);
}
__attribute__((unused)) static __device__ __forceinline__ const uint8_t *rx_ok_hi(const RFrame &f)
{
	return (const uint8_t *)(((uintptr_t)f.eth + rx_len(f) + 15u) & ~(uintptr_t)15);
}

__device__ u32x4 g_rx_zero[4];

template <int G, int K>
static __device__ __forceinline__ void rx_issue(const RxArgs &a, const RFrame &f, uint32_t lane,
						u32x4 (&v)[K])
{
	const uint8_t *zero = (const uint8_t *)g_rx_zero;
	const uint32_t nc = rx_nchunks(f);
	const uint32_t h = rx_h(f, nc);
	/* all chunks under VERIFY, else only the header stage */
	const uint32_t nl = (a.flags & XCSUM_F_VERIFY) || nc < STAGE_CHUNKS ? nc : STAGE_CHUNKS;
#pragma unroll
	for (int k = 0; k < K; k++) {
		const uint32_t c = lane + k * G;
		v[k] = __builtin_nontemporal_load(
			(gu32x4 *)(c < nl ? XB_LOAD(f.eth + rx_chunk_off(h, c), 16, rx_ok_lo(f),
						    rx_ok_hi(f), XB_RX_CHUNK, c, zero)
					  : zero));
	}
}

/* Byte masks of a chunk, from a 17-entry LDS table: SPAN[n] keeps bytes
 * [0, n) of 16.  keep_span(v, a, b) keeps bytes [a, b) (both clamped to
 * [0, 16]): two ds_read_b128 and one and-not per dword, where building the
 * masks with 64-bit shifts took ~55 VALU per edge chunk (the ISA). */
constexpr uint32_t SPAN_DWORDS = 17 * 4;

static __device__ __forceinline__ void span_init(uint32_t *tab)
{
	/* called by every thread, then a block barrier */
	for (uint32_t t = threadIdx.x; t < SPAN_DWORDS; t += blockDim.x) {
		const int n = (int)(t >> 2) - 4 * (int)(t & 3u);   /* bytes kept of dword t & 3 */
		tab[t] = n >= 4 ? 0xffffffffu : (n <= 0 ? 0u : 0xffffffffu >> (32 - 8 * n));
	}
}

static __device__ __forceinline__ u32x4 span_mask(const uint32_t *tab, int n)
{
	n = n < 0 ? 0 : (n > 16 ? 16 : n);
	return *(const u32x4 *)(tab + 4 * n);
}

static __device__ __forceinline__ u32x4 keep_span(const uint32_t *tab, u32x4 v, int a, int b)
{
	return v & span_mask(tab, b) & ~span_mask(tab, a);
}

/* Everything for frame p once its chunks v[] have landed: stage, parse,
 * verify, record.  Group-uniform; every lane of the wave must call it. */
template <int G, int K>
static __device__ __forceinline__ void rx_frame(const RxArgs &a, uint32_t *st, const uint32_t *tab,
						const RFrame &fc,
						const u32x4 (&vc)[K], uint32_t p, uint32_t lane,
						bool verify, bool iphdr, uint32_t &delivered)
{
	const uint32_t len = rx_len(fc);
	const uint32_t nchunks = rx_nchunks(fc);
	const uint32_t fh = rx_h(fc, nchunks);          /* frame byte 12 = header byte fh */

	/* 1. the header: hdr[i] = frame bytes [12 + 4i, 16 + 4i), i < 13 (every
	 * field the fast path can use lies in bytes 12..61).  Chunks 0..5 of
	 * the grid hold it, spread over the group's lanes. */
	uint32_t hdr[13];
	/* Through the group's LDS stage: the lanes holding chunks 0..5 write
	 * them, every lane reads the 14 dwords from frame byte 12 back in one
	 * batch (same addresses across the group: broadcast reads) and realigns
	 * them with v_alignbyte.  Measured against broadcasting the chunks with
	 * DPP / v_readlane and selecting dwords with v_cndmask: 1-2% faster at
	 * MTU and 64 B, 5% on config 5 (profiles/r01/rx_mtu/hdr_*). */
#pragma unroll
	for (int k = 0; k < K; k++) {
		const uint32_t c = lane + k * G;
		if (k * G < (int)STAGE_CHUNKS && c < STAGE_CHUNKS)
			*((u32x4 *)(st + 4 * c)) = vc[k];
	}
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	{
		const uint32_t *dw = st + (fh >> 2);
		uint32_t d[14];
#pragma unroll
		for (int i = 0; i < 14; i++)
			d[i] = dw[i];
#pragma unroll
		for (int i = 0; i < 13; i++)
			hdr[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], fh & 3u);
	}
	auto f0 = [&](int x) { return hdr[(x - 12) >> 2]; };          /* x = 0 mod 4 */
	auto f2 = [&](int x) {                                         /* x = 2 mod 4 */
		const int i = (x - 12) >> 2;
		return __builtin_amdgcn_alignbyte(hdr[i + 1], hdr[i], 2u);
	};

	/* 2. packet_parse() */
	const uint32_t w12 = f0(12);                    /* h_proto, ver/ihl, tos */
	const uint32_t w20 = f0(20);                    /* v4: proto at 23; v6: nexthdr at 20 */
	const uint32_t w26 = f2(26), w30 = f2(30);      /* iph saddr / daddr fields */

	/* packet_parse(), branch-free for the common cases */
	const uint32_t p0 = w12 & 0xffu, p1 = (w12 >> 8) & 0xffu;
	const uint32_t ihl = (w12 >> 16) & 0xfu;
	const bool present = rx_present(fc);
	const bool eth_ok = present && len >= 14;
	const bool is4 = eth_ok && (p0 == 0x08 || p1 == 0x00);
	const uint32_t l4v4 = 14u + (ihl == 5 ? 20u : (ihl << 2));
	const bool ok4 = is4 && len >= 34 && (w20 >> 24) == 17 && l4v4 + 8 <= len;
	const bool is6 = eth_ok && !is4 && p0 == 0x86 && p1 == 0xDD && len >= 54;
	const bool ok6 = is6 && (w20 & 0xffu) == 17 && len >= 62;  /* pos+2, 14+40+8 <= len */
	/* IPv4 options (UDP header outside the batch) and IPv6 extension
	 * headers (walk them) go the general way */
	const bool slow = (ok4 && ihl != 5) || (is6 && (w20 & 0xffu) != 17);
	const bool ok = (ok4 && ihl == 5) || ok6;
	const uint32_t family = ok ? (ok4 ? 4u : 6u) : 0u;
	const uint32_t l4 = ok ? (ok4 ? 34u : 54u) : 0u;
	/* selects only: every branch here would cost an exec-mask round trip */
	const uint32_t wck = ok ? (ok4 ? f2(38) : f2(58)) : 0u;   /* len, check */
	Rec r;
	r.family = family;
	r.l4 = l4;
	r.ports = ok ? (ok4 ? f2(34) : f2(54)) : 0u;
	r.ulen = ((wck & 0xffu) << 8) | ((wck >> 8) & 0xffu);
	r.status = !ok ? XCSUM_RX_PARSE : (w26 == w30 ? XCSUM_RX_STATS : XCSUM_RX_OK);
	/* record addresses: IPv4 iph + 12 / + 16, IPv6 iph6 + 8 / + 24 */
	u32x4 saddr = ok4 ? u32x4{w26, 0u, 0u, 0u} : u32x4{f2(22), w26, w30, f2(34)};
	u32x4 daddr = ok4 ? u32x4{w30, 0u, 0u, 0u} : u32x4{f2(38), f2(42), f2(46), f2(50)};
	/* IPv4 header words (iphdr verify): bytes 14..33 */
	const uint32_t hsum = be_words4(f2(14)) + be_words4(f2(18)) + be_words4(f2(22)) +
			      be_words4(w26) + be_words4(w30);

	/* 3. verify: sum [addresses, udp + ulen) from the chunk registers */
	const bool want = verify && r.status == XCSUM_RX_OK && !slow;
	bool good = want && r.ulen >= 8 && l4 + r.ulen <= len && !(family == 4 && ihl < 5);
	const int lo = family == 4 ? 26 : 22;            /* frame-relative span */
	const int hi = (int)(l4 + r.ulen);
	if (__builtin_amdgcn_ballot_w64(want)) {
		uint32_t E = 0, O = 0;
		if (__builtin_amdgcn_ballot_w64(good && nchunks > K * G)) {
			for (uint32_t c = lane; c < nchunks; c += G) {
				const int cb = rx_chunk_off(fh, c);
				u32x4 v = __builtin_nontemporal_load((gu32x4 *)XB_LOAD(
					fc.eth + cb, 16, rx_ok_lo(fc), rx_ok_hi(fc), XB_RX_CHUNK, c, g_rx_zero));
				if (cb < lo || cb + 16 > hi)
					v = keep_span(tab, v, lo - cb, hi - cb);
				accum(v, E, O);
			}
		} else {
#pragma unroll
			for (int k = 0; k < K; k++) {
				const int cb = rx_chunk_off(fh, lane + k * G);
				/* every chunk masked, no per-chunk branch (a ballot and a
				 * branch per chunk measured 5-10% slower): the span's start
				 * lies in chunks 0..1 (k == 0), its end anywhere; lanes
				 * that are not `good` sum bytes nobody reads */
				const u32x4 v = k == 0 ? keep_span(tab, vc[k], lo - cb, hi - cb)
						       : vc[k] & span_mask(tab, hi - cb);
				accum(v, E, O);
			}
		}
		uint32_t s = ((uintptr_t)fc.eth & 1u) ? (O << 8) + E : (E << 8) + O;
		s = seg_sum<G>(s);
		if (good) {
			s += 17u + r.ulen;
			good = (wck >> 16) == 0 ? family == 4 : fold16(s) == 0xffffu;
		}
		/* RFC 1071 over the 20-byte IPv4 header (ihl == 5 here) */
		if (iphdr && family == 4)
			good = good && fold16(hsum) == 0xffffu;
		if (want && !good)
			r.status = XCSUM_RX_CSUM;
	}

	/* 4. general case */
	if (__builtin_amdgcn_ballot_w64(slow)) {
		const Rec rs = rx_slow<G>(fc.eth, len, lane, slow, verify, iphdr);
		if (slow) {
			r = rs;
			/* addresses from global memory, iph + 12 / iph6 + 8 */
			u32x4 ad[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
			if (r.status != XCSUM_RX_PARSE) {
				const uint32_t nb = r.family == 4 ? 4 : 16;
				for (uint32_t t = 0; t < 2; t++)
					for (uint32_t q = 0; q < nb; q++)
						ad[t][q >> 2] |= (uint32_t)fc.eth[(r.family == 4 ? 26u : 22u) +
										 t * nb + q]
								 << (8 * (q & 3));
			}
			saddr = ad[0];
			daddr = ad[1];
		}
	}

	/* 5. the record: four 16-byte pieces, piece j stored by lane j % G;
	 * every piece is built with selects (no per-lane branches) */
	const bool pok = r.status != XCSUM_RX_PARSE;
	const uint64_t addr = (uint64_t)(fc.eth - a.umem);
	const uint64_t body = pok ? addr + r.l4 + 8 : 0;
	const u32x4 w0 = {(uint32_t)addr, (uint32_t)(addr >> 32), (uint32_t)body,
			  (uint32_t)(body >> 32)};
	const u32x4 w1 = {pok ? r.ulen - 8u : 0u,
			  r.status | (r.family << 8) | ((pok ? r.l4 : 0u) << 16), r.ports, 0u};
	const u32x4 zero4 = {0u, 0u, 0u, 0u};
	if (!pok) {
		saddr = zero4;
		daddr = zero4;
	}
#pragma unroll
	for (int i = 0; i < (G < 4 ? 4 / G : 1); i++) {
		const uint32_t j = lane + i * G;       /* piece */
		const u32x4 w = j == 0 ? w0 : (j == 1 ? w1 : (j == 2 ? saddr : daddr));
		if (present && j < 4 && XB_IDX(p, a.n, XB_RX_REC))
			store_rec((u32x4 *)(a.msgs + p) + j, w);
	}
	if (lane == 0 && present && r.status == XCSUM_RX_OK)
		delivered++;

	/* the stage is rewritten by the next frame: reads first */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/*
 * Persistent grid, G lanes per frame.  Two-stage software pipeline written
 * as a ping-pong over two register sets (A, B): while frame p's chunks are
 * processed, frame p + nseg's chunks and the descriptor after it are in
 * flight.  No copy from the "next" set into the "current" one: such a copy
 * needs the in-flight loads to have landed and would drain the pipeline
 * every iteration (vmcnt(0) at the loop latch, seen in the ISA).
 */
/* per-frame header stage of the group kernel: STAGE_CHUNKS chunks + one
 * dword of slack per G-lane group */
template <int G>
struct GroupStage {
	static constexpr uint32_t SW = STAGE_CHUNKS * 4 + 4;   /* dwords per group */
	static constexpr uint32_t DWORDS = (256 / G) * SW;
};

/* stage: GroupStage<G>::DWORDS of LDS, 16-byte aligned; span: the mask
 * table, initialised (span_init + block barrier) by the caller */
template <int G, int K, int U>
static __device__ __forceinline__ void rx_group_body(RxArgs a, uint32_t *stage,
						     const uint32_t *span)
{
	constexpr uint32_t SW = GroupStage<G>::SW;
	const uint32_t lane = threadIdx.x & (G - 1);
	const uint32_t grp = threadIdx.x / G;
	uint32_t *st = stage + grp * SW;
	uint32_t seg = (blockIdx.x * 256u + threadIdx.x) / G;
	const uint32_t nseg = gridDim.x * (256u / G);
	if (G == 64)
		seg = __builtin_amdgcn_readfirstlane(seg);
	const bool verify = (a.flags & XCSUM_F_VERIFY) != 0;
	const bool iphdr = (a.flags & XCSUM_F_IPHDR) != 0;
	uint32_t delivered = 0;
	if (lane == 0)
		st[SW - 1] = 0u;
	rx_resolve_order(a);
	/* q is a logical index: frame frame_of(q), present below a.n */
	const uint32_t limit = a.ord.nlog;
	auto phys = [&](uint32_t q) { return frame_of(a.ord, q); };
	auto has = [&](uint32_t q) { return q < limit && phys(q) < a.n; };
	auto desc = [&](uint32_t q) { return rx_desc(a, phys(q)); };

	/* set A holds frames p + u*nseg, set B frames p + (U + u)*nseg */
	u32x3 d[U];
	RFrame fa[U], fb[U];
	u32x4 va[U][K], vb[U][K];
#pragma unroll
	for (int u = 0; u < U; u++)
		d[u] = desc(seg + u * nseg);
#pragma unroll
	for (int u = 0; u < U; u++) {
		fa[u] = rx_resolve(a, d[u], has(seg + u * nseg));
		d[u] = desc(seg + (U + u) * nseg);
	}
	__builtin_amdgcn_sched_barrier(0);
#pragma unroll
	for (int u = 0; u < U; u++)
		rx_issue<G, K>(a, fa[u], lane, va[u]);

	for (uint32_t p = seg; p < limit; p += 2 * U * nseg) {
#pragma unroll
		for (int u = 0; u < U; u++) {
			fb[u] = rx_resolve(a, d[u], has(p + (U + u) * nseg));
			d[u] = desc(p + (2 * U + u) * nseg);
		}
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int u = 0; u < U; u++)
			rx_issue<G, K>(a, fb[u], lane, vb[u]);
		/* keep the other set's work below its loads: hoisted above them,
		 * its first use waits for everything in flight (vmcnt(2) in the
		 * ISA) and the loads go out only after it -- one set in flight */
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int u = 0; u < U; u++)
			rx_frame<G, K>(a, st, span, fa[u], va[u], phys(p + u * nseg), lane, verify, iphdr,
				       delivered);

#pragma unroll
		for (int u = 0; u < U; u++) {
			fa[u] = rx_resolve(a, d[u], has(p + (2 * U + u) * nseg));
			d[u] = desc(p + (3 * U + u) * nseg);
		}
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int u = 0; u < U; u++)
			rx_issue<G, K>(a, fa[u], lane, va[u]);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int u = 0; u < U; u++)
			rx_frame<G, K>(a, st, span, fb[u], vb[u], phys(p + (U + u) * nseg), lane, verify,
				       iphdr, delivered);
	}
	/* The delivered count: one plain store per block, summed by a second
	 * one-block kernel.  Device-scope atomics to one address serialise
	 * (~8 ns each): even one per wave cost ~20 us on a config-3 batch. */
	if (a.count) {
		__shared__ uint32_t wsum[4];
		const uint32_t tot = seg_sum<64>(delivered);   /* all lanes live again */
		if ((threadIdx.x & 63) == 0)
			wsum[threadIdx.x >> 6] = tot;
		__syncthreads();
		if (threadIdx.x == 0 && XB_IDX(blockIdx.x, RX_PART_MAX, XB_RX_PART))
			a.part[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
	}
}

template <int G, int K, int U>
__global__ void __launch_bounds__(256) rx_kernel(RxArgs a)
{
	__shared__ __attribute__((aligned(16))) uint32_t stage[GroupStage<G>::DWORDS];
	__shared__ __attribute__((aligned(16))) uint32_t span[SPAN_DWORDS];
	span_init(span);
	__syncthreads();
	rx_group_body<G, K, U>(a, stage, span);
}

/* ---- lane-per-frame parse (geometry U = 0) ---------------------------------
 * rx_kernel pays the header work (parse, masks, record) once per G-lane group,
 * i.e. once per 64/G frames per wave instruction.  Here a wave takes 64
 * frames at a time and lane l parses frame l from its own 6 header chunks, so
 * the header work is paid once per 64 frames.  The wave then sums the 64
 * spans 64/G frames per step, G lanes each, with the ping-pong pipeline; each
 * group fetches its frame's parameters from the owning lane (ds_bpermute),
 * the owning lane collects its frame's sum and finishes the verify; the
 * 64 records go out through LDS, 1 KB contiguous per store instruction.  The next batch's
 * descriptors and header chunks are in flight during the current batch's
 * spans. */

/* one frame's parse, lane = frame */
struct WParse {
	Rec r;
	u32x4 saddr, daddr;
	uint32_t wck;          /* udp len | check << 16 (wire bytes) */
	uint32_t hsum;         /* IPv4 header word sum (iphdr verify) */
	int hi;                /* frame-relative span end */
	bool want, good, slow, v4;
};

/* per-lane header stage: 6 chunks, 16-byte aligned lane stride */
constexpr uint32_t WSTAGE = 4 * STAGE_CHUNKS + 4;

/* The batch's header chunks are loaded 8 lanes per frame (chunk wl % 8 of
 * frame 8i + wl / 8 in hv[i]): 8 frames per load instruction instead of 64
 * scattered lines per instruction with one lane per frame (measured 1.7x
 * slower without VERIFY).  The lanes then write them to the owning frames'
 * LDS stages. */
constexpr int WHDR = 8;

static __device__ __forceinline__ WParse rx_parse_hdr(const RFrame &f, const uint32_t (&hdr)[13],
						      bool verify);

static __device__ __forceinline__ WParse rx_parse_lane(const RFrame &f, const u32x4 (&hv)[WHDR],
						       uint32_t *hstage, uint32_t wl, bool verify)
{
	const uint32_t nc = rx_nchunks(f);
	const uint32_t fh = rx_h(f, nc);
	uint32_t *wst = hstage + (wl & ~63u) * WSTAGE;        /* the wave's stages */
#pragma unroll
	for (int i = 0; i < WHDR; i++)
		if ((wl & 7u) < STAGE_CHUNKS)
			*((u32x4 *)(wst + (8u * i + ((wl & 63u) >> 3)) * WSTAGE + 4u * (wl & 7u))) = hv[i];
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	/* hdr[i] = frame bytes [12 + 4i, 16 + 4i): from the lane's own stage
	 * (dword offset fh / 4 is per lane; selects over registers made the
	 * compiler index a scratch copy), realigned by fh % 4 */
	const uint32_t *st = wst + (wl & 63u) * WSTAGE;
	uint32_t d[14];
#pragma unroll
	for (int i = 0; i < 14; i++)
		d[i] = st[(fh >> 2) + i];
	/* the next batch rewrites the stages: reads first */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	uint32_t hdr[13];
#pragma unroll
	for (int i = 0; i < 13; i++)
		hdr[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], fh & 3u);
	return rx_parse_hdr(f, hdr, verify);
}

/* packet_parse(), as rx_frame, from hdr[i] = frame bytes [12 + 4i, 16 + 4i)
 * (bytes past the frame's length may be anything: every field read from
 * them is behind a length test) */
static __device__ __forceinline__ WParse rx_parse_hdr(const RFrame &f, const uint32_t (&hdr)[13],
						      bool verify)
{
	const uint32_t len = rx_len(f);
	auto f0 = [&](int x) { return hdr[(x - 12) >> 2]; };
	auto f2 = [&](int x) {
		const int i = (x - 12) >> 2;
		return __builtin_amdgcn_alignbyte(hdr[i + 1], hdr[i], 2u);
	};
	const uint32_t w12 = f0(12), w20 = f0(20), w26 = f2(26), w30 = f2(30);
	const uint32_t p0 = w12 & 0xffu, p1 = (w12 >> 8) & 0xffu;
	const uint32_t ihl = (w12 >> 16) & 0xfu;
	const bool present = rx_present(f);
	const bool eth_ok = present && len >= 14;
	const bool is4 = eth_ok && (p0 == 0x08 || p1 == 0x00);
	const uint32_t l4v4 = 14u + (ihl == 5 ? 20u : (ihl << 2));
	const bool ok4 = is4 && len >= 34 && (w20 >> 24) == 17 && l4v4 + 8 <= len;
	const bool is6 = eth_ok && !is4 && p0 == 0x86 && p1 == 0xDD && len >= 54;
	const bool ok6 = is6 && (w20 & 0xffu) == 17 && len >= 62;
	WParse P;
	P.slow = (ok4 && ihl != 5) || (is6 && (w20 & 0xffu) != 17);
	const bool ok = (ok4 && ihl == 5) || ok6;
	P.v4 = ok4;
	const uint32_t l4 = ok ? (ok4 ? 34u : 54u) : 0u;
	P.wck = ok ? (ok4 ? f2(38) : f2(58)) : 0u;
	P.r.family = ok ? (ok4 ? 4u : 6u) : 0u;
	P.r.l4 = l4;
	P.r.ports = ok ? (ok4 ? f2(34) : f2(54)) : 0u;
	P.r.ulen = ((P.wck & 0xffu) << 8) | ((P.wck >> 8) & 0xffu);
	P.r.status = !ok ? XCSUM_RX_PARSE : (w26 == w30 ? XCSUM_RX_STATS : XCSUM_RX_OK);
	P.saddr = ok4 ? u32x4{w26, 0u, 0u, 0u} : u32x4{f2(22), w26, w30, f2(34)};
	P.daddr = ok4 ? u32x4{w30, 0u, 0u, 0u} : u32x4{f2(38), f2(42), f2(46), f2(50)};
	P.hsum = be_words4(f2(14)) + be_words4(f2(18)) + be_words4(f2(22)) + be_words4(w26) +
		 be_words4(w30);
	P.want = verify && P.r.status == XCSUM_RX_OK && !P.slow;
	P.good = P.want && P.r.ulen >= 8 && l4 + P.r.ulen <= len;
	P.hi = (int)(l4 + P.r.ulen);
	return P;
}

static __device__ __forceinline__ uint32_t bperm(uint32_t src_lane, uint32_t v)
{
	return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

/* a step's frame, fetched from its owning lane */
struct WStep {
	RFrame f;
	int hi;
	uint32_t fl;           /* bit 0: IPv4 span start, bit 1: good */
};

template <int G>
static __device__ __forceinline__ WStep rx_step_frame(const RFrame &f, int hi, uint32_t fl,
						      uint32_t src)
{
	const uint64_t e = (uint64_t)(uintptr_t)f.eth;
	WStep s;
	if (G == 64) {   /* one frame per step: wave-uniform, scalar reads */
		const int j = (int)__builtin_amdgcn_readfirstlane(src);
		s.f.eth = (const uint8_t *)(uintptr_t)(
			((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(e >> 32), j) << 32) |
			(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, j));
		s.f.meta = (uint32_t)__builtin_amdgcn_readlane((int)f.meta, j);
		s.hi = __builtin_amdgcn_readlane(hi, j);
		s.fl = (uint32_t)__builtin_amdgcn_readlane((int)fl, j);
		return s;
	}
	s.f.eth = (const uint8_t *)(uintptr_t)(((uint64_t)bperm(src, (uint32_t)(e >> 32)) << 32) |
					       bperm(src, (uint32_t)e));
	s.f.meta = bperm(src, f.meta);
	s.hi = (int)bperm(src, (uint32_t)hi);
	s.fl = bperm(src, fl);
	return s;
}

/* the G-lane span sum of a step's frame (all lanes of the group get it) */
template <int G, int K>
static __device__ __forceinline__ uint32_t rx_step_sum(const uint32_t *tab, const WStep &s,
						       const u32x4 (&v)[K], uint32_t lane)
{
	const uint32_t nchunks = rx_nchunks(s.f);
	const uint32_t fh = rx_h(s.f, nchunks);
	const int lo = (s.fl & 1u) ? 26 : 22;
	const int hi = s.hi;
	uint32_t E = 0, O = 0;
	if (__builtin_amdgcn_ballot_w64((s.fl & 2u) && nchunks > K * G)) {
		for (uint32_t c = lane; c < nchunks; c += G) {
			const int cb = rx_chunk_off(fh, c);
			u32x4 x = __builtin_nontemporal_load((gu32x4 *)XB_LOAD(
				s.f.eth + cb, 16, rx_ok_lo(s.f), rx_ok_hi(s.f), XB_RX_CHUNK, c, g_rx_zero));
			if (cb < lo || cb + 16 > hi)
				x = keep_span(tab, x, lo - cb, hi - cb);
			accum(x, E, O);
		}
	} else {
#pragma unroll
		for (int k = 0; k < K; k++) {
			const int cb = rx_chunk_off(fh, lane + k * G);
			const u32x4 x = k == 0 ? keep_span(tab, v[k], lo - cb, hi - cb)
					       : v[k] & span_mask(tab, hi - cb);
			accum(x, E, O);
		}
	}
	const uint32_t sum = ((uintptr_t)s.f.eth & 1u) ? (O << 8) + E : (E << 8) + O;
	return seg_sum<G>(sum);
}


/* hstage: 256 * WSTAGE dwords of LDS, 16-byte aligned; span: the mask table,
 * initialised (span_init + block barrier) by the caller */
template <int G, int K>
static __device__ __forceinline__ void rx_wide_body(RxArgs a, uint32_t *hstage,
						    const uint32_t *span)
{
	constexpr uint32_t FPS = 64 / G;        /* frames per step */
	constexpr uint32_t STEPS = G;           /* 64 frames per batch */
	/* the next batch's headers go out HDR_LEAD steps before this batch ends:
	 * 4 steps config 2 -2.3 %, config 5 -3.1 % against 0 (rx_wide/rxlead) */
	constexpr uint32_t HDR_LEAD = 4;   /* even */
	const uint32_t wl = threadIdx.x & 63u;  /* lane = frame of the batch */
	const uint32_t lane = wl & (G - 1);     /* lane in the step's group */
	const uint32_t grp = wl / G;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
	const uint32_t nw = gridDim.x * 4u;
	const bool verify = (a.flags & XCSUM_F_VERIFY) != 0;
	const bool iphdr = (a.flags & XCSUM_F_IPHDR) != 0;
	/* batch b: logical frames 64b..64b+63, one 64-frame tile of the visiting
	 * order (launch_rx prepares tiles of 2^6), so frames base(b) + wl */
	rx_resolve_order(a);
	const uint32_t nb = (a.ord.nlog + 63u) / 64u;
	auto base = [&](uint32_t bb) { return frame_of(a.ord, bb * 64u); };
	const uint8_t *zero = (const uint8_t *)g_rx_zero;
	uint32_t delivered = 0;

	auto hdr_issue = [&](const RFrame &f, u32x4 (&hv)[WHDR]) {
		const uint32_t c = wl & 7u;
#pragma unroll
		for (int i = 0; i < WHDR; i++) {
			const WStep s = rx_step_frame<8>(f, 0, 0u, 8u * i + (wl >> 3));
			const uint32_t nc = rx_nchunks(s.f);
			const uint32_t h = rx_h(s.f, nc);
			/* temporal: the span loads re-read these lines one batch
			 * later; loaded nontemporal they were evicted first and
			 * fetched twice (+220 B per MTU frame, FETCH_SIZE) */
			hv[i] = *((gu32x4 *)(c < nc && c < STAGE_CHUNKS
						     ? XB_LOAD(s.f.eth + rx_chunk_off(h, c), 16, rx_ok_lo(s.f),
							       rx_ok_hi(s.f), XB_RX_CHUNK, c, zero)
						     : zero));
		}
	};
	auto span_issue = [&](const WStep &s, u32x4 (&v)[K]) {
		const uint32_t nc = (s.fl & 2u) ? rx_nchunks(s.f) : 0u;  /* only frames to verify */
		const uint32_t h = rx_h(s.f, rx_nchunks(s.f));
#pragma unroll
		for (int k = 0; k < K; k++) {
			const uint32_t c = lane + k * G;
			v[k] = __builtin_nontemporal_load(
				(gu32x4 *)(c < nc ? XB_LOAD(s.f.eth + rx_chunk_off(h, c), 16, rx_ok_lo(s.f),
							    rx_ok_hi(s.f), XB_RX_CHUNK, c, zero)
						  : zero));
		}
	};

	uint32_t b = wid;
	uint32_t fb = b < nb ? base(b) : a.n;   /* frame of lane 0 */
	RFrame f = rx_resolve(a, rx_desc(a, fb + wl), fb + wl < a.n);
	u32x4 hv[WHDR];
	hdr_issue(f, hv);
	for (; b < nb; b += nw) {
		const uint32_t bn = b + nw;
		const uint32_t fbn = bn < nb ? base(bn) : a.n;
		const u32x3 dn = rx_desc(a, fbn + wl);
		WParse P = rx_parse_lane(f, hv, hstage, threadIdx.x, verify);
		const RFrame fn = rx_resolve(a, dn, fbn + wl < a.n);
		__builtin_amdgcn_sched_barrier(0);
		const bool spans = __builtin_amdgcn_ballot_w64(P.want) != 0;
		/* the next batch's headers: HDR_LEAD steps before this batch's
		 * last (or now when there are no spans to sum) */
		if (bn < nb && (!spans || HDR_LEAD == 0 || HDR_LEAD >= STEPS))
			hdr_issue(fn, hv);

		if (spans) {
			const uint32_t fl = (P.v4 ? 1u : 0u) | (P.good ? 2u : 0u);
			uint32_t mysum = 0;
			u32x4 va[K], vb[K];
			/* A step's frame parameters come from the owning lane
			 * (ds_bpermute, ~100s of cycles) and its loads need them:
			 * fetched two steps ahead, so the loads of step t + 2 go out
			 * as soon as step t's registers are free instead of one
			 * bpermute latency later (the pipeline then keeps two steps
			 * in flight throughout). */
			WStep sa = rx_step_frame<G>(f, P.hi, fl, grp);
			span_issue(sa, va);
			WStep sb = rx_step_frame<G>(f, P.hi, fl, FPS + grp);
#pragma unroll 1
			for (uint32_t t = 0; t < STEPS; t += 2) {
				if (HDR_LEAD > 0 && HDR_LEAD < STEPS && t + HDR_LEAD == STEPS && bn < nb)
					hdr_issue(fn, hv);
				__builtin_amdgcn_sched_barrier(0);
				span_issue(sb, vb);
				__builtin_amdgcn_sched_barrier(0);
				/* parameters of steps t + 2 and t + 3 (clamped past the end:
				 * never issued) */
				const uint32_t t2 = t + 2 < STEPS ? t + 2 : t;
				const uint32_t t3 = t + 3 < STEPS ? t + 3 : t + 1;
				const WStep sc = rx_step_frame<G>(f, P.hi, fl, t2 * FPS + grp);
				const WStep sd = rx_step_frame<G>(f, P.hi, fl, t3 * FPS + grp);
				uint32_t s = rx_step_sum<G, K>(span, sa, va, lane);
				uint32_t x = G == 64 ? s : bperm((wl % FPS) * G, s);
				if (wl / FPS == t)
					mysum = x;
				if (t + 2 < STEPS) {
					__builtin_amdgcn_sched_barrier(0);
					span_issue(sc, va);
					__builtin_amdgcn_sched_barrier(0);
				}
				s = rx_step_sum<G, K>(span, sb, vb, lane);
				x = G == 64 ? s : bperm((wl % FPS) * G, s);
				if (wl / FPS == t + 1)
					mysum = x;
				sa = sc;
				sb = sd;
			}
			bool good = P.good;
			if (good) {
				const uint32_t s = mysum + 17u + P.r.ulen;
				good = (P.wck >> 16) == 0 ? P.r.family == 4 : fold16(s) == 0xffffu;
			}
			if (iphdr && P.r.family == 4)
				good = good && fold16(P.hsum) == 0xffffu;
			if (P.want && !good)
				P.r.status = XCSUM_RX_CSUM;
		}

		/* the general case, one frame at a time by the whole wave */
		uint64_t sm = __builtin_amdgcn_ballot_w64(P.slow);
		while (sm) {
			const uint32_t j = __builtin_ctzll(sm);
			sm &= sm - 1;
			const uint64_t e = (uint64_t)(uintptr_t)f.eth;
			const uint8_t *eth = (const uint8_t *)(uintptr_t)(
				((uint64_t)__builtin_amdgcn_readlane((int)(e >> 32), (int)j) << 32) |
				(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, (int)j));
			const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)rx_len(f), (int)j);
			const Rec rs = rx_slow<64>(eth, len, wl, true, verify, iphdr);
			if (wl == j) {
				P.r = rs;
				/* addresses from global memory, iph + 12 / iph6 + 8 */
				auto ld4 = [&](uint32_t o) {
					return (uint32_t)eth[o] | ((uint32_t)eth[o + 1] << 8) |
					       ((uint32_t)eth[o + 2] << 16) | ((uint32_t)eth[o + 3] << 24);
				};
				if (rs.family == 4) {
					P.saddr = u32x4{ld4(26), 0u, 0u, 0u};
					P.daddr = u32x4{ld4(30), 0u, 0u, 0u};
				} else if (rs.status != XCSUM_RX_PARSE) {
					P.saddr = u32x4{ld4(22), ld4(26), ld4(30), ld4(34)};
					P.daddr = u32x4{ld4(38), ld4(42), ld4(46), ld4(50)};
				}
			}
		}

		/* the record: 64 bytes per lane */
		const Rec &r = P.r;
		const bool pok = r.status != XCSUM_RX_PARSE;
		const uint64_t addr = (uint64_t)(f.eth - a.umem);
		const uint64_t body = pok ? addr + r.l4 + 8 : 0;
		const u32x4 zero4 = {0u, 0u, 0u, 0u};
		/* through the wave's stage, so that each store instruction writes
		 * 1 KB contiguous (lane l: bytes 16l.. of the i-th KB); per-lane
		 * 64-byte stores measured 7-10% slower header-only, 1-2% with
		 * VERIFY (profiles/r01/rx_wide/reclds) */
		{
			uint32_t *wst = hstage + (threadIdx.x & ~63u) * WSTAGE;
			u32x4 *rs = (u32x4 *)(wst + 16u * wl);
			rs[0] = u32x4{(uint32_t)addr, (uint32_t)(addr >> 32), (uint32_t)body,
				      (uint32_t)(body >> 32)};
			rs[1] = u32x4{pok ? r.ulen - 8u : 0u,
				      r.status | (r.family << 8) | ((pok ? r.l4 : 0u) << 16), r.ports, 0u};
			rs[2] = pok ? P.saddr : zero4;
			rs[3] = pok ? P.daddr : zero4;
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			u32x4 *m = (u32x4 *)(a.msgs + fb);
#pragma unroll
			for (uint32_t i = 0; i < 4; i++) {
				const u32x4 v = *((const u32x4 *)(wst + 256u * i + 4u * wl));
				if (fb + 16u * i + (wl >> 2) < a.n &&
				    XB_IDX(fb + 16u * i + (wl >> 2), a.n, XB_RX_REC))
					store_rec(&m[64u * i + wl], v);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			if (rx_present(f) && r.status == XCSUM_RX_OK)
				delivered++;
		}
		f = fn;
		fb = fbn;
	}
	if (a.count) {
		__shared__ uint32_t wsum[4];
		const uint32_t tot = seg_sum<64>(delivered);
		if ((threadIdx.x & 63) == 0)
			wsum[threadIdx.x >> 6] = tot;
		__syncthreads();
		if (threadIdx.x == 0 && XB_IDX(blockIdx.x, RX_PART_MAX, XB_RX_PART))
			a.part[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
	}
}

template <int G, int K>
__global__ void __launch_bounds__(256) rx_wide_kernel(RxArgs a)
{
	__shared__ __attribute__((aligned(16))) uint32_t span[SPAN_DWORDS];
	__shared__ __attribute__((aligned(16))) uint32_t hstage[256 * WSTAGE];
	span_init(span);
	__syncthreads();
	rx_wide_body<G, K>(a, hstage, span);
}

/* ---- stream receive kernel (geometry U = 3): packed small frames ---------
 * The receive side of csum_stream_kernel.  A wave takes 64 consecutive
 * descriptors (lane = frame) and reads the region the 64 frames occupy --
 * [first frame, last frame's end) -- as KC coalesced 1 KiB loads into its LDS
 * stage, with no per-frame chunk grid.  Every lane then parses its frame
 * (rx_parse_hdr), sums its span for VERIFY and builds its record from that
 * copy; the 64 records go out through the same stage, 1 KiB per nontemporal
 * store instruction.  The next region's loads (and the descriptors after
 * it) are in flight while one region is processed.
 * A wave whose frames do not fit the stage (a long frame, descriptors out of
 * UMEM order) takes every frame through rx_slow, the general path; a sparse
 * batch (one frame per UMEM chunk, as an RX ring delivers them) runs the
 * group kernel (4,2,1) in region order, decided once per launch. */
constexpr uint32_t RXS_SLACK = 8;   /* chunks past the region: a short last
				       frame's header reads stay in the stage */

template <int KC>
__global__ void __launch_bounds__(256) rx_stream_kernel(RxArgs a)
{
	constexpr uint32_t SC = KC * 64 + RXS_SLACK;   /* stage chunks per wave */
	static_assert(KC >= 4, "the 64 records (4 KiB) go out through the stage");
	static_assert(4 * SC * 4 >= GroupStage<4>::DWORDS && 4 * SC * 4 >= 256 * WSTAGE,
		      "the fallbacks' stages fit");
	__shared__ __attribute__((aligned(16))) u32x4 rstage[4 * SC];
	__shared__ __attribute__((aligned(16))) uint32_t span[SPAN_DWORDS];
	span_init(span);
	__syncthreads();
	rx_resolve_order(a);
	if (a.ord.rshift != 0) {
		/* sparse batch, in region order (rx_resolve_order): what the
		 * small-frame defaults were before this kernel -- frame groups
		 * (4,2,1) with VERIFY, the lane-per-frame parse (4,2,0) without */
		if (a.flags & XCSUM_F_VERIFY)
			rx_group_body<4, 2, 1>(a, (uint32_t *)rstage, span);
		else
			rx_wide_body<4, 2>(a, (uint32_t *)rstage, span);
		return;
	}
	const uint32_t lane = threadIdx.x & 63u;
	u32x4 *stage = rstage + (threadIdx.x >> 6) * SC;
	const uint8_t *st8 = (const uint8_t *)stage;
	const uint32_t nw = gridDim.x * 4u;
	const bool verify = (a.flags & XCSUM_F_VERIFY) != 0;
	const bool iphdr = (a.flags & XCSUM_F_IPHDR) != 0;
	const uint8_t *zero = (const uint8_t *)g_rx_zero;
	uint32_t delivered = 0;
	uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));

	auto frame_at = [&](uint32_t wi, u32x3 d) {
		return rx_resolve(a, d, 64ull * wi + lane < a.n);
	};
	auto desc_at = [&](uint32_t wi) {
		const uint64_t p = 64ull * wi + lane;
		return rx_desc(a, p < a.n ? (uint32_t)p : a.n - 1u);
	};
	/* the region: the first lane's frame start to the last present lane's
	 * end (two readlanes); every present frame must lie inside it (one
	 * ballot) and it must fit the stage, else nch = ~0u (walk) */
	auto region = [&](uint32_t wi, const RFrame &f, uintptr_t &base, uint32_t &nch) {
		const uint64_t rem = a.n - 64ull * wi;
		const uint32_t last = rem > 64 ? 63u : (uint32_t)rem - 1u;
		const uint64_t e = (uint64_t)(uintptr_t)f.eth;
		const uint64_t end = e + rx_len(f);
		const uint64_t lo =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(e >> 32), 0) << 32) |
			(uint32_t)__builtin_amdgcn_readlane((uint32_t)e, 0);
		const uint64_t hi =
			((uint64_t)__builtin_amdgcn_readlane((uint32_t)(end >> 32), last) << 32) |
			(uint32_t)__builtin_amdgcn_readlane((uint32_t)end, last);
		base = (uintptr_t)(lo & ~15ull);
		const bool out = rx_present(f) && (e < lo || end > hi);
		nch = (__builtin_amdgcn_ballot_w64(out) || hi < lo ||
		       hi - base > (uint64_t)KC * 1024u) ? ~0u : (uint32_t)((hi - base + 15) >> 4);
	};
	auto issue_region = [&](const RFrame &f, uintptr_t base, uint32_t nch, u32x4 (&v)[KC]) {
		(void)f;
#ifdef XCSUM_DEBUG_BOUNDS
		/* the present frames' 16-byte blocks, apart from region() */
		uint64_t mn = rx_present(f) ? (uint64_t)(uintptr_t)f.eth : ~0ull;
		uint64_t mx = rx_present(f) ? (uint64_t)(uintptr_t)f.eth + rx_len(f) : 0ull;
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
			v[k] = __builtin_nontemporal_load(
				(gu32x4 *)(nch != ~0u && c < nch
						   ? XB_LOAD((const uint8_t *)base + 16u * c, 16, ok_lo, ok_hi,
							     XB_RX_STREAM, c, zero)
						   : zero));
		}
	};
	auto wave_sync = [] {
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	};

	RFrame fc = frame_at(w, desc_at(w));
	uintptr_t bc = 0;
	uint32_t nc = ~0u;
	u32x4 v[KC];
	if (64ull * w < a.n) {
		region(w, fc, bc, nc);
		issue_region(fc, bc, nc, v);
	}
	u32x3 dn = desc_at(w + nw);
	for (; 64ull * w < a.n; w += nw) {
		/* this region -> LDS (waits for its loads only) */
#pragma unroll
		for (int k = 0; k < KC; k++)
			stage[k * 64 + lane] = v[k];
		const RFrame cur = fc;
		const uintptr_t cbase = bc;
		const uint32_t cnch = nc;
		/* the next region's loads go out before this one is processed */
		if (64ull * (w + nw) < a.n) {
			fc = frame_at(w + nw, dn);
			region(w + nw, fc, bc, nc);
			__builtin_amdgcn_sched_barrier(0);
			issue_region(fc, bc, nc, v);
			dn = desc_at(w + 2 * nw);
		}
		__builtin_amdgcn_sched_barrier(0);
		wave_sync();

		/* parse from the stage (lane = frame) */
		const uint32_t oe = (uint32_t)((uintptr_t)cur.eth - cbase);  /* frame in the stage */
		WParse P;
		if (cnch != ~0u) {
			const uint32_t o = oe + 12u;
			const uint32_t *dw = (const uint32_t *)(st8 + (o & ~3u));
			uint32_t d[14], hdr[13];
#pragma unroll
			for (int i = 0; i < 14; i++)
				d[i] = dw[i];
#pragma unroll
			for (int i = 0; i < 13; i++)
				hdr[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], o & 3u);
			P = rx_parse_hdr(cur, hdr, verify);
		} else {
			/* does not fit the stage: every frame the general way */
			P.r = Rec{XCSUM_RX_PARSE, 0u, 0u, 0u, 0u};
			P.saddr = P.daddr = u32x4{0u, 0u, 0u, 0u};
			P.wck = P.hsum = 0u;
			P.hi = 0;
			P.v4 = false;
			P.want = P.good = false;
			P.slow = rx_present(cur);
		}

		/* verify: the span [addresses, udp + ulen) summed from the stage */
		if (__builtin_amdgcn_ballot_w64(P.want)) {
			bool good = P.good;
			if (good) {
				const uint32_t lo = oe + (P.v4 ? 26u : 22u), hi = oe + (uint32_t)P.hi;
				uint32_t E = 0, O = 0;
				for (uint32_t c = lo >> 4; c < (hi + 15u) >> 4; c++) {
					u32x4 x = stage[c];
					const int cb = (int)(16u * c);
					if (cb < (int)lo || cb + 16 > (int)hi)
						x = keep_span(span, x, (int)lo - cb, (int)hi - cb);
					accum(x, E, O);
				}
				/* the stage base is 16-byte aligned: oe has the frame's
				 * address parity */
				const uint32_t s = ((oe & 1u) ? (O << 8) + E : (E << 8) + O) + 17u + P.r.ulen;
				good = (P.wck >> 16) == 0 ? P.r.family == 4 : fold16(s) == 0xffffu;
			}
			if (iphdr && P.r.family == 4)
				good = good && fold16(P.hsum) == 0xffffu;
			if (P.want && !good)
				P.r.status = XCSUM_RX_CSUM;
		}

		/* the general case, one frame at a time by the whole wave */
		uint64_t sm = __builtin_amdgcn_ballot_w64(P.slow);
		while (sm) {
			const uint32_t j = __builtin_ctzll(sm);
			sm &= sm - 1;
			const uint64_t e = (uint64_t)(uintptr_t)cur.eth;
			const uint8_t *eth = (const uint8_t *)(uintptr_t)(
				((uint64_t)__builtin_amdgcn_readlane((int)(e >> 32), (int)j) << 32) |
				(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, (int)j));
			const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)rx_len(cur), (int)j);
			const Rec rs = rx_slow<64>(eth, len, lane, true, verify, iphdr);
			if (lane == j) {
				P.r = rs;
				auto ld4 = [&](uint32_t o) {
					return (uint32_t)eth[o] | ((uint32_t)eth[o + 1] << 8) |
					       ((uint32_t)eth[o + 2] << 16) | ((uint32_t)eth[o + 3] << 24);
				};
				if (rs.family == 4) {
					P.saddr = u32x4{ld4(26), 0u, 0u, 0u};
					P.daddr = u32x4{ld4(30), 0u, 0u, 0u};
				} else if (rs.status != XCSUM_RX_PARSE) {
					P.saddr = u32x4{ld4(22), ld4(26), ld4(30), ld4(34)};
					P.daddr = u32x4{ld4(38), ld4(42), ld4(46), ld4(50)};
				}
			}
		}

		/* the records through the stage (every read of the region is done) */
		const Rec &r = P.r;
		const bool pok = r.status != XCSUM_RX_PARSE;
		const uint64_t addr = (uint64_t)(cur.eth - a.umem);
		const uint64_t body = pok ? addr + r.l4 + 8 : 0;
		const u32x4 zero4 = {0u, 0u, 0u, 0u};
		wave_sync();
		u32x4 *rs = stage + 4u * lane;
		rs[0] = u32x4{(uint32_t)addr, (uint32_t)(addr >> 32), (uint32_t)body,
			      (uint32_t)(body >> 32)};
		rs[1] = u32x4{pok ? r.ulen - 8u : 0u,
			      r.status | (r.family << 8) | ((pok ? r.l4 : 0u) << 16), r.ports, 0u};
		rs[2] = pok ? P.saddr : zero4;
		rs[3] = pok ? P.daddr : zero4;
		wave_sync();
		u32x4 *m = (u32x4 *)(a.msgs + 64ull * w);
#pragma unroll
		for (uint32_t i = 0; i < 4; i++) {
			const u32x4 x = stage[64u * i + lane];
			if (64ull * w + 16u * i + (lane >> 2) < a.n &&
			    XB_IDX(64ull * w + 16u * i + (lane >> 2), a.n, XB_RX_REC))
				store_rec(&m[64u * i + lane], x);
		}
		wave_sync();   /* the next region overwrites the stage */
		if (rx_present(cur) && r.status == XCSUM_RX_OK)
			delivered++;
	}
	if (a.count) {
		__shared__ uint32_t wsum[4];
		const uint32_t tot = seg_sum<64>(delivered);
		if ((threadIdx.x & 63) == 0)
			wsum[threadIdx.x >> 6] = tot;
		__syncthreads();
		if (threadIdx.x == 0 && XB_IDX(blockIdx.x, RX_PART_MAX, XB_RX_PART))
			a.part[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
	}
}

__global__ void __launch_bounds__(256) rx_count_kernel(const uint32_t *part, uint32_t nblocks,
						      uint32_t *count)
{
	__shared__ uint32_t wsum[4];
	uint32_t v = 0;
	for (uint32_t i = threadIdx.x; i < nblocks; i += 256)
		v += part[i];
	v = seg_sum<64>(v);
	if ((threadIdx.x & 63) == 0)
		wsum[threadIdx.x >> 6] = v;
	__syncthreads();
	if (threadIdx.x == 0)
		*count = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

template <int G, int K, int U>
static hipError_t launch_rx_t(const RxArgs &a, int cus, int bpc, hipStream_t s)
{
	static std::atomic<int> occ_cache[OCC_MAX_DEVICES];
	const int occ = occupancy_cached(occ_cache, [] {
		int nb = 0;
		hipError_t e;
		if constexpr (U == 0)
			e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_wide_kernel<G, K>, 256, 0);
		else if constexpr (U == 3)
			e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_stream_kernel<K>, 256, 0);
		else
			e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel<G, K, U>, 256, 0);
		if (e != hipSuccess || nb <= 0)
			nb = 4;
		return nb;
	});
	/* U == 0 / 3: lane-per-frame parse / stream, a wave per 64 frames */
	uint64_t blocks = (U == 0 || U == 3) ? ((uint64_t)a.n + 255) / 256
				 : (((uint64_t)a.n + (U ? U : 1) - 1) / (U ? U : 1) * G + 255) / 256;
	const uint64_t cap = (uint64_t)cus * ((bpc > 0 && bpc < occ) ? bpc : occ);
	if (blocks > cap)
		blocks = cap;
	if (blocks > RX_PART_MAX)
		blocks = RX_PART_MAX;
	if (blocks == 0)
		blocks = 1;
	(void)hipGetLastError();  /* clear a stale error (e.g. hipErrorNotReady from
	                           * someone's hipEventQuery) before checking ours */
	if constexpr (U == 0)
		hipLaunchKernelGGL((rx_wide_kernel<G, K>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	else if constexpr (U == 3)
		hipLaunchKernelGGL((rx_stream_kernel<K>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	else
		hipLaunchKernelGGL((rx_kernel<G, K, U>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	if (a.count)
		hipLaunchKernelGGL(rx_count_kernel, dim3(1), dim3(256), 0, s, a.part,
				   (uint32_t)blocks, a.count);
	return hipGetLastError();
}

#define XCSUM_RX_GEOMETRIES(X) \
	X(2, 4, 1) X(2, 4, 2) X(4, 2, 1) X(4, 2, 2) X(8, 1, 2) X(8, 2, 1) \
	X(16, 2, 1) X(16, 3, 1) X(16, 6, 1) X(16, 6, 2) X(64, 9, 1) \
	X(4, 2, 0) X(8, 2, 0) X(16, 3, 0) X(16, 6, 0) X(32, 3, 0) X(64, 2, 0) X(64, 9, 0) \
	X(64, 8, 3)

/* xcsum_ctx_set_tuning(XCSUM_TUNE_RX_GEOMETRY): compiled in? */
bool rx_geometry_supported(int G, int K, int U)
{
#define X(g_, k_, u_) if (G == g_ && K == k_ && U == u_) return true;
	XCSUM_RX_GEOMETRIES(X)
#undef X
	return false;
}

hipError_t launch_rx(const RxArgs &a, uint32_t len_hint, int cus, const Tuning &t, hipStream_t s)
{
	if (a.n == 0)
		return hipSuccess;
	RxArgs b = a;
	/* the context's forced geometry (sweeps and tests); B = blocks per CU
	 * (0: occupancy) */
	int G = t.rx_G, K = t.rx_K, U = t.rx_U, B = t.rx_B;
	if (!G) {
		U = 1;
		B = 0;
		/* chunks of a typical frame from eth+12 to its end: cover it in
		 * one preload with as few lanes as that allows; without VERIFY
		 * only the 6-chunk header stage is loaded.  Measured
		 * (tools/bench_rx.py, profiles/r01/bench_rx_*.log): two frames per
		 * group per stage pay for their registers only on small frames;
		 * MTU frames run best at two waves per SIMD (B = 2), one frame
		 * per group (profiles/r01/rx_mtu/); 64-byte frames (4,2,1): 17%
		 * faster than (2,4,2) once the edge masks lost their branches
		 * (profiles/r01/rx_mtu/geo_c3.log); the header-only pass at 2
		 * blocks per CU: 9% faster than at full occupancy (geo_plain.log). */
		const uint32_t chunks = (len_hint + 6) / 16;  /* ceil((len + 3 - 12) / 16) */
		if (!(a.flags & XCSUM_F_VERIFY)) {
			/* header only: lane-per-frame parse (no span loads, so
			 * G and K only set the code size): config 4 0.052 ->
			 * 0.039 ms, config 2 0.060 -> 0.057, config 3 0.040 ->
			 * 0.0375 (rx_wide/rxwide6, reclds, rxsmall) */
			if (chunks > 16) { G = 32; K = 3; U = 0; }
			else if (chunks > 8) { G = 4; K = 2; U = 0; }
			else { G = 64; K = 8; U = 3; }   /* stream: config 3 0.0363 ->
							    0.0341 ms (session2/rx_stream) */
		}
		else if (chunks <= 8) { G = 64; K = 8; U = 3; }   /* stream: config 3 VERIFY
								     0.0415 -> 0.0352 ms, group
								     (4,2,1) before */
		else if (chunks <= 16) { G = 8; K = 2; }
		else if (chunks <= 32) { G = 16; K = 2; }
		else if (chunks <= 48) { G = 16; K = 3; }
		else if (chunks <= 96) { G = 32; K = 3; U = 0; }  /* MTU: lane-per-frame
								    * parse, 0.301 -> 0.291 ms
								    * (config 2), 0.286 -> 0.282
								    * (config 4), rxwide6 */
		else { G = 64; K = 9; U = 0; }   /* lane-per-frame parse: config 5
						  * 7.73 -> 6.93 ms (rxwide/) */
	}
	/* visiting order for frames spread over the UMEM (one per 2-4 KB
	 * chunk, as an AF_XDP RX ring delivers them): 32 regions of 64-frame
	 * tiles (the batch-per-wave kernel needs >= 64: a batch is one tile, so
	 * its records stay contiguous); resolved in-kernel (rx_resolve_order),
	 * packed batches keep descriptor order.  On 4096-B chunks
	 * (tools/sweep_rx_order.sh, profiles/r02/rx_order/): config 2 VERIFY
	 * 0.345 -> 0.321 ms, header-only 0.0755 -> 0.069, config 3 VERIFY
	 * 0.070 -> 0.067; 8 or 128 regions and 16-frame tiles were slower.
	 * The context's tuning turns it off (rx_rlog 0) or forces "R,T" (A/B). */
	int rlog = t.rx_rlog < 0 ? 5 : t.rx_rlog, tlog = t.rx_rlog < 0 ? 6 : t.rx_tlog;
	b.dense = order_identity(a.n);
	if (rlog == 0) {
		b.ord = order_identity(a.n);   /* "0": off */
	} else {
		/* "R,T": 2^R regions of 2^T-frame tiles (sweeps) */
		if (U == 0 && tlog < 6)
			tlog = 6;
		b.ord = order_regions(a.n, rlog, tlog);
		/* dense batches keep descriptor order: 8-32 regions measured
		 * slower for the receive kernels (session2/order_dense s23), and
		 * the stream kernel (U = 3) reads consecutive frames */
		b.ord.sparse_only = 1u;
	}
#define X(g_, k_, u_) \
	if (G == g_ && K == k_ && U == u_) return launch_rx_t<g_, k_, u_>(b, cus, B, s);
	XCSUM_RX_GEOMETRIES(X)
#undef X
	return hipErrorInvalidValue;
}

} /* namespace xcsum */
