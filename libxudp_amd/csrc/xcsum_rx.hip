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
 * G lanes own a frame.  The header parse is a handful of byte loads every
 * lane of the group makes itself (same addresses: one cache line, no
 * cross-lane traffic), so each lane knows every field; lanes 0..3 then store
 * the 64-byte record as four coalesced 16-byte pieces.  The UDP segment is
 * summed in 16-byte chunks on the dword grid of the checksum kernel (chunks
 * laid back from the segment end rounded up to 4 bytes, edge bytes masked
 * before summing), K chunks per lane in flight, G-lane DPP reduction.
 * HBM-bound: the frame bytes once, 16 B descriptor in, 64 B record out.
 */
#include "xcsum_internal.h"
#include <stdlib.h>

namespace xcsum {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

static __device__ __forceinline__ uint32_t dot_even(uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot4(w, 0x00010001u, acc, false);
}
static __device__ __forceinline__ uint32_t dot_odd(uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot4(w, 0x01000100u, acc, false);
}

static __device__ __forceinline__ void accum(u32x4 v, uint32_t &E, uint32_t &O)
{
	E = dot_even(v.x, E); O = dot_odd(v.x, O);
	E = dot_even(v.y, E); O = dot_odd(v.y, O);
	E = dot_even(v.z, E); O = dot_odd(v.z, O);
	E = dot_even(v.w, E); O = dot_odd(v.w, O);
}

template <int G>
static __device__ __forceinline__ uint32_t seg_sum(uint32_t v)
{
	if (G >= 2)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
	if (G >= 4)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
	if (G >= 8)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
	if (G >= 16)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
	if (G >= 32) {
		auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
		v = p[0] + p[1];
	}
	if (G >= 64) {
		auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
		v = q[0] + q[1];
	}
	return v;
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
						   uint32_t head, uint32_t tail, uint32_t c)
{
	u32x4 v = {0u, 0u, 0u, 0u};
	if (c < n) {
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

template <int G, int K>
__global__ void __launch_bounds__(256) rx_kernel(RxArgs a)
{
	const uint32_t lane = threadIdx.x & (G - 1);
	const uint32_t seg = (blockIdx.x * 256u + threadIdx.x) / G;
	const uint32_t nseg = gridDim.x * (256u / G);
	const bool verify = (a.flags & XCSUM_F_VERIFY) != 0;
	const bool iphdr = (a.flags & XCSUM_F_IPHDR) != 0;
	uint32_t delivered = 0;

	for (uint32_t p = seg; p < a.n; p += nseg) {
		const u32x4 d = *((gu32x4 *)(a.desc + p));
		const uint64_t addr = ((uint64_t)d.y << 32) | d.x;
		const uint32_t len = d.z;
		const uint8_t *pkt = a.umem + addr;
		const Parsed ps = packet_parse(pkt, len);

		uint32_t status = XCSUM_RX_PARSE;
		uint32_t ulen = 0, sport = 0, dport = 0;
		if (ps.ok) {
			const uint8_t *udp = pkt + ps.l4;
			ulen = be16(udp + 4);
			sport = (uint32_t)udp[0] | ((uint32_t)udp[1] << 8);
			dport = (uint32_t)udp[2] | ((uint32_t)udp[3] << 8);
			/* xudp_stats_req_check(): iphdr saddr/daddr fields, both
			 * families (the union, channel.c:241) */
			const uint8_t *ip = pkt + ps.l3;
			const bool stats = ip[12] == ip[16] && ip[13] == ip[17] &&
					   ip[14] == ip[18] && ip[15] == ip[19];
			status = stats ? XCSUM_RX_STATS : XCSUM_RX_OK;
		}

		/* ---- verify (group-uniform control flow: the reductions
		 * below need every lane of the group) ---- */
		if (verify && status == XCSUM_RX_OK) {
			const uint8_t *ip = pkt + ps.l3;
			const uint32_t ihl = ip[0] & 0xfu;
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
				for (uint32_t c0 = lane; c0 < n; c0 += K * G) {
					u32x4 v[K];
#pragma unroll
					for (int k = 0; k < K; k++)
						v[k] = grid_chunk(base, n, head, tail, c0 + k * G);
#pragma unroll
					for (int k = 0; k < K; k++)
						accum(v[k], E, O);
				}
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
				status = XCSUM_RX_CSUM;
		}

		/* ---- the record: lanes 0..3 store one 16-byte piece each ---- */
		if (lane < 4) {
			u32x4 w = {0u, 0u, 0u, 0u};
			if (lane == 0) {
				const uint64_t body = ps.ok ? addr + ps.l4 + 8 : 0;
				w = u32x4{(uint32_t)addr, (uint32_t)(addr >> 32), (uint32_t)body,
					  (uint32_t)(body >> 32)};
			} else if (lane == 1) {
				w.x = ps.ok ? ulen - 8u : 0u;
				w.y = status | (ps.family << 8) | ((ps.ok ? ps.l4 : 0u) << 16);
				w.z = sport | (dport << 16);
				w.w = 0;
			} else if (ps.ok) {
				/* lane 2: saddr, lane 3: daddr (IPv4: 4 bytes) */
				const uint8_t *src = pkt + ps.l3 + (ps.family == 4 ? 12 : 8) +
						     (lane == 3 ? (ps.family == 4 ? 4 : 16) : 0);
				const uint32_t nb = ps.family == 4 ? 4 : 16;
				uint32_t b[4] = {0u, 0u, 0u, 0u};
				for (uint32_t i = 0; i < nb; i++)
					b[i >> 2] |= (uint32_t)src[i] << (8 * (i & 3));
				w = u32x4{b[0], b[1], b[2], b[3]};
			}
			*((u32x4 *)(a.msgs + p) + lane) = w;
		}
		if (lane == 0 && status == XCSUM_RX_OK)
			delivered++;
	}
	if (a.count && lane == 0 && delivered)
		atomicAdd(a.count, delivered);
}

template <int G, int K>
static hipError_t launch_rx_t(const RxArgs &a, int cus, hipStream_t s)
{
	static int occ = 0;
	if (!occ) {
		int nb = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel<G, K>, 256, 0) !=
			    hipSuccess || nb <= 0)
			nb = 4;
		occ = nb;
	}
	uint64_t blocks = ((uint64_t)a.n * G + 255) / 256;
	const uint64_t cap = (uint64_t)cus * occ;
	if (blocks > cap)
		blocks = cap;
	if (blocks == 0)
		blocks = 1;
	hipLaunchKernelGGL((rx_kernel<G, K>), dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

hipError_t launch_rx(const RxArgs &a, uint32_t len_hint, int cus, hipStream_t s)
{
	if (a.n == 0)
		return hipSuccess;
	int G = 16;
	const char *e = getenv("XCSUM_RX_GEOMETRY");   /* "G" for sweeps */
	if (e)
		G = atoi(e);
	else if (len_hint && len_hint <= 160)
		G = 4;
	else if (len_hint > 3000)
		G = 64;
	switch (G) {
	case 4:  return launch_rx_t<4, 2>(a, cus, s);
	case 64: return launch_rx_t<64, 2>(a, cus, s);
	default: return launch_rx_t<16, 4>(a, cus, s);
	}
}

} /* namespace xcsum */
