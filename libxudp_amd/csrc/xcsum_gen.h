/*
 * xcsum_gen.h -- synthetic UDP frames, one definition for host and device.
 *
 * A frame is what xudp_packet_udp() writes (cclinuxer/libxudp
 * xudp/packet.c:156-194) at the moment the checksum is taken: eth +
 * IPv4(ihl 5, DF, TTL 64) or IPv6(nexthdr UDP, hop 64) + UDP header with
 * both check fields 0, then the payload.  All variable bytes come from a
 * counter-based SplitMix64 stream keyed by (seed, global frame index), so any
 * shard of a job regenerates exactly the frames of the whole job, on the CPU
 * or on the GPU.
 */
#ifndef XCSUM_GEN_H
#define XCSUM_GEN_H

#include <stdint.h>

#ifdef __HIPCC__
#define XG_FN static inline __host__ __device__
#else
#define XG_FN static inline
#endif

XG_FN uint64_t xg_sm64(uint64_t x)
{
	x += 0x9E3779B97F4A7C15ull;
	x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
	x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
	return x ^ (x >> 31);
}

/* per-frame key */
XG_FN uint64_t xg_key(uint64_t seed, uint64_t gidx)
{
	return xg_sm64(seed ^ xg_sm64(gidx ^ 0x5851F42D4C957F2Dull));
}

/* payload size of frame gidx, uniform in [pmin, pmax] */
XG_FN uint32_t xg_payload_size(uint64_t seed, uint64_t gidx, uint32_t pmin, uint32_t pmax)
{
	if (pmax <= pmin)
		return pmin;
	return pmin + (uint32_t)(xg_sm64(seed * 3u + 0x2545F4914F6CDD1Dull ^ xg_sm64(gidx)) %
				 (uint64_t)(pmax - pmin + 1));
}

#define XG_HDR4 42u /* eth 14 + ip 20 + udp 8 */
#define XG_HDR6 62u /* eth 14 + ip6 40 + udp 8 */

XG_FN uint8_t xg_byte_of(uint64_t w, uint32_t i) { return (uint8_t)(w >> (8 * i)); }

/* 8 payload bytes [8j, 8j+8), little-endian in the returned word */
XG_FN uint64_t xg_payload_word(uint64_t key, uint64_t j)
{
	return xg_sm64(key + 16u + j);
}

/* byte `o` (< header size) of the eth/IP/UDP header of a frame of `len` bytes */
XG_FN uint8_t xg_header_byte(uint32_t family, uint64_t key, uint32_t len, uint32_t o)
{
	uint64_t ports = xg_sm64(key + 7u);
	if (o < 6)
		return xg_byte_of(xg_sm64(key + 1u), o);          /* h_dest */
	if (o < 12)
		return xg_byte_of(xg_sm64(key + 2u), o - 6);      /* h_source */
	if (family == 6) {
		uint32_t ulen = len - 54u;
		uint32_t sport_raw = (uint32_t)xg_byte_of(ports, 0) | ((uint32_t)xg_byte_of(ports, 1) << 8);
		/* ip6_flow_hdr(iph6, 0, (0x3 << 16) + src->sin6_port), packet.c:96 */
		uint32_t flow = 0x60000000u | ((0x3u << 16) + sport_raw);
		switch (o) {
		case 12: return 0x86;
		case 13: return 0xDD;
		case 14: return (uint8_t)(flow >> 24);
		case 15: return (uint8_t)(flow >> 16);
		case 16: return (uint8_t)(flow >> 8);
		case 17: return (uint8_t)flow;
		case 18: case 58: return (uint8_t)(ulen >> 8);
		case 19: case 59: return (uint8_t)ulen;
		case 20: return 17;     /* nexthdr */
		case 21: return 64;     /* hop_limit */
		case 54: return xg_byte_of(ports, 0);
		case 55: return xg_byte_of(ports, 1);
		case 56: return xg_byte_of(ports, 2);
		case 57: return xg_byte_of(ports, 3);
		case 60: case 61: return 0; /* udp->check */
		default: break;
		}
		if (o >= 22 && o < 38)
			return xg_byte_of(xg_sm64(key + 3u + (o - 22) / 8), (o - 22) % 8);
		if (o >= 38 && o < 54)
			return xg_byte_of(xg_sm64(key + 5u + (o - 38) / 8), (o - 38) % 8);
		return 0;
	} else {
		uint32_t tot = len - 14u, ulen = len - 34u;
		uint64_t addrs = xg_sm64(key + 3u);
		switch (o) {
		case 12: return 0x08;
		case 13: return 0x00;
		case 14: return 0x45;   /* IP_VIT, packet.c:21 */
		case 15: return 0x00;
		case 16: return (uint8_t)(tot >> 8);
		case 17: return (uint8_t)tot;
		case 18: case 19: return 0;         /* id */
		case 20: return 0x40; case 21: return 0x00; /* IP_DF */
		case 22: return 64;     /* IP_XUDP_TTL */
		case 23: return 17;     /* IPPROTO_UDP */
		case 24: case 25: return 0;         /* iph->check (left 0) */
		case 34: return xg_byte_of(ports, 0);
		case 35: return xg_byte_of(ports, 1);
		case 36: return xg_byte_of(ports, 2);
		case 37: return xg_byte_of(ports, 3);
		case 38: return (uint8_t)(ulen >> 8);
		case 39: return (uint8_t)ulen;
		case 40: case 41: return 0;         /* udp->check */
		default: break;
		}
		if (o >= 26 && o < 34)
			return xg_byte_of(addrs, o - 26);   /* saddr, daddr */
		return 0;
	}
}

/* byte `o` of the whole frame */
XG_FN uint8_t xg_frame_byte(uint32_t family, uint64_t key, uint32_t len, uint32_t o)
{
	uint32_t hdr = family == 6 ? XG_HDR6 : XG_HDR4;
	if (o < hdr)
		return xg_header_byte(family, key, len, o);
	o -= hdr;
	return xg_byte_of(xg_payload_word(key, o >> 3), o & 7);
}

#endif /* XCSUM_GEN_H */
