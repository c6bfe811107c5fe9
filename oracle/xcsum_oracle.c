/*
 * xcsum_oracle.c -- CPU restatement of libxudp's UDP checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline.  The product library
 * (libxudp_amd/libxcsum.so) never links, loads or calls it.
 *
 * Each function restates the reference algorithm with the SAME loop shape
 * (so timing it is a faithful proxy for checksum.h) and cites the reference
 * file:line it follows (paths relative to cclinuxer/libxudp).
 *
 * Parity is pinned two ways (see DESIGN.md "Oracle"):
 *   - against tests/golden fixtures and digests produced by the reference's
 *     own checksum.h / packet.c compiled in the build container
 *     (oracle/_ref, recipe oracle/Makefile, generator tests/golden/make_golden.py);
 *   - against the reference's known-answer vectors.
 */
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

#define ORC_IPPROTO_UDP 17u

static inline u16 orc_bswap16(u16 x) { return (u16)((x >> 8) | (x << 8)); }
static inline u32 orc_bswap32(u32 x)
{
	return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

/* xudp/checksum.h:84-105  checksum(): bytewise big-endian word sum seeded
 * with `sum`, odd tail byte shifted <<8, then ONE fold truncated to u16
 * (the end-around carry of that fold is dropped -- the "legacy quirk"). */
u16 orc_checksum(const u8 *p, u32 num, u32 sum)
{
	u32 i;

	if (num % 2 == 1) {
		--num;
		sum += (u32)p[num] << 8;
	}
	for (i = 0; i < num; i += 2) {
		sum += (u32)p[i] << 8;
		sum += p[i + 1];
	}
	{
		u32 l = sum & 0x0000FFFFu;
		u32 h = sum >> 16;
		u16 c = (u16)(l + h);
		return (u16)~c;
	}
}

/* xudp/checksum.h:107-140  udp_checksum(): IPv4 pseudo-header (saddr, daddr
 * as BE words, + IPPROTO_UDP, + size as a BE word) seeded into checksum().
 * saddr/daddr are passed in network byte order (memory order), exactly as the
 * reference's __be32 arguments.  Returns the HOST-order u16. */
u16 orc_udp_checksum(const u8 *u, u32 saddr_be, u32 daddr_be, u16 size)
{
	u32 sum = 0;
	const u8 *p;
	u8 l[2];

	p = (const u8 *)&saddr_be;
	sum += (u32)p[0] << 8;
	sum += p[1];
	sum += (u32)p[2] << 8;
	sum += p[3];

	p = (const u8 *)&daddr_be;
	sum += (u32)p[0] << 8;
	sum += p[1];
	sum += (u32)p[2] << 8;
	sum += p[3];

	sum += ORC_IPPROTO_UDP;

	l[0] = (u8)(size >> 8); /* htons(size) in memory order */
	l[1] = (u8)size;
	sum += (u32)l[0] << 8;
	sum += l[1];

	return orc_checksum(u, size, sum);
}

/* xudp/checksum.h:142-147  sum32 macro: 32-bit add with end-around carry. */
static inline u32 orc_sum32(u32 sum, u32 val)
{
	u32 carry;
	sum += val;
	carry = sum < val;
	sum += carry;
	return sum;
}

static inline u32 orc_load32(const u8 *p) { u32 v; memcpy(&v, p, 4); return v; }
static inline u16 orc_load16(const u8 *p) { u16 v; memcpy(&v, p, 2); return v; }

/* xudp/checksum.h:149-166  udp6_hdr_csum(): native-endian (little-endian
 * host) u32 words of both addresses, htonl(size), htonl(IPPROTO_UDP). */
u32 orc_udp6_hdr_csum(u32 sum, const u8 *saddr16, const u8 *daddr16, u32 size)
{
	int i;
	for (i = 0; i < 4; i++)
		sum = orc_sum32(sum, orc_load32(saddr16 + 4 * i));
	for (i = 0; i < 4; i++)
		sum = orc_sum32(sum, orc_load32(daddr16 + 4 * i));
	sum = orc_sum32(sum, orc_bswap32(size));
	sum = orc_sum32(sum, orc_bswap32(ORC_IPPROTO_UDP));
	return sum;
}

/* xudp/checksum.h:168-194  do_csum(): native u32 accumulate with carry
 * (the hot loop, :172-176), fold to 17 bits, + u16 tail, + byte tail
 * (glibc defines __LITTLE_ENDIAN, so the byte is added unshifted, :186-187). */
u32 orc_do_csum(const u8 *buf, u32 size)
{
	u32 sum = 0;

	while (size >= 4) {
		sum = orc_sum32(sum, orc_load32(buf));
		buf += 4;
		size -= 4;
	}
	sum = (sum & 0xffffu) + (sum >> 16);
	if (size & 2) {
		sum += orc_load16(buf);
		buf += 2;
	}
	if (size & 1)
		sum += *buf;
	return sum;
}

/* xudp/checksum.h:224-229  csum_fold(): two folds then complement. */
u16 orc_csum_fold(u32 sum)
{
	sum = (sum & 0xffffu) + (sum >> 16);
	sum = (sum & 0xffffu) + (sum >> 16);
	return (u16)~sum;
}

/* xudp/packet.c:105-117  udp_csum6(): do_csum + udp6_hdr_csum + csum_fold,
 * 0 -> CSUM_MANGLED_0 (0xffff, packet.c:23).  Returns the value the
 * reference stores raw into udp->check (memory order == wire order). */
u16 orc_udp_csum6(const u8 *udp, u32 size, const u8 *saddr16, const u8 *daddr16)
{
	u32 sum = orc_do_csum(udp, size);
	u16 c;
	sum = orc_udp6_hdr_csum(sum, saddr16, daddr16, size);
	c = orc_csum_fold(sum);
	if (c == 0)
		c = 0xffff;
	return c;
}

/* xudp/packet.c:43-66  xudp_checksum_half(): IPv4 header checksum from the
 * constant half-sum (ver/ihl/tos, ttl/proto, DF) + tot_len + addresses, in
 * native u16 order; fold, fold, complement.  `iph` points at a 20-byte
 * header built by iph_build (packet.c:68-84).  Returns the raw value stored
 * into iph->check (memory order). */
u16 orc_ip_checksum_half(const u8 *iph)
{
	/* ntohs(IP_VIT) + ntohs((64<<8)+17) + ntohs(IP_DF) on a little-endian host */
	u32 sum = (u32)orc_bswap16(0x4500) + orc_bswap16((64 << 8) + 17) + orc_bswap16(0x4000);
	sum += orc_load16(iph + 2);          /* tot_len (network order, raw) */
	sum += orc_load16(iph + 12);
	sum += orc_load16(iph + 14);
	sum += orc_load16(iph + 16);
	sum += orc_load16(iph + 18);
	sum = (sum & 0xFFFFu) + (sum >> 16);
	sum += sum >> 16;
	return (u16)~sum;
}

/* RFC 1071 checksum over the 20-byte IPv4 header (ihl 5, packet.c:21) with
 * the check field (bytes 10..11) treated as zero.  Equals
 * xudp_checksum_half() on every header iph_build() produces; used to check
 * the fused IP-header output. */
u16 orc_ip_header_rfc(const u8 *iph)
{
	u32 i, sum = 0;
	for (i = 0; i < 20; i += 2) {
		if (i == 10)
			continue;
		sum += ((u32)iph[i] << 8) | iph[i + 1];
	}
	while (sum >> 16)
		sum = (sum & 0xffff) + (sum >> 16);
	return orc_bswap16((u16)~sum); /* memory order */
}

/* ------------------------------------------------------------------------ */
/* Batch driver with the product's semantics (include/xcsum.h):            */
/*   desc[i] = {addr, len, options} (struct xdp_desc, tx.c:450-452),        */
/*   addr = Ethernet frame offset in umem, len = frame length               */
/*   (xudp_packet_udp sets len = payload + 42 / 62, packet.c:168, :190).    */
/*   out[i] = the u16 to store into udp->check (wire order).                */
/* ------------------------------------------------------------------------ */

struct orc_desc { u64 addr; u32 len; u32 options; };

enum { ORC_MODE_V4_LEGACY = 0, ORC_MODE_V4_RFC = 1, ORC_MODE_V6 = 2, ORC_MODE_AUTO = 3 };
#define ORC_FLAG_V4_RFC 0x4u  /* == XCSUM_F_V4_RFC: AUTO mode, IPv4 frames use RFC */

/* RFC 768 IPv4 UDP checksum computed through the reference's own IPv6
 * machinery (do_csum + sum32 + csum_fold, checksum.h:142-229), with the
 * IPv4 pseudo-header.  The reference never emits this (IPv4 check is 0,
 * packet.c:125); it is the optional "V4_RFC" mode. */
static u16 orc_udp_csum4_rfc(const u8 *udp, u32 size, const u8 *saddr4, const u8 *daddr4)
{
	u32 sum = orc_do_csum(udp, size);
	u16 c;
	sum = orc_sum32(sum, orc_load32(saddr4));
	sum = orc_sum32(sum, orc_load32(daddr4));
	sum = orc_sum32(sum, orc_bswap32(size));
	sum = orc_sum32(sum, orc_bswap32(ORC_IPPROTO_UDP));
	c = orc_csum_fold(sum);
	if (c == 0)
		c = 0xffff;
	return c;
}

#define ORC_FLAG_IPHDR  0x2u   /* == XCSUM_F_IPHDR */
#define ORC_FLAG_VERIFY 0x10u  /* == XCSUM_F_VERIFY */

/* RFC 1071 residue of a received IPv4 header, check field included:
 * 0 if it verifies (memory order). */
static u16 orc_ip_header_verify(const u8 *iph)
{
	u32 i, sum = 0;
	for (i = 0; i < 20; i += 2)
		sum += ((u32)iph[i] << 8) | iph[i + 1];
	while (sum >> 16)
		sum = (sum & 0xffff) + (sum >> 16);
	return orc_bswap16((u16)~sum);
}

/* Receive-side verify (the reference has none: group/channel.c:231-255
 * parses but never checks).  The frame's check field is summed with the
 * rest through the reference's own do_csum/sum32/csum_fold
 * (checksum.h:142-229); a valid RFC 768 checksum folds to 0xffff, so
 * csum_fold() returns 0.  udp->check == 0: IPv4 "no checksum" (valid),
 * IPv6 invalid (RFC 2460 8.1). */
static u16 orc_verify(const u8 *frame, u32 len, int fam6, u32 flags)
{
	u32 hdr = fam6 ? 54 : 34, size, sum;
	const u8 *ip = frame + 14, *udp = frame + hdr;
	u16 r;
	if (len < hdr + 8 || len - hdr > 0xffff)
		return 0xffff;
	/* RFC 768: the UDP length is the header's, not the frame's -- received
	 * frames may carry Ethernet padding (xudp_fill_msg, group/channel.c:86, reads it the
	 * same way); a length below 8 or past the frame never verifies */
	size = ((u32)udp[4] << 8) | udp[5];
	if (size < 8 || size > len - hdr)
		return 0xffff;
	sum = orc_do_csum(udp, size);
	if (fam6) {
		sum = orc_udp6_hdr_csum(sum, ip + 8, ip + 24, size);
	} else {
		sum = orc_sum32(sum, orc_load32(ip + 12));
		sum = orc_sum32(sum, orc_load32(ip + 16));
		sum = orc_sum32(sum, orc_bswap32(size));
		sum = orc_sum32(sum, orc_bswap32(ORC_IPPROTO_UDP));
	}
	r = orc_csum_fold(sum);
	if (orc_load16(udp + 6) == 0)
		r = fam6 ? 0xffff : 0;
	if (r == 0 && !fam6 && (flags & ORC_FLAG_IPHDR))
		r = orc_ip_header_verify(ip);
	return r;
}

#define ORC_FLAG_IPHDR_ONLY 0x80u  /* == XCSUM_F_IPHDR_ONLY */

/* XCSUM_F_IPHDR_ONLY (include/xcsum.h): libxudp's IPv4 TX checksum work and
 * nothing else -- xudp_checksum_half() (packet.c:43-66, called from
 * iph_build :83; udp->check stays 0, :125), here as the RFC 1071 header sum
 * orc_ip_header_rfc, equal to it on every header iph_build writes (pinned
 * in tests/test_oracle.py); VERIFY: the residue with the check field, 0 =
 * valid.  AUTO: IPv6 frames have no header checksum: 0.  Malformed under
 * orc_one's rules (frame shorter than its headers, UDP length > 65535,
 * another h_proto): 0, or 0xffff under VERIFY. */
static u16 orc_iphdr_only(const u8 *frame, u32 len, int mode, u32 flags)
{
	const u16 bad = (flags & ORC_FLAG_VERIFY) ? 0xffff : 0;
	if (len < 42)
		return bad;
	if (mode == ORC_MODE_AUTO) {
		u16 proto = ((u16)frame[12] << 8) | frame[13];
		if (proto == 0x86DD)
			return (len >= 62 && len - 54 <= 0xffff) ? 0 : bad;
		if (proto != 0x0800)
			return bad;
	}
	if (len - 34 > 0xffff)
		return bad;
	return (flags & ORC_FLAG_VERIFY) ? orc_ip_header_verify(frame + 14)
					 : orc_ip_header_rfc(frame + 14);
}

static u16 orc_one(const u8 *frame, u32 len, int mode, u32 flags)
{
	int fam6;
	if (flags & ORC_FLAG_IPHDR_ONLY)
		return orc_iphdr_only(frame, len, mode, flags);
	if (mode == ORC_MODE_AUTO) {
		u16 proto = ((u16)frame[12] << 8) | frame[13];
		if (proto == 0x0800)
			mode = (flags & ORC_FLAG_V4_RFC) ? ORC_MODE_V4_RFC : ORC_MODE_V4_LEGACY;
		else if (proto == 0x86DD)
			mode = ORC_MODE_V6;
		else
			return (flags & ORC_FLAG_VERIFY) ? 0xffff : 0;
	}
	fam6 = mode == ORC_MODE_V6;
	if (flags & ORC_FLAG_VERIFY)
		return orc_verify(frame, len, fam6, flags);
	if (len < (fam6 ? 62u : 42u))
		return 0;
	if (fam6) {
		const u8 *ip6 = frame + 14;
		u32 size = len - 54;
		if (size > 0xffff) /* payload_len is 16 bits (packet.c:91) */
			return 0;
		return orc_udp_csum6(ip6 + 40, size, ip6 + 8, ip6 + 24);
	} else {
		const u8 *iph = frame + 14;
		u32 size = len - 34;
		u32 s, d;
		if (size > 0xffff)
			return 0;
		if (mode == ORC_MODE_V4_RFC)
			return orc_udp_csum4_rfc(iph + 20, size, iph + 12, iph + 16);
		memcpy(&s, iph + 12, 4);
		memcpy(&d, iph + 16, 4);
		return orc_bswap16(orc_udp_checksum(iph + 20, s, d, (u16)size));
	}
}

void orc_batch(const u8 *umem, const struct orc_desc *desc, u32 n, u16 *out,
	       int mode, u32 flags)
{
	u32 i;
	for (i = 0; i < n; i++)
		out[i] = orc_one(umem + desc[i].addr, desc[i].len, mode, flags);
}

/* Threaded CPU baseline: static packet partition, one pthread per slice.
 * Returns elapsed wall seconds for `reps` passes (CLOCK_MONOTONIC). */
struct orc_job { const u8 *umem; const struct orc_desc *desc; u32 n; u16 *out; int mode; u32 flags; int reps; };

static void *orc_worker(void *arg)
{
	struct orc_job *j = (struct orc_job *)arg;
	int r;
	for (r = 0; r < j->reps; r++)
		orc_batch(j->umem, j->desc, j->n, j->out, j->mode, j->flags);
	return 0;
}

double orc_batch_timed(const u8 *umem, const struct orc_desc *desc, u32 n, u16 *out,
		       int mode, u32 flags, int nthreads, int reps)
{
	struct orc_job jobs[256];
	pthread_t th[256];
	struct timespec t0, t1;
	u32 per, start = 0;
	int t;

	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	per = (n + nthreads - 1) / nthreads;
	for (t = 0; t < nthreads; t++) {
		u32 cnt = start >= n ? 0 : (n - start < per ? n - start : per);
		jobs[t].umem = umem; jobs[t].desc = desc + start; jobs[t].n = cnt;
		jobs[t].out = out + start; jobs[t].mode = mode; jobs[t].flags = flags;
		jobs[t].reps = reps;
		start += cnt;
	}
	clock_gettime(CLOCK_MONOTONIC, &t0);
	if (nthreads == 1) {
		orc_worker(&jobs[0]);
	} else {
		for (t = 0; t < nthreads; t++)
			pthread_create(&th[t], 0, orc_worker, &jobs[t]);
		for (t = 0; t < nthreads; t++)
			pthread_join(th[t], 0);
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------------ */
/* Frame build: xudp/packet.c:68-203 restated (eth_build :141-150, iph_build  */
/* :68-84 + xudp_checksum_half :43-66, iph_build6 :92-103, udp_build          */
/* :119-126, udp_csum6 :105-117, xudp_packet_udp_payload's copy :196-203).    */
/* Writes the frame at `eth` and returns its length (payload + 42 / 62).      */
/* family 4 or 6; addresses/ports in network order; v4_rfc != 0 fills the    */
/* IPv4 UDP checksum (RFC) where the reference leaves 0 (packet.c:125).       */
/* ------------------------------------------------------------------------ */
static void orc_put16be(u8 *p, u16 v) { p[0] = (u8)(v >> 8); p[1] = (u8)v; }

u32 orc_build_frame(u8 *eth, const u8 *payload, u32 psize, int family,
		    const u8 *dmac, const u8 *smac, const u8 *saddr, u16 sport_be,
		    const u8 *daddr, u16 dport_be, int v4_rfc)
{
	u32 size = 8 + psize;
	u8 *udp;
	memcpy(eth, dmac, 6);                           /* copy_eth(h_dest) */
	memcpy(eth + 6, smac, 6);                       /* copy_eth(h_source) */
	if (family == 4) {
		u8 *iph = eth + 14;
		udp = iph + 20;
		orc_put16be(eth + 12, 0x0800);
		orc_put16be(iph, 0x4500);               /* IP_VIT */
		orc_put16be(iph + 2, (u16)(20 + size)); /* tot_len */
		orc_put16be(iph + 4, 0);                /* id */
		orc_put16be(iph + 6, 0x4000);           /* IP_DF */
		iph[8] = 64;                            /* IP_XUDP_TTL */
		iph[9] = 17;
		memcpy(iph + 12, saddr, 4);
		memcpy(iph + 16, daddr, 4);
		{
			u16 c = orc_ip_checksum_half(iph);
			memcpy(iph + 10, &c, 2);
		}
	} else {
		u8 *ip6 = eth + 14;
		u32 flow = 0x60000000u | ((0x3u << 16) + sport_be);  /* packet.c:96 */
		udp = ip6 + 40;
		orc_put16be(eth + 12, 0x86DD);
		ip6[0] = (u8)(flow >> 24); ip6[1] = (u8)(flow >> 16);
		ip6[2] = (u8)(flow >> 8); ip6[3] = (u8)flow;
		orc_put16be(ip6 + 4, (u16)size);        /* payload_len */
		ip6[6] = 17;
		ip6[7] = 64;
		memcpy(ip6 + 8, saddr, 16);
		memcpy(ip6 + 24, daddr, 16);
	}
	memcpy(udp, &sport_be, 2);
	memcpy(udp + 2, &dport_be, 2);
	orc_put16be(udp + 4, (u16)size);
	orc_put16be(udp + 6, 0);                        /* "must", packet.c:125 */
	memcpy(udp + 8, payload, psize);
	if (family == 6) {
		u16 c = orc_udp_csum6(udp, size, eth + 22, eth + 38);
		memcpy(udp + 6, &c, 2);
	} else if (v4_rfc) {
		u16 c = orc_udp_csum4_rfc(udp, size, eth + 26, eth + 30);
		memcpy(udp + 6, &c, 2);
	}
	return psize + (family == 4 ? 42 : 62);
}

/* ---- receive path: xudp_nic_recv_channel's per-frame work ----------------
 * (group/channel.c:211-267): packet_parse() (include/packet_parse.h:101-165,
 * parse_ipv6 :33-99), the stats-request test (channel.c:182-190) and
 * xudp_fill_msg() (channel.c:69-128), plus an RFC 768/2460 verify driven by
 * the UDP header's own length (received frames may carry Ethernet padding),
 * which the reference does not do.  Restated with the reference's quirks:
 *   - IPv4 is taken when h_proto's first byte is 0x08 OR its second is 0x00
 *     (packet_parse.h:117), so ARP (0x0806) and VLAN (0x8100) frames parse
 *     as IPv4 when their bytes allow;
 *   - ihl != 5 places the UDP header at iph + 4*ihl, ihl < 5 included (:127);
 *   - parse_ipv6 walks up to 8 extension headers but returns iph6 + 1 for
 *     UDP wherever it is found (:62);
 *   - the stats test compares the iphdr saddr/daddr fields (offsets 12, 16
 *     of the IP header) for IPv6 frames too (union, channel.c:241).
 * The reference's own `ret < 0` test (channel.c:241) never fires, so its
 * unparseable frames go on with stale headers; here they are reported
 * (ORC_RX_PARSE) instead. */
enum { ORC_RX_OK = 0, ORC_RX_PARSE = 1, ORC_RX_STATS = 2, ORC_RX_CSUM = 3 };

struct orc_rx_msg {
	u64 frame, body;
	u32 size;
	u8 status, family;
	u16 l4_off, sport_be, dport_be;
	u32 reserved;
	u8 saddr[16], daddr[16];
};

/* packet_parse(): 1 and the L3/L4 offsets, or 0 */
int orc_packet_parse(const u8 *pkt, u32 len, int *family, u32 *l3, u32 *l4)
{
	const u8 *p = pkt + 12;
	if (len < 14)
		return 0;                                   /* access_obj_ok(eth) */
	if (p[0] == 0x08 || p[1] == 0x00) {
		u32 ihl, udp;
		if (len < 14 + 20)
			return 0;
		if (pkt[14 + 9] != 17)
			return 0;
		ihl = pkt[14] & 0xf;
		udp = 14 + (ihl == 5 ? 20 : (ihl << 2));
		if (udp + 8 > len)
			return 0;
		*family = 4;
		*l3 = 14;
		*l4 = udp;
		return 1;
	}
	if (p[0] == 0x86 && p[1] == 0xDD) {
		u32 pos = 14 + 40, i, ol;
		u8 nexthdr;
		if (len < 14 + 40)
			return 0;
		nexthdr = pkt[14 + 6];
		for (i = 0; i < 8; i++) {
			if (pos + 2 > len)
				return 0;
			switch (nexthdr) {
			case 132: case 58: case 59: case 6: case 41:
				return 0;
			case 17:
				if (14 + 40 + 8 > len)
					return 0;
				*family = 6;
				*l3 = 14;
				*l4 = 14 + 40;          /* iph6 + 1, packet_parse.h:62 */
				return 1;
			case 51:
				ol = ((u32)pkt[pos + 1] + 2) << 2;
				break;
			case 44:
				ol = 8;
				break;
			case 0: case 43: case 47: case 50: case 60: case 135:
				ol = ((u32)pkt[pos + 1] + 1) << 3;
				break;
			default:
				return 0;
			}
			nexthdr = pkt[pos];
			pos += ol;
		}
		return 0;
	}
	return 0;
}

/* one's-complement sum check of a received UDP datagram at pkt + l4 with the
 * pseudo header of the parsed family: 1 = valid */
static int orc_rx_udp_ok(const u8 *pkt, u32 len, int family, u32 l3, u32 l4)
{
	u32 ulen = ((u32)pkt[l4 + 4] << 8) | pkt[l4 + 5], sum;
	if (ulen < 8 || l4 + ulen > len)
		return 0;
	if (orc_load16(pkt + l4 + 6) == 0)
		return family == 4;                 /* IPv4: no checksum; IPv6: invalid */
	sum = orc_do_csum(pkt + l4, ulen);
	if (family == 6) {
		sum = orc_udp6_hdr_csum(sum, pkt + l3 + 8, pkt + l3 + 24, ulen);
	} else {
		sum = orc_sum32(sum, orc_load32(pkt + l3 + 12));
		sum = orc_sum32(sum, orc_load32(pkt + l3 + 16));
		sum = orc_sum32(sum, orc_bswap32(ulen));
		sum = orc_sum32(sum, orc_bswap32(ORC_IPPROTO_UDP));
	}
	return orc_csum_fold(sum) == 0;
}

/* RFC 1071 over the 4*ihl-byte IPv4 header, check included: 1 = valid */
static int orc_rx_iphdr_ok(const u8 *iph)
{
	u32 n = (u32)(iph[0] & 0xf) << 2, i, sum = 0;
	if (n < 20)
		return 0;
	for (i = 0; i < n; i += 2)
		sum += ((u32)iph[i] << 8) | iph[i + 1];
	while (sum >> 16)
		sum = (sum & 0xffff) + (sum >> 16);
	return sum == 0xffff;
}

void orc_rx_one(const u8 *pkt, u32 len, u64 addr, u32 flags, struct orc_rx_msg *m)
{
	int family = 0;
	u32 l3 = 0, l4 = 0;
	memset(m, 0, sizeof(*m));
	m->frame = addr;
	if (!orc_packet_parse(pkt, len, &family, &l3, &l4)) {
		m->status = ORC_RX_PARSE;
		return;
	}
	m->family = (u8)family;
	m->l4_off = (u16)l4;
	/* xudp_fill_msg(): body = udp + 1, size = ntohs(udp->len) - 8 */
	m->body = addr + l4 + 8;
	m->size = (u32)((((u32)pkt[l4 + 4] << 8) | pkt[l4 + 5]) - 8);
	memcpy(&m->sport_be, pkt + l4, 2);
	memcpy(&m->dport_be, pkt + l4 + 2, 2);
	if (family == 4) {
		memcpy(m->saddr, pkt + l3 + 12, 4);
		memcpy(m->daddr, pkt + l3 + 16, 4);
	} else {
		memcpy(m->saddr, pkt + l3 + 8, 16);
		memcpy(m->daddr, pkt + l3 + 24, 16);
	}
	/* xudp_stats_req_check(): iph->saddr == iph->daddr (channel.c:189) */
	if (memcmp(pkt + l3 + 12, pkt + l3 + 16, 4) == 0) {
		m->status = ORC_RX_STATS;
		return;
	}
	if (flags & ORC_FLAG_VERIFY) {
		/* an IPv4 header shorter than 20 bytes is invalid (RFC 791) */
		if ((family == 4 && (pkt[l3] & 0xf) < 5) ||
		    !orc_rx_udp_ok(pkt, len, family, l3, l4) ||
		    ((flags & ORC_FLAG_IPHDR) && family == 4 && !orc_rx_iphdr_ok(pkt + l3)))
			m->status = ORC_RX_CSUM;
	}
}

void orc_rx_batch(const u8 *umem, const struct orc_desc *desc, u32 n, u32 flags,
		  struct orc_rx_msg *out)
{
	u32 i;
	for (i = 0; i < n; i++)
		orc_rx_one(umem + desc[i].addr, desc[i].len, desc[i].addr, flags, out + i);
}
