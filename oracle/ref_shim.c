/*
 * ref_shim.c -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
 *
 * Builds the REFERENCE's own hot-path sources in place, so that the oracle
 * restatement (xcsum_oracle.c) and the golden fixtures can be checked against
 * the real thing.  Compiled by oracle/Makefile in the build container only
 * (needs /root/reference); output goes to oracle/_ref/libxudpref.so, which is
 * git-ignored and travels to the GPU box as a prebuilt binary for the
 * cpu_baseline leg of bench.py ("kind": "reference").
 *
 * The reference's packet.c is #included (not copied): that compiles it from
 * where it lies under /root/reference with its own static helpers
 * (udp_csum6, xudp_checksum_half) reachable from this translation unit,
 * and packet.c in turn includes checksum.h.
 */
#include "packet.c" /* -I /root/reference/xudp : xudp/packet.c + xudp/checksum.h */

#include <pthread.h>
#include <time.h>
#include <stdint.h>

/* xudp/checksum.h:107-140 -- returns the host-order value. */
uint16_t ref_udp_checksum(const uint8_t *u, uint32_t saddr_be, uint32_t daddr_be, uint16_t size)
{
	return udp_checksum((u8 *)u, saddr_be, daddr_be, size);
}

/* xudp/packet.c:105-117 -- writes udp->check in place and returns it. */
uint16_t ref_udp_csum6(uint8_t *udp, uint32_t size, const uint8_t *saddr16, const uint8_t *daddr16)
{
	struct in6_addr s, d;
	memcpy(&s, saddr16, 16);
	memcpy(&d, daddr16, 16);
	udp_csum6((struct udphdr *)udp, size, &s, &d);
	return ((struct udphdr *)udp)->check;
}

/* IPv4 RFC 768 UDP checksum composed from the reference's own primitives
 * (do_csum, sum32, csum_fold: checksum.h:142-229) in udp_csum6's order
 * (packet.c:105-117) with the IPv4 pseudo-header.  The reference never emits
 * it (IPv4 udp->check stays 0, packet.c:125); it pins XCSUM_MODE_V4_RFC. */
uint16_t ref_udp_csum4_rfc(const uint8_t *udp, uint32_t size, const uint8_t *saddr4,
			   const uint8_t *daddr4)
{
	u32 sum = do_csum((unsigned char *)udp, size), s, d;
	u16 c;
	memcpy(&s, saddr4, 4);
	memcpy(&d, daddr4, 4);
	sum32(sum, s);
	sum32(sum, d);
	sum32(sum, htonl(size));
	sum32(sum, htonl(IPPROTO_UDP));
	c = csum_fold(sum);
	return c ? c : CSUM_MANGLED_0;
}

/* xudp/packet.c:43-66 -- writes iph->check in place and returns it. */
uint16_t ref_ip_checksum_half(uint8_t *iph)
{
	xudp_checksum_half((struct iphdr *)iph);
	return ((struct iphdr *)iph)->check;
}

/* xudp/packet.c:156-203 -- expose the exported builders with flat arguments.
 * family: 4 or 6.  addresses/ports in network order, as in sockaddr_in(6). */
int ref_packet_udp_payload(uint8_t *head, const uint8_t *payload, int payload_size, int family,
			   const uint8_t *smac, const uint8_t *dmac,
			   const uint8_t *saddr, uint16_t sport_be,
			   const uint8_t *daddr, uint16_t dport_be,
			   int64_t *packet_off)
{
	struct packet_info info;
	struct sockaddr_in from4, to4;
	struct sockaddr_in6 from6, to6;

	memset(&info, 0, sizeof(info));
	info.family = family == 6 ? AF_INET6 : AF_INET;
	info.smac = (unsigned char *)smac;
	info.dmac = (unsigned char *)dmac;
	if (family == 6) {
		memset(&from6, 0, sizeof(from6));
		memset(&to6, 0, sizeof(to6));
		from6.sin6_family = to6.sin6_family = AF_INET6;
		memcpy(&from6.sin6_addr, saddr, 16);
		memcpy(&to6.sin6_addr, daddr, 16);
		from6.sin6_port = sport_be;
		to6.sin6_port = dport_be;
		info.from6 = &from6;
		info.to6 = &to6;
	} else {
		memset(&from4, 0, sizeof(from4));
		memset(&to4, 0, sizeof(to4));
		from4.sin_family = to4.sin_family = AF_INET;
		memcpy(&from4.sin_addr, saddr, 4);
		memcpy(&to4.sin_addr, daddr, 4);
		from4.sin_port = sport_be;
		to4.sin_port = dport_be;
		info.from = &from4;
		info.to = &to4;
	}
	info.head = (char *)head;
	info.payload = (char *)payload;
	info.payload_size = payload_size;
	xudp_packet_udp_payload(&info);
	*packet_off = (int64_t)(info.packet - info.head);
	return info.len;
}

/* Batch driver with the product's descriptor semantics (include/xcsum.h),
 * calling the reference functions per frame.  mode: 0 = IPv4 udp_checksum
 * (legacy, checksum.h:107), 2 = IPv6 udp_csum6 (packet.c:105), 4 = IPv4
 * xudp_checksum_half (packet.c:43, the IPv4 TX call's one checksum).  The IPv6
 * call writes udp->check in place exactly as the reference does, so frames
 * must have check == 0 on entry and are restored to 0 afterwards (the
 * reference's udp_build zeroes it before every call, packet.c:125). */
struct ref_desc { uint64_t addr; uint32_t len; uint32_t options; };

static uint16_t ref_one(uint8_t *f, uint32_t len, int mode)
{
	if (mode == 4) {
		/* libxudp's IPv4 TX checksum: xudp_checksum_half (packet.c:43-66)
		 * alone, storing iph->check in place as the reference does (it
		 * reads neither the old check nor anything past the addresses) */
		if (len < 42 || len - 34 > 0xffff)
			return 0;
		xudp_checksum_half((struct iphdr *)(f + 14));
		return ((struct iphdr *)(f + 14))->check;
	}
	if (mode == 2) {
		uint8_t *ip6 = f + 14;
		uint8_t *udp = ip6 + 40;
		uint16_t c, save;
		if (len < 62)
			return 0;
		memcpy(&save, udp + 6, 2);
		c = ref_udp_csum6(udp, len - 54, ip6 + 8, ip6 + 24);
		memcpy(udp + 6, &save, 2);
		return c;
	} else {
		uint8_t *iph = f + 14;
		uint32_t s, d;
		uint16_t c;
		if (len < 42 || len - 34 > 0xffff)
			return 0;
		memcpy(&s, iph + 12, 4);
		memcpy(&d, iph + 16, 4);
		c = udp_checksum(iph + 20, s, d, (u16)(len - 34));
		return htons(c);
	}
}

void ref_batch(uint8_t *umem, const struct ref_desc *desc, uint32_t n, uint16_t *out, int mode)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		out[i] = ref_one(umem + desc[i].addr, desc[i].len, mode);
}

struct ref_job { uint8_t *umem; const struct ref_desc *desc; uint32_t n; uint16_t *out; int mode; int reps; };

static void *ref_worker(void *arg)
{
	struct ref_job *j = (struct ref_job *)arg;
	int r;
	for (r = 0; r < j->reps; r++)
		ref_batch(j->umem, j->desc, j->n, j->out, j->mode);
	return 0;
}

double ref_batch_timed(uint8_t *umem, const struct ref_desc *desc, uint32_t n, uint16_t *out,
		       int mode, int nthreads, int reps)
{
	struct ref_job jobs[256];
	pthread_t th[256];
	struct timespec t0, t1;
	uint32_t per, start = 0;
	int t;

	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	per = (n + nthreads - 1) / nthreads;
	for (t = 0; t < nthreads; t++) {
		uint32_t cnt = start >= n ? 0 : (n - start < per ? n - start : per);
		jobs[t].umem = umem; jobs[t].desc = desc + start; jobs[t].n = cnt;
		jobs[t].out = out + start; jobs[t].mode = mode; jobs[t].reps = reps;
		start += cnt;
	}
	clock_gettime(CLOCK_MONOTONIC, &t0);
	if (nthreads == 1) {
		ref_worker(&jobs[0]);
	} else {
		for (t = 0; t < nthreads; t++)
			pthread_create(&th[t], 0, ref_worker, &jobs[t]);
		for (t = 0; t < nthreads; t++)
			pthread_join(th[t], 0);
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* include/packet_parse.h:101-165 (packet_parse, parse_ipv6 :33-99), the
 * reference's receive-side parser, compiled where it lies.  Returns its
 * result and the L3/L4 offsets of the headers it found. */
#include <linux/ipv6.h>
#include "packet_parse.h"

int ref_packet_parse(const uint8_t *pkt, uint32_t len, int *family, uint32_t *l3, uint32_t *l4)
{
	struct pkthdrs h;
	int r;
	memset(&h, 0, sizeof(h));
	r = packet_parse(&h, (void *)pkt, (void *)(pkt + len));
	if (r == 1) {
		*family = h.family == AF_INET ? 4 : 6;
		*l3 = (uint32_t)((const uint8_t *)(h.family == AF_INET ? (void *)h.iph : (void *)h.iph6) - pkt);
		*l4 = (uint32_t)((const uint8_t *)h.udp - pkt);
	}
	return r;
}

/* The reference's own per-frame TX work, timed: xudp_packet_udp()
 * (packet.c:156-194: headers, then xudp_checksum_half for IPv4 or udp_csum6
 * for IPv6) on n frames whose payload already sits at its data offset in
 * xudp's 4096-byte slots (data at F + 384, tx.c:31-53) -- what
 * xudp_frame_send does per frame (tx.c:696-726) -- repeated reps times on
 * one thread.  Returns seconds.  For the crossover of DESIGN.md 5.10. */
double ref_packet_udp_timed(uint8_t *umem, uint32_t n, int family, int payload_size, int reps)
{
	struct packet_info info;
	struct sockaddr_in from4, to4;
	struct sockaddr_in6 from6, to6;
	unsigned char smac[6] = {2, 0, 0, 0, 0, 1}, dmac[6] = {2, 0, 0, 0, 0, 2};
	struct timespec t0, t1;
	uint32_t i;
	int r;

	memset(&from4, 0, sizeof(from4));
	memset(&to4, 0, sizeof(to4));
	memset(&from6, 0, sizeof(from6));
	memset(&to6, 0, sizeof(to6));
	from4.sin_family = to4.sin_family = AF_INET;
	from4.sin_addr.s_addr = htonl(0x0a002302);
	to4.sin_addr.s_addr = htonl(0x0a002301);
	from4.sin_port = htons(3486);
	to4.sin_port = htons(40000);
	from6.sin6_family = to6.sin6_family = AF_INET6;
	from6.sin6_addr.s6_addr[0] = 0x10;
	from6.sin6_addr.s6_addr[15] = 2;
	to6.sin6_addr.s6_addr[0] = 0x10;
	to6.sin6_addr.s6_addr[15] = 1;
	from6.sin6_port = htons(3487);
	to6.sin6_port = htons(40000);
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (r = 0; r < reps; r++)
		for (i = 0; i < n; i++) {
			memset(&info, 0, sizeof(info));
			info.family = family == 6 ? AF_INET6 : AF_INET;
			info.smac = smac;
			info.dmac = dmac;
			if (family == 6) {
				info.from6 = &from6;
				info.to6 = &to6;
			} else {
				info.from = &from4;
				info.to = &to4;
			}
			info.head = (char *)umem + (uint64_t)i * 4096 + 320;
			info.data = info.head + 64;
			info.payload = info.data;
			info.payload_size = payload_size;
			xudp_packet_udp(&info);
		}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
