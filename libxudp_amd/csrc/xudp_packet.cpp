/*
 * xudp_packet.cpp -- the packet.c-level mirror (include/xudp_packet.h).
 *
 * Header bytes are written on the host with exactly the field values of
 * cclinuxer/libxudp xudp/packet.c (eth_build :141-150, iph_build :68-84,
 * iph_build6 :92-103, udp_build :119-126); both check fields are left 0.
 * All checksum arithmetic -- the IPv4 header checksum (packet.c:43-66) and
 * the UDP checksum (checksum.h / packet.c:105-117) -- runs in the gfx950
 * kernel through xcsum::batch_host_impl.  There is no CPU checksum here.
 */
#include <errno.h>
#include <string.h>
#include <arpa/inet.h>
#include <vector>

#include "xudp_packet.h"
#include "xcsum_internal.h"

#define PKT_ETH 14u
#define PKT_IP4 20u
#define PKT_IP6 40u
#define PKT_UDP 8u

static inline void put16(uint8_t *p, uint16_t v_host)
{
	uint16_t be = htons(v_host);
	memcpy(p, &be, 2);
}

extern "C" void xudp_packet_build_headers(struct packet_info *info)
{
	const uint32_t size = PKT_UDP + (uint32_t)info->payload_size; /* packet.c:162 */
	uint8_t *eth, *udp;

	if (info->family == AF_INET) {
		eth = (uint8_t *)info->data - (PKT_ETH + PKT_IP4 + PKT_UDP);
		uint8_t *iph = eth + PKT_ETH;
		udp = iph + PKT_IP4;
		memcpy(eth + 6, info->smac, 6);
		memcpy(eth, info->dmac, 6);
		put16(eth + 12, 0x0800);
		put16(iph, 0x4500);                      /* IP_VIT */
		put16(iph + 2, (uint16_t)(PKT_IP4 + size));
		put16(iph + 4, 0);                       /* id */
		put16(iph + 6, 0x4000);                  /* IP_DF */
		iph[8] = 64;                             /* IP_XUDP_TTL */
		iph[9] = 17;                             /* IPPROTO_UDP */
		put16(iph + 10, 0);                      /* check: filled by the kernel */
		memcpy(iph + 12, &info->from->sin_addr.s_addr, 4);
		memcpy(iph + 16, &info->to->sin_addr.s_addr, 4);
		memcpy(udp, &info->from->sin_port, 2);
		memcpy(udp + 2, &info->to->sin_port, 2);
		info->len = info->payload_size + (int)(PKT_ETH + PKT_IP4 + PKT_UDP);
	} else {
		eth = (uint8_t *)info->data - (PKT_ETH + PKT_IP6 + PKT_UDP);
		uint8_t *ip6 = eth + PKT_ETH;
		udp = ip6 + PKT_IP6;
		memcpy(eth + 6, info->smac, 6);
		memcpy(eth, info->dmac, 6);
		put16(eth + 12, 0x86DD);
		/* ip6_flow_hdr(iph6, 0, (0x3 << 16) + sin6_port): the raw
		 * network-order port is added as an integer (packet.c:96) */
		uint32_t flow = htonl(0x60000000u | ((0x3u << 16) + info->from6->sin6_port));
		memcpy(ip6, &flow, 4);
		put16(ip6 + 4, (uint16_t)size);          /* payload_len */
		ip6[6] = 17;                             /* nexthdr */
		ip6[7] = 64;                             /* hop_limit */
		memcpy(ip6 + 8, &info->from6->sin6_addr, 16);
		memcpy(ip6 + 24, &info->to6->sin6_addr, 16);
		memcpy(udp, &info->from6->sin6_port, 2);
		memcpy(udp + 2, &info->to6->sin6_port, 2);
		info->len = info->payload_size + (int)(PKT_ETH + PKT_IP6 + PKT_UDP);
	}
	put16(udp + 4, (uint16_t)size);
	put16(udp + 6, 0);                               /* "must", packet.c:125 */
	info->packet = (char *)eth;
}

/* Lazily created per-thread default context, created on first use (i.e.
 * after any fork of the caller) or by xcsum_thread_init: on the thread's
 * group device, else $XCSUM_DEVICE if set, else the next device of the
 * process's round robin (include/xcsum.h, device placement).  Kept for the
 * life of the process, as before: a destructor at thread or process exit
 * could run after the HIP runtime's own teardown. */
namespace {
struct ThreadCtx {
	xcsum_ctx *ctx = nullptr;
};
thread_local ThreadCtx t_ctx;
} /* namespace */

static int default_device()
{
	return getenv("XCSUM_DEVICE") ? XCSUM_DEVICE_ENV : XCSUM_DEVICE_AUTO;
}

extern "C" int xcsum_thread_init(int gid)
{
	if (gid > 1000000)
		return -XCSUM_ERR_INVAL;
	const int want = gid >= 0 ? XCSUM_DEVICE_GROUP(gid) : default_device();
	const int ndev = xcsum_device_count();
	if (ndev < 0)
		return ndev;
	if (t_ctx.ctx) {
		/* already there: keep it if it is on the wanted device */
		if (gid < 0 || xcsum_ctx_device(t_ctx.ctx) == xcsum_device_resolve(want, ndev))
			return 0;
		xcsum_ctx_destroy(t_ctx.ctx);
		t_ctx.ctx = nullptr;
	}
	xcsum_ctx *c = nullptr;
	const int rc = xcsum_ctx_create(want, &c);
	if (rc)
		return rc;
	t_ctx.ctx = c;
	return 0;
}

extern "C" xcsum_ctx *xcsum_thread_ctx(void)
{
	if (!t_ctx.ctx && xcsum_thread_init(-1) != 0)
		return nullptr;
	return t_ctx.ctx;
}

static xcsum_ctx *default_ctx()
{
	return xcsum_thread_ctx();
}

extern "C" int xudp_packet_udp_batch(xcsum_ctx *ctx, struct packet_info *infos, uint32_t n,
				     uint32_t flags)
{
	if (n == 0)
		return 0;
	if (!infos)
		return -XCSUM_ERR_INVAL;
	/* headers first, as packet.c does: every frame is built (info->packet
	 * and info->len set, both check fields 0) even if no device can
	 * checksum it -- the caller then sees the error, never a half-built
	 * frame */
	uint8_t *lo = nullptr, *hi = nullptr;
	for (uint32_t i = 0; i < n; i++) {
		xudp_packet_build_headers(&infos[i]);
		uint8_t *p = (uint8_t *)infos[i].packet, *e = p + infos[i].len;
		if (!lo || p < lo) lo = p;
		if (!hi || e > hi) hi = e;
	}
	if (!ctx)
		ctx = default_ctx();
	if (!ctx)
		return -XCSUM_ERR_NODEV;
	/* descriptors relative to a registered UMEM when every frame is inside
	 * one (pinned DMA / zero-copy), else relative to address 0 */
	uint8_t *base = nullptr;
	for (auto &r : ctx->regions)
		if (r.mapped && lo >= r.host && hi <= r.host + r.size)
			base = r.host;
	/* IPv4 without XCSUM_F_V4_RFC: udp->check stays 0 (packet.c:125) and
	 * only iph->check is computed, from the 20-byte header (its tot_len
	 * field included).  A batch of such frames only is libxudp's IPv4 call,
	 * XCSUM_F_IPHDR_ONLY: the header kernel on the frames' first 42 bytes.
	 * In a mixed batch, and on a context with resident workgroups (they run
	 * the checksum kernel, and serve libxudp's 100-frame batches faster than
	 * a launch: DESIGN.md 5.10), the checksum kernel is handed eth + IP +
	 * UDP headers of those frames (42 bytes; the UDP result it also returns
	 * is unused). */
	const bool v4_rfc = (flags & XCSUM_F_V4_RFC) != 0;
	bool v4_hdr = !v4_rfc;   /* every frame needs its IPv4 header only */
	for (uint32_t i = 0; i < n && v4_hdr; i++)
		v4_hdr = infos[i].family == AF_INET;
	const bool hdr_only = v4_hdr && ctx->res_wg == 0;   /* the header kernel */
	std::vector<struct xcsum_desc> desc(n);
	std::vector<uint16_t> out(n), out_ip(n);
	for (uint32_t i = 0; i < n; i++) {
		desc[i].addr = (uint64_t)((uint8_t *)infos[i].packet - base);
		desc[i].len = (uint32_t)infos[i].len;
		if (!hdr_only && infos[i].family == AF_INET && !v4_rfc && desc[i].len > 42u)
			desc[i].len = 42u;
		desc[i].options = 0;
	}
	uint32_t kflags = (hdr_only ? XCSUM_F_IPHDR_ONLY : XCSUM_F_IPHDR) |
			  (flags & (XCSUM_F_V4_RFC | XCSUM_F_ZEROCOPY));
	if (!base)
		kflags &= ~XCSUM_F_ZEROCOPY;
	/* Staged copies gather frame by frame when the frames are the caller's
	 * buffers anywhere in memory (a copy of the address range they span
	 * could read unmapped pages between them), and when only headers are
	 * needed (42 of ~1500 bytes per frame).  Whole frames inside one
	 * registered UMEM go by DMA of the range, no host copy. */
	const bool gather = !(kflags & XCSUM_F_ZEROCOPY) && (!base || v4_hdr);
	int rc = xcsum::batch_host_impl(ctx, base, desc.data(), n, out.data(),
					hdr_only ? nullptr : out_ip.data(), XCSUM_MODE_AUTO, kflags,
					gather);
	if (rc)
		return rc;
	if (hdr_only)
		out_ip.swap(out);   /* the header kernel's result is iph->check */
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *eth = (uint8_t *)infos[i].packet;
		if (infos[i].family == AF_INET) {
			memcpy(eth + 24, &out_ip[i], 2);                 /* iph->check */
			if (flags & XCSUM_F_V4_RFC)
				memcpy(eth + 40, &out[i], 2);            /* opt-in RFC UDP check */
		} else {
			memcpy(eth + 60, &out[i], 2);                    /* udp_csum6 */
		}
	}
	return 0;
}

/* xudp_packet_udp / xudp_packet_udp_payload, the void packet.c mirrors, are
 * not in this library: they would clash with libxudp's own packet.o
 * (Makefile:41).  They live in libxcsum_packet.so (xudp_packet_mirror.cpp),
 * which a maintainer links instead of packet.o. */
