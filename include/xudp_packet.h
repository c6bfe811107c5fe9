/*
 * xudp_packet.h -- packet.c-level mirror (drop-in for cclinuxer/libxudp
 * xudp/packet.h + xudp/packet.c), backed by libxcsum.so.
 *
 * struct packet_info is layout-identical to xudp/packet.h:28-53.  Two
 * libraries: libxcsum.so (the batch call, linkable beside libxudp's own
 * packet.o) and libxcsum_packet.so (xudp_packet_udp / _payload, the same
 * symbols as packet.o, linked instead of it).  Header bytes are written on
 * the host exactly as packet.c does (they are the frame's own fields, not
 * checksum work); every checksum is computed by the gfx950 kernel.
 */
#ifndef XUDP_PACKET_H
#define XUDP_PACKET_H

#include <stdint.h>
#include <netinet/in.h>
#include "xcsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* xudp/packet.h:28-53 */
struct packet_info {
	uint8_t family;
	unsigned char *dmac;
	unsigned char *smac;
	union {
		struct sockaddr_in *to;
		struct sockaddr_in6 *to6;
	};
	union {
		struct sockaddr_in *from;
		struct sockaddr_in6 *from6;
	};
	union {
		struct sockaddr_in _from;
		struct sockaddr_in6 _from6;
	};

	char *head;
	char *data;

	char *payload;
	int payload_size;

	char *packet;
	int len;
};

/* xudp/packet.h:58-60: 14 + 2 + 40 + 8 */
#define XUDP_TX_HEADROOM 64

/* ---- libxcsum.so (links beside libxudp's own packet.o) ------------------ */

/* Batched xudp_packet_udp over n frames (the xudp_frame_send loop,
 * tx.c:696-726): host header build for all n, then ONE checksum batch for
 * them all.  ctx NULL = the thread's default context.  flags: XCSUM_F_V4_RFC
 * fills the IPv4 UDP checksum (RFC) instead of 0, XCSUM_F_ZEROCOPY as in
 * xcsum_batch_host.  Frames may live anywhere in host memory; if all of them
 * lie in one registered UMEM the DMA is pinned.  Returns 0 or -XCSUM_ERR_*;
 * on an error every frame is built (info->packet, info->len set) with both
 * check fields 0, so the caller must not publish them. */
int xudp_packet_udp_batch(xcsum_ctx *ctx, struct packet_info *infos, uint32_t n,
			  uint32_t flags);

/* Header build only (both check fields left 0): the host half of
 * xudp_packet_udp, exposed for callers that checksum device-resident frames
 * with xcsum_batch_device(). */
void xudp_packet_build_headers(struct packet_info *info);

/* ---- libxcsum_packet.so: link it INSTEAD of libxudp's packet.o ----------
 * The same two symbols as objs/xudp/packet.o (ref Makefile:41), so they live
 * in their own library; libxcsum.so does not define them.
 * Failure contract: the reference functions cannot fail and their caller
 * publishes the frame right after (tx.c:649-671, :500).  If the device path
 * fails these print the error and abort() the process -- a frame without its
 * checksum is never published.  Use xudp_packet_udp_batch() for an error
 * code instead, and call xcsum_thread_init(gid) when a worker starts: a
 * missing device is then an error code at start-up, not an abort on the
 * first send. */

/* Replaces xudp/packet.c:156-194.  Builds eth + IPv4/IPv6 + UDP headers in
 * front of info->data and fills info->packet / info->len like the reference;
 * IPv4: iph->check via the kernel, udp->check = 0 (packet.c:125);
 * IPv6: udp->check = udp_csum6 (packet.c:188) via the kernel.
 * One-frame batch on the calling thread's default context: correct, but
 * latency-bound (a launch + PCIe round trip per call); batch with
 * xudp_packet_udp_batch(). */
void xudp_packet_udp(struct packet_info *info);

/* Replaces xudp/packet.c:196-203: data = head + XUDP_TX_HEADROOM, copy the
 * payload there, then xudp_packet_udp(). */
void xudp_packet_udp_payload(struct packet_info *info);

#ifdef __cplusplus
}
#endif
#endif /* XUDP_PACKET_H */
