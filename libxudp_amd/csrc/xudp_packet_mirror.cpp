/*
 * xudp_packet_mirror.cpp -- libxcsum_packet.so: the two void packet.c entry
 * points, xudp_packet_udp() and xudp_packet_udp_payload() (cclinuxer/libxudp
 * xudp/packet.c:156-203), on top of libxcsum.so's xudp_packet_udp_batch().
 *
 * A separate library so that libxcsum.so links beside libxudp's own
 * objs/xudp/packet.o (Makefile:41), which defines the same two symbols: a
 * maintainer either keeps packet.o and calls xudp_packet_udp_batch() from the
 * xudp_frame_send hook (tx.c:696-726; the recommended setup), or links
 * -lxcsum_packet -lxcsum INSTEAD of packet.o to put every per-frame call on
 * the GPU.
 *
 * Failure contract.  The reference functions cannot fail, and their caller
 * publishes the frame right after the call (__xudp_frame_send, tx.c:649-671;
 * xudp_xsk_send_one, tx.c:500) without looking at errno.  A frame whose
 * checksum the device could not compute must never reach the TX ring, and
 * the library computes no checksum on the CPU, so on any failure of the
 * device path these functions print the error and abort() the process
 * before returning -- the frame is never published.  Callers that want an
 * error code instead use xudp_packet_udp_batch(), which returns it.
 *
 * A device that is missing altogether is a start-up problem, not a send-path
 * one: a worker calls xcsum_thread_init(gid) once when it starts (after any
 * fork), which creates its thread's default context on its group's GPU and
 * returns -XCSUM_ERR_NODEV (or another code) then -- before any frame is
 * built.  Without that call the first xudp_packet_udp() creates the context
 * and a missing device ends the process there.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xudp_packet.h"

static void fail(const char *fn, int rc)
{
	int line = 0;
	const char *name = nullptr;
	const int hip = xcsum_last_hip_error(&line, &name);
	fprintf(stderr,
		"%s: the GPU checksum path failed (%d%s%s); the frame cannot be built and would "
		"be published without its checksum: aborting (libxcsum_packet failure contract, "
		"INTEGRATION.md 1)\n",
		fn, rc, hip ? ", " : "", hip && name ? name : "");
	abort();
}

extern "C" void xudp_packet_udp(struct packet_info *info)
{
	const int rc = xudp_packet_udp_batch(nullptr, info, 1, 0);
	if (rc != 0)
		fail("xudp_packet_udp", rc);
}

extern "C" void xudp_packet_udp_payload(struct packet_info *info)
{
	info->data = info->head + XUDP_TX_HEADROOM;           /* packet.c:198 */
	memcpy(info->data, info->payload, info->payload_size); /* packet.c:200 */
	xudp_packet_udp(info);
}
