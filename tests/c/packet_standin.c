/*
 * packet_standin.c -- test infrastructure: a stand-in for libxudp's own
 * objs/xudp/packet.o (ref Makefile:41), which defines xudp_packet_udp() and
 * xudp_packet_udp_payload() (xudp/packet.c:156-203).  tests/c/coexist links
 * it next to -lxcsum to show the two coexist: these definitions are the ones
 * the program's calls reach, and libxcsum.so's batch call does not route
 * through them.  It only counts calls and marks the frame; it builds nothing.
 */
#include "xudp_packet.h"

int standin_calls;

void xudp_packet_udp(struct packet_info *info)
{
	standin_calls++;
	info->len = -1;
}

void xudp_packet_udp_payload(struct packet_info *info)
{
	info->data = info->head + XUDP_TX_HEADROOM;
	xudp_packet_udp(info);
}
