/*
 * coexist.c -- libxcsum.so linked beside libxudp's own packet.o (a stand-in,
 * packet_standin.c), the setup INTEGRATION.md 1 recommends: xudp_send_channel
 * keeps the CPU packet.c (tx.c:605 -> :500) and xudp_frame_send's loop
 * (tx.c:696-726) calls xudp_packet_udp_batch().  Checks:
 *   - the link has no duplicate symbols and the program's xudp_packet_udp /
 *     xudp_packet_udp_payload calls reach packet.o's definitions;
 *   - libxcsum.so defines neither (dlsym on its handle);
 *   - xudp_packet_udp_batch() builds SURVEY Appendix A's KAT4 (IPv4) and KAT3
 *     (IPv6) frames byte for byte, checksums from the GPU, without calling
 *     packet.o's functions.
 * Exit 0: pass; 1: a check failed; 77: no GPU (the batch call said NODEV).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <stdlib.h>

#include "harness.h"
#include "xudp_packet.h"

extern int standin_calls;

static int hex_eq(const uint8_t *p, const char *hex)
{
	for (size_t i = 0; hex[2 * i]; i++) {
		unsigned v;
		if (sscanf(hex + 2 * i, "%2x", &v) != 1 || p[i] != v)
			return 0;
	}
	return 1;
}

static const char KAT4[] = "020000000002020000000001080045000022000040004011e0c80a0023020a0023010d9e"
			   "9c40000e0000616263646566";
static const char KAT3[] = "02000000000202000000000186dd60039f0d000e11401000200030004000000000000000"
			   "0002100020003000400000000000000000010d9f9c40000eebc1616263646566";

int main(void)
{
	unsigned char dmac[6] = {2, 0, 0, 0, 0, 2}, smac[6] = {2, 0, 0, 0, 0, 1};
	static char buf4[256], buf6[256], buf0[256];
	struct sockaddr_in to4, from4;
	struct sockaddr_in6 to6, from6;
	struct packet_info info[2];

	/* libxcsum.so itself defines neither packet.o symbol */
	void *h = dlopen("libxcsum.so", RTLD_NOW | RTLD_NOLOAD);
	CHECK(h != NULL, "libxcsum.so not loaded: %s", dlerror());
	if (h) {
		CHECK(dlsym(h, "xudp_packet_udp_batch") != NULL, "batch call missing");
		CHECK(dlsym(h, "xudp_packet_udp") == NULL, "libxcsum.so defines xudp_packet_udp");
		CHECK(dlsym(h, "xudp_packet_udp_payload") == NULL,
		      "libxcsum.so defines xudp_packet_udp_payload");
	}

	/* the per-packet call reaches packet.o (xudp_send_channel's path) */
	memset(&info[0], 0, sizeof(info[0]));
	info[0].head = buf0;
	xudp_packet_udp_payload(&info[0]);
	CHECK(standin_calls == 1 && info[0].len == -1, "packet.o's definition not reached");

	memset(&to4, 0, sizeof(to4));
	memset(&from4, 0, sizeof(from4));
	to4.sin_family = from4.sin_family = AF_INET;
	to4.sin_port = htons(40000);
	from4.sin_port = htons(3486);
	inet_pton(AF_INET, "10.0.35.1", &to4.sin_addr);
	inet_pton(AF_INET, "10.0.35.2", &from4.sin_addr);
	memset(&to6, 0, sizeof(to6));
	memset(&from6, 0, sizeof(from6));
	to6.sin6_family = from6.sin6_family = AF_INET6;
	to6.sin6_port = htons(40000);
	from6.sin6_port = htons(3487);
	inet_pton(AF_INET6, "1000:2000:3000:4000::1", &to6.sin6_addr);
	inet_pton(AF_INET6, "1000:2000:3000:4000::2", &from6.sin6_addr);

	memset(info, 0, sizeof(info));
	memset(buf4, 0, sizeof(buf4));
	memset(buf6, 0, sizeof(buf6));
	info[0].family = AF_INET;
	info[0].to = &to4;
	info[0].from = &from4;
	info[0].head = buf4;
	info[1].family = AF_INET6;
	info[1].to6 = &to6;
	info[1].from6 = &from6;
	info[1].head = buf6;
	for (int i = 0; i < 2; i++) {
		info[i].dmac = dmac;
		info[i].smac = smac;
		/* the payload already at its data offset, as xudp_frame_send's
		 * zero-copy frames are (tx.c:708-712) */
		info[i].data = info[i].head + XUDP_TX_HEADROOM;
		memcpy(info[i].data, "abcdef", 6);
		info[i].payload_size = 6;
	}
	/* the xudp_frame_send loop, batched (tx.c:696-726) */
	int rc = xudp_packet_udp_batch(NULL, info, 2, 0);
	if (rc == -XCSUM_ERR_NODEV) {
		printf("coexist: no GPU, skipped (link and symbol checks: %d checks, %d failures)\n",
		       checks, failures);
		return failures ? 1 : 77;
	}
	CHECK(rc == 0, "xudp_packet_udp_batch: %d", rc);
	CHECK(standin_calls == 1, "the batch call went through packet.o's functions");
	CHECK(info[0].len == 48 && hex_eq((uint8_t *)info[0].packet, KAT4), "KAT4 frame");
	CHECK(info[1].len == 68 && hex_eq((uint8_t *)info[1].packet, KAT3), "KAT3 frame");
	printf("coexist: %d checks, %d failures\n", checks, failures);
	return failures ? 1 : 0;
}
