/*
 * umem_ring.c -- the TX loop of libxudp with the GPU checksum in it, end to
 * end on the host side, in plain C.  Test infrastructure (and the source of
 * DESIGN.md's end-to-end numbers for xudp's own UMEM mapping).
 *
 * What it replays (cclinuxer/libxudp):
 *   - the UMEM: anon_map() (include/common.h:37-41) as __umem_configure()
 *     maps it (xudp/xsk.c:234), 4096-byte frames, headroom 256: payload at
 *     F + 384;
 *   - xudp_frame_send() (xudp/tx.c:673-734): one route per batch
 *     (xudp_tx_info_prepare, :690), then for every message the packet build
 *     (__xudp_frame_send -> xudp_packet_udp, :649-671) -- here ONE
 *     xudp_packet_udp_batch() call for the batch, or the header build plus one
 *     xcsum_batch_host(INPLACE | IPHDR) call on the registered UMEM;
 *   - xudp_send_tx() -> xq_enq() (tx.c:433-483, include/queue.h:170-189):
 *     descriptors written into the TX ring, then the producer index
 *     published with a write barrier (ring_update_produce, queue.h:90-94).
 *     The checksum call returns before the first descriptor is written, so a
 *     frame is final before the NIC can see it;
 *   - the "NIC": a consumer thread that dequeues like xq_deq() (acquire on
 *     the producer index, queue.h:191-212), checks every frame it is handed
 *     (headers and checksums, against the oracle), and returns the frame
 *     through a completion ring the producer drains before reusing frames
 *     (cq_deq, queue.h:144-168).
 *
 * Variants: the UMEM unregistered (frames gathered and staged), registered
 * (pinned DMA), registered + zero-copy (the kernel reads the UMEM over
 * PCIe); IPv4 (udp->check 0 as packet.c:125), IPv4 with the opt-in RFC UDP
 * checksum, IPv6 (udp_csum6); the batch-host hook with in-place writes; and
 * the same calls served by resident workgroups (xcsum_ctx_set_resident).
 *
 * usage: umem_ring [--bench [B1,B2,...]]     exit 0 ok, 1 failure, 77 no GPU
 *   --bench: MTU frames per variant in batches of B (default 4096; 1M frames
 *   for B >= 1024, fewer for smaller batches), payloads written on a frame's
 *   first use only, every 64th frame checked by the NIC thread (all are
 *   checked for order): the producer loop's own rate.  Small B shows the
 *   fixed cost of one call (libxudp's tx_batch_num is 100, xudp.c:74).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "harness.h"
#include "xudp_packet.h"

#define FRAME_SIZE 4096u
#define DATA_OFF 384u          /* 64 frame info + 256 headroom + 64 XUDP_TX_HEADROOM */
#define RING_SIZE 8192u        /* power of two, like the kernel's rings */

/* An AF_XDP-style single-producer single-consumer ring (queue.h:60-110). */
struct ring {
	_Atomic uint32_t producer;
	_Atomic uint32_t consumer;
	uint32_t cached_prod;      /* producer side only */
	uint32_t cached_cons;      /* consumer side only */
	struct xcsum_desc desc[RING_SIZE];
};

/* completion ring: frame addresses back to the producer (the CQ) */
struct cring {
	_Atomic uint32_t producer;
	_Atomic uint32_t consumer;
	uint32_t cached_prod, cached_cons;
	uint64_t addr[RING_SIZE];
};

struct variant {
	const char *name;
	int family;            /* 4 or 6 */
	uint32_t pkt_flags;    /* xudp_packet_udp_batch flags (XCSUM_F_V4_RFC) */
	int registered;
	int zerocopy;
	int batch_host;        /* header build + xcsum_batch_host(INPLACE|IPHDR) */
	int resident;          /* xcsum_ctx_set_resident workgroups (0: launches) */
};

struct run {
	const struct variant *v;
	uint8_t *umem;
	uint32_t nframes;
	struct ring tx;
	struct cring cq;
	uint64_t total;            /* frames to send */
	_Atomic int done;
	uint64_t seen, bad, bad_order;
	uint32_t pmin, pmax;
	uint32_t verify_every;     /* the NIC checks every n-th frame (1: all) */
	int fill_once;             /* bench: payload bytes written on a frame's first use */
};

static uint64_t rng_next(uint64_t *s)
{
	uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

static double now_s(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* the NIC side: dequeue, check the frame as it would go on the wire, and
 * complete it */
static void *nic_main(void *arg)
{
	struct run *r = arg;
	uint8_t scratch[FRAME_SIZE];
	uint64_t expect_seq = 0;
	for (;;) {
		const uint32_t prod = atomic_load_explicit(&r->tx.producer, memory_order_acquire);
		if (prod == r->tx.cached_cons) {
			if (atomic_load_explicit(&r->done, memory_order_acquire) &&
			    prod == atomic_load_explicit(&r->tx.producer, memory_order_acquire))
				break;
			continue;
		}
		while (r->tx.cached_cons != prod) {
			const struct xcsum_desc d = r->tx.desc[r->tx.cached_cons & (RING_SIZE - 1)];
			r->tx.cached_cons++;
			const uint8_t *eth = r->umem + d.addr;
			const int v6 = r->v->family == 6;
			const uint32_t hdr = v6 ? 62 : 42;
			int ok = d.len >= hdr && d.len <= FRAME_SIZE;
			const int check = r->seen % r->verify_every == 0;
			if (ok && d.len >= hdr + 8) {
				uint64_t seq;
				memcpy(&seq, eth + hdr, sizeof(seq));
				if (seq != expect_seq)
					r->bad_order++;
			}
			expect_seq++;
			if (ok && check) {
				memcpy(scratch, eth, d.len);
				struct xcsum_desc z = {0, d.len, 0};
				uint16_t want = 0, have;
				if (v6) {
					memcpy(&have, eth + 60, 2);
					scratch[60] = scratch[61] = 0;
					orc_batch(scratch, &z, 1, &want, XCSUM_MODE_V6, 0);
				} else {
					uint16_t ipc;
					memcpy(&ipc, eth + 24, 2);
					ok &= ipc == orc_ip_header_rfc(eth + 14);
					memcpy(&have, eth + 40, 2);
					scratch[40] = scratch[41] = 0;
					if (r->v->pkt_flags & XCSUM_F_V4_RFC)
						orc_batch(scratch, &z, 1, &want, XCSUM_MODE_V4_RFC, 0);
				}
				ok &= have == want;
			}
			r->seen++;
			r->bad += !ok;
			/* transmit done: hand the frame back (queue.h:90-94 order) */
			const uint64_t fa = d.addr & ~(uint64_t)(FRAME_SIZE - 1);
			r->cq.addr[r->cq.cached_prod++ & (RING_SIZE - 1)] = fa;
			atomic_store_explicit(&r->cq.producer, r->cq.cached_prod, memory_order_release);
		}
		atomic_store_explicit(&r->tx.consumer, r->tx.cached_cons, memory_order_release);
	}
	return NULL;
}

/* one variant: returns 0 ok; *secs = producer wall time */
static int run_variant(xcsum_ctx *ctx, struct run *r, uint32_t batch, double *secs,
		       double *csum_secs)
{
	const struct variant *v = r->v;
	uint8_t dmac[6] = {2, 0, 0, 0, 0, 2}, smac[6] = {2, 0, 0, 0, 0, 1};
	struct sockaddr_in to4 = {0}, from4 = {0};
	struct sockaddr_in6 to6 = {0}, from6 = {0};
	to4.sin_family = from4.sin_family = AF_INET;
	to4.sin_port = htons(40000);
	from4.sin_port = htons(3486);
	inet_pton(AF_INET, "10.0.35.1", &to4.sin_addr);
	inet_pton(AF_INET, "10.0.35.2", &from4.sin_addr);
	to6.sin6_family = from6.sin6_family = AF_INET6;
	to6.sin6_port = htons(40000);
	from6.sin6_port = htons(3487);
	inet_pton(AF_INET6, "1000:2000:3000:4000::1", &to6.sin6_addr);
	inet_pton(AF_INET6, "1000:2000:3000:4000::2", &from6.sin6_addr);

	uint64_t *freelist = malloc(r->nframes * sizeof(uint64_t));
	uint8_t *filled = calloc(r->nframes, 1);
	uint32_t nfree = r->nframes;
	for (uint32_t i = 0; i < r->nframes; i++)
		freelist[i] = (uint64_t)i * FRAME_SIZE;
	struct packet_info *infos = calloc(batch, sizeof(*infos));
	struct xcsum_desc *descs = calloc(batch, sizeof(*descs));
	uint16_t *res = calloc(batch, sizeof(uint16_t));
	uint64_t seed = 0x75646d70 ^ (uint64_t)v->family, seq = 0;
	int rc = 0;

	pthread_t nic;
	atomic_store(&r->done, 0);
	if (pthread_create(&nic, NULL, nic_main, r) != 0)
		return -1;
	const double t0 = now_s();
	double tc = 0;
	for (uint64_t sent = 0; sent < r->total && !rc;) {
		/* reclaim completed frames (cq_deq) */
		const uint32_t cp = atomic_load_explicit(&r->cq.producer, memory_order_acquire);
		while (r->cq.cached_cons != cp)
			freelist[nfree++] = r->cq.addr[r->cq.cached_cons++ & (RING_SIZE - 1)];
		atomic_store_explicit(&r->cq.consumer, r->cq.cached_cons, memory_order_release);
		/* room in the TX ring (ring_free, queue.h:60-71) */
		const uint32_t cons = atomic_load_explicit(&r->tx.consumer, memory_order_acquire);
		uint32_t room = RING_SIZE - (r->tx.cached_prod - cons);
		uint32_t b = batch;
		if (b > nfree) b = nfree;
		if (b > room) b = room;
		if ((uint64_t)b > r->total - sent) b = (uint32_t)(r->total - sent);
		if (b == 0)
			continue;
		/* the application writes its payloads into the frames it got from
		 * xudp_frame_alloc (tx.c:760), then xudp_frame_send */
		for (uint32_t i = 0; i < b; i++) {
			uint8_t *f = r->umem + freelist[nfree - 1 - i];
			uint32_t len = r->pmin + (r->pmax > r->pmin ?
				(uint32_t)(rng_next(&seed) % (r->pmax - r->pmin + 1)) : 0);
			uint8_t *p = f + DATA_OFF;
			const uint64_t fi = (uint64_t)(f - r->umem) / FRAME_SIZE;
			for (uint32_t q = 0; q < len && !(r->fill_once && filled[fi]); q += 8) {
				uint64_t w = rng_next(&seed);
				memcpy(p + q, &w, len - q < 8 ? len - q : 8);
			}
			filled[fi] = 1;
			if (len >= 8) {
				uint64_t s = seq + i;
				memcpy(p, &s, 8);
			}
			struct packet_info *in = &infos[i];
			memset(in, 0, sizeof(*in));
			in->family = v->family == 6 ? AF_INET6 : AF_INET;
			in->dmac = dmac;
			in->smac = smac;
			if (v->family == 6) {
				in->to6 = &to6;
				in->from6 = &from6;
			} else {
				in->to = &to4;
				in->from = &from4;
			}
			in->head = (char *)f + 320;
			in->data = (char *)p;
			in->payload_size = (int)len;
		}
		const double tb = now_s();
		if (v->batch_host) {
			/* headers on the host, one in-place
			 * checksum batch over the registered UMEM */
			for (uint32_t i = 0; i < b; i++) {
				xudp_packet_build_headers(&infos[i]);
				descs[i].addr = (uint64_t)((uint8_t *)infos[i].packet - r->umem);
				descs[i].len = (uint32_t)infos[i].len;
				descs[i].options = 0;
			}
			const uint32_t mode = v->family == 6 ? XCSUM_MODE_V6 : XCSUM_MODE_V4_RFC;
			rc = xcsum_batch_host(ctx, r->umem, descs, b, res, mode,
					      XCSUM_F_INPLACE | XCSUM_F_IPHDR |
					      (v->zerocopy ? XCSUM_F_ZEROCOPY : 0));
		} else {
			rc = xudp_packet_udp_batch(ctx, infos, b,
						   v->pkt_flags | (v->zerocopy ? XCSUM_F_ZEROCOPY : 0));
		}
		tc += now_s() - tb;
		if (rc) {
			fprintf(stderr, "%s: checksum call failed: %d\n", v->name, rc);
			break;
		}
		/* xq_enq: descriptors, then the producer index (release) */
		for (uint32_t i = 0; i < b; i++) {
			struct xcsum_desc *d = &r->tx.desc[r->tx.cached_prod++ & (RING_SIZE - 1)];
			d->addr = (uint64_t)((uint8_t *)infos[i].packet - r->umem);
			d->len = (uint32_t)infos[i].len;
			d->options = 0;
		}
		atomic_store_explicit(&r->tx.producer, r->tx.cached_prod, memory_order_release);
		nfree -= b;
		sent += b;
		seq += b;
	}
	atomic_store_explicit(&r->done, 1, memory_order_release);
	pthread_join(nic, NULL);
	*secs = now_s() - t0;
	*csum_secs = tc;
	free(freelist);
	free(filled);
	free(infos);
	free(descs);
	free(res);
	return rc;
}

int main(int argc, char **argv)
{
	const int bench = argc > 1 && strcmp(argv[1], "--bench") == 0;
	uint32_t batches[16] = {4096u};
	int nbatch = 1;
	if (bench && argc > 2) {
		nbatch = 0;
		for (char *t = strtok(argv[2], ","); t && nbatch < 16; t = strtok(NULL, ","))
			if (atoi(t) > 0)
				batches[nbatch++] = (uint32_t)atoi(t);
		if (!nbatch)
			batches[nbatch++] = 4096u;
	}
	xcsum_ctx *ctx = NULL;
	int rc = xcsum_ctx_create(-1, &ctx);
	if (rc == -XCSUM_ERR_NODEV) {
		printf("umem_ring: no GPU, skipped\n");
		return 77;
	}
	if (rc) {
		fprintf(stderr, "xcsum_ctx_create: %d\n", rc);
		return 1;
	}
	const uint32_t nframes = 16384;                /* 64 MiB of UMEM */
	const size_t bytes = (size_t)nframes * FRAME_SIZE;
	int locked = 0;
	uint8_t *umem = xudp_anon_map(bytes, &locked);
	CHECK(umem != NULL, "anon_map");
	if (!umem)
		return 1;
	printf("umem_ring: UMEM %zu bytes by anon_map (MAP_LOCKED %s)\n", bytes,
	       locked ? "granted" : "refused, mapped without it");
	static const struct variant vars[] = {
		{"v4 staged", 4, 0, 0, 0, 0, 0},
		{"v4 registered", 4, 0, 1, 0, 0, 0},
		{"v4 zero-copy", 4, 0, 1, 1, 0, 0},
		{"v4+rfc staged", 4, XCSUM_F_V4_RFC, 0, 0, 0, 0},
		{"v4+rfc registered", 4, XCSUM_F_V4_RFC, 1, 0, 0, 0},
		{"v4+rfc zero-copy", 4, XCSUM_F_V4_RFC, 1, 1, 0, 0},
		{"v6 staged", 6, 0, 0, 0, 0, 0},
		{"v6 registered", 6, 0, 1, 0, 0, 0},
		{"v6 zero-copy", 6, 0, 1, 1, 0, 0},
		{"v4 batch_host in place, registered", 4, XCSUM_F_V4_RFC, 1, 0, 1, 0},
		{"v4 batch_host in place, zero-copy", 4, XCSUM_F_V4_RFC, 1, 1, 1, 0},
		{"v6 batch_host in place, zero-copy", 6, 0, 1, 1, 1, 0},
		/* resident workgroups instead of a launch per batch */
		{"v4 registered, resident", 4, 0, 1, 0, 0, 8},
		{"v4+rfc registered, resident", 4, XCSUM_F_V4_RFC, 1, 0, 0, 8},
		{"v6 staged, resident", 6, 0, 0, 0, 0, 8},
		{"v6 registered, resident", 6, 0, 1, 0, 0, 8},
		{"v4 batch_host in place, registered, resident", 4, XCSUM_F_V4_RFC, 1, 0, 1, 8},
		{"v6 batch_host in place, registered, resident", 6, 0, 1, 0, 1, 8},
	};
	struct run *r = calloc(1, sizeof(*r));
	for (size_t k = 0; k < sizeof(vars) / sizeof(vars[0]); k++) {
		const struct variant *v = &vars[k];
		if (v->registered)
			CHECK(xcsum_register_umem(ctx, umem, bytes) == 0, "%s: register", v->name);
		/* $RING_RESIDENT_WG overrides the resident variants' workgroup count */
		const char *rw = getenv("RING_RESIDENT_WG");
		const int wg = v->resident && rw ? atoi(rw) : v->resident;
		CHECK(xcsum_ctx_set_resident(ctx, wg, 0) == 0, "%s: resident", v->name);
		for (int pass = bench; pass < (bench ? 1 + nbatch : 1); pass++) {
			/* tx_batch_num is 100 (xudp.c:74); the bench batches as asked */
			const uint32_t batch = pass ? batches[pass - 1] : 100u;
			memset(r, 0, sizeof(*r));
			r->v = v;
			r->umem = umem;
			r->nframes = nframes;
			/* correctness: ragged sizes; bench: MTU payloads */
			r->pmin = pass ? 1472u - (v->family == 6 ? 20u : 0u) : 0u;
			r->pmax = pass ? r->pmin : 1438u;
			r->total = !pass ? 40000u : batch >= 1024u ? 1048576u
				 : batch >= 64u ? 262144u : 16384u * batch;
			r->verify_every = pass ? 64u : 1u;
			r->fill_once = pass;
			double secs = 0, csecs = 0;
			int e = run_variant(ctx, r, batch, &secs, &csecs);
			CHECK(e == 0, "%s: run failed", v->name);
			CHECK(r->seen == r->total, "%s: NIC saw %llu of %llu frames", v->name,
			      (unsigned long long)r->seen, (unsigned long long)r->total);
			CHECK(r->bad == 0, "%s: %llu frames wrong on the wire", v->name,
			      (unsigned long long)r->bad);
			CHECK(r->bad_order == 0, "%s: %llu frames out of order", v->name,
			      (unsigned long long)r->bad_order);
			const double fb = (double)(r->pmin + (v->family == 6 ? 62 : 42));
			if (pass)
				printf("{\"variant\": \"%s\", \"frames\": %llu, \"batch\": %u, "
				       "\"frame_bytes\": %.0f, \"wall_s\": %.4f, \"mpps\": %.3f, "
				       "\"frames_GBps\": %.3f, \"checksum_call_s\": %.4f, "
				       "\"checksum_call_GBps\": %.3f, \"us_per_call\": %.2f}\n",
				       v->name, (unsigned long long)r->total, batch, fb, secs,
				       r->total / secs / 1e6, r->total * fb / secs / 1e9, csecs,
				       r->total * fb / csecs / 1e9, csecs * 1e6 * batch / r->total);
		}
		if (v->registered)
			CHECK(xcsum_unregister_umem(ctx, umem) == 0, "%s: unregister", v->name);
	}
	free(r);
	munmap(umem, bytes);
	xcsum_ctx_destroy(ctx);
	printf("umem_ring: %d checks, %d failures\n", checks, failures);
	return failures ? 1 : 0;
}
