/*
 * capi_check.c -- the C ABI used from plain C11, the way libxudp (a C
 * library) would link it: include/xcsum.h + include/xudp_packet.h, -lxcsum.
 * Test infrastructure: expected checksums come from the oracle restatement
 * (oracle/liboracle.so, pinned to the reference by tests/test_oracle.py) and
 * from the reference's known-answer frames.
 *
 * Also the process model libxudp runs in:
 *   - fork() before any HIP call (the master/worker model forks its workers,
 *     test/case/lib.c:169); each child initialises HIP lazily through its own
 *     context and checks a batch;
 *   - two host threads, each with its own context and stream on device 0
 *     (and later its own resident workgroups),
 *     running concurrently (one TX channel per thread, xudp/xsk.c:303-304);
 *   - eight group threads (libxudp's group_num groups, test/case/lib.c:196-221)
 *     creating contexts under each device placement policy (AUTO round
 *     robin, XCSUM_DEVICE_GROUP, the thread's default context via
 *     xcsum_thread_init) and checking a batch on each;
 *   - the UMEM allocated exactly as xudp does (anon_map, include/common.h:37-41,
 *     xudp/xsk.c:234), registered, checksummed staged / zero-copy / in place.
 *
 * Exit 0 = all checks passed, 77 = no GPU (skip), 1 = a check failed.
 * `capi_check --threads` runs only the thread test (the TSan build,
 * tests/c/Makefile `tsan`).  Run by tests/test_capi.py on the GPU box.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "harness.h"
#include "xudp_packet.h"

static int hex_eq(const uint8_t *p, const char *hex)
{
	size_t n = strlen(hex) / 2;
	for (size_t i = 0; i < n; i++) {
		unsigned v;
		if (sscanf(hex + 2 * i, "%2x", &v) != 1 || p[i] != (uint8_t)v)
			return 0;
	}
	return 1;
}

/* Host-resident batches (xcsum_batch_host) and the device path
 * (xcsum_batch_device on hipMalloc'ed frames) against the oracle. */
static void check_batches(xcsum_ctx *c, uint32_t family, uint32_t stride, uint32_t offset,
			  int xudp_map)
{
	const uint32_t n = 4000;
	struct xcsum_desc *desc = calloc(n, sizeof(*desc));
	uint64_t bytes = 0;
	CHECK(xcsum_gen_layout(n, family, 0, 3000, 7 + family, 0, 8, stride, offset, desc,
			       &bytes) == 0, "gen_layout");
	/* xudp_map: the UMEM as xudp maps it (anon_map), else the C heap */
	int locked = 0;
	const size_t map_bytes = (bytes + 64 + 4095) & ~(size_t)4095;
	uint8_t *umem = xudp_map ? xudp_anon_map(map_bytes, &locked) : calloc(bytes + 64, 1);
	CHECK(umem != NULL, "umem allocation");
	if (!umem)
		return;
	CHECK(xcsum_gen_fill_host(umem, desc, n, family, 7 + family, 0) == 0, "gen_fill_host");
	uint16_t *exp = calloc(n, 2), *got = calloc(n, 2);
	const uint32_t mode = family == 6 ? XCSUM_MODE_V6 : XCSUM_MODE_V4_LEGACY;
	orc_batch(umem, desc, n, exp, (int)mode, 0);

	/* staged copies */
	CHECK(xcsum_batch_host(c, umem, desc, n, got, mode, 0) == 0, "batch_host");
	CHECK(count_diff(got, exp, n) == 0, "batch_host v%u: %u mismatches", family,
	      count_diff(got, exp, n));

	/* registered UMEM: staged copies through the pinned mapping ... */
	CHECK(xcsum_register_umem(c, umem, bytes + 64) == 0, "register_umem");
	memset(got, 0, 2 * n);
	CHECK(xcsum_batch_host(c, umem, desc, n, got, mode, 0) == 0, "batch_host registered");
	CHECK(count_diff(got, exp, n) == 0, "registered v%u: %u mismatches", family,
	      count_diff(got, exp, n));
	/* ... and zero-copy, results written into the frames */
	memset(got, 0, 2 * n);
	CHECK(xcsum_batch_host(c, umem, desc, n, got, mode, XCSUM_F_ZEROCOPY | XCSUM_F_INPLACE) ==
	      0, "batch_host zerocopy");
	CHECK(count_diff(got, exp, n) == 0, "zerocopy v%u", family);
	uint32_t bad = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint16_t v;
		memcpy(&v, umem + desc[i].addr + (family == 6 ? 60 : 40), 2);
		bad += v != exp[i];
	}
	CHECK(bad == 0, "in-place udp->check v%u: %u wrong", family, bad);
	if (family == 4) {
		/* libxudp's IPv4 call: iph->check alone (XCSUM_F_IPHDR_ONLY), read
		 * in place from the UMEM when the GPU maps it, else gathered */
		uint16_t *exp_ip = calloc(n, 2);
		orc_batch(umem, desc, n, exp_ip, XCSUM_MODE_V4_LEGACY, (int)XCSUM_F_IPHDR_ONLY);
		memset(got, 0, 2 * n);
		CHECK(xcsum_batch_host(c, umem, desc, n, got, XCSUM_MODE_V4_LEGACY,
				       XCSUM_F_IPHDR_ONLY | XCSUM_F_INPLACE) == 0, "batch_host iphdr only");
		CHECK(count_diff(got, exp_ip, n) == 0, "iphdr only: %u mismatches",
		      count_diff(got, exp_ip, n));
		bad = 0;
		for (uint32_t i = 0; i < n; i++) {
			uint16_t v;
			memcpy(&v, umem + desc[i].addr + 24, 2);
			bad += v != exp_ip[i];
		}
		CHECK(bad == 0, "in-place iph->check: %u wrong", bad);
		free(exp_ip);
	}
	CHECK(xcsum_unregister_umem(c, umem) == 0, "unregister_umem");

	/* receive side on the host frames: write RFC checksums (and the IPv4
	 * header's), then every frame must parse and verify; one flipped
	 * payload byte fails exactly that frame */
	const uint32_t rfc = family == 6 ? XCSUM_MODE_V6 : XCSUM_MODE_V4_RFC;
	for (uint32_t i = 0; i < n; i++)   /* the pass above wrote udp->check */
		memset(umem + desc[i].addr + (family == 6 ? 60 : 40), 0, 2);
	CHECK(xcsum_batch_host(c, umem, desc, n, got, rfc, XCSUM_F_INPLACE | XCSUM_F_IPHDR) == 0,
	      "batch_host rfc in place");
	struct xcsum_rx_msg *msgs = calloc(n, sizeof(*msgs));
	uint32_t count = 0;
	const uint32_t hdr = family == 6 ? 62 : 42;
	CHECK(xcsum_rx_host(c, umem, desc, n, msgs, &count, XCSUM_F_VERIFY | XCSUM_F_IPHDR) == 0,
	      "rx_host");
	CHECK(count == n, "rx_host v%u: %u of %u delivered", family, count, n);
	bad = 0;
	for (uint32_t i = 0; i < n; i++)
		bad += msgs[i].status != XCSUM_RX_OK || msgs[i].family != family ||
		       msgs[i].frame != desc[i].addr || msgs[i].body != desc[i].addr + hdr ||
		       msgs[i].size != desc[i].len - hdr;
	CHECK(bad == 0, "rx_host v%u: %u wrong records", family, bad);
	umem[desc[n / 2].addr + desc[n / 2].len - 1] ^= 0x40;
	CHECK(xcsum_rx_host(c, umem, desc, n, msgs, &count, XCSUM_F_VERIFY) == 0, "rx_host 2");
	CHECK(count == n - 1 && msgs[n / 2].status == XCSUM_RX_CSUM, "rx_host v%u: corrupted frame",
	      family);
	free(msgs);

	/* device-resident: the frames as xudp would have them in HBM */
	uint8_t *d_umem = NULL;
	struct xcsum_desc *d_desc = NULL;
	uint16_t *d_out = NULL;
	CHECK(hipMalloc((void **)&d_umem, bytes + 64) == hipSuccess, "hipMalloc");
	CHECK(hipMalloc((void **)&d_desc, n * sizeof(*desc)) == hipSuccess, "hipMalloc");
	CHECK(hipMalloc((void **)&d_out, 2 * n) == hipSuccess, "hipMalloc");
	CHECK(xcsum_gen_fill_device(d_umem, NULL, 0, family, 0, 0, NULL) == 0, "fill n=0");
	(void)hipMemcpy(d_desc, desc, n * sizeof(*desc), hipMemcpyHostToDevice);
	CHECK(xcsum_gen_fill_device(d_umem, d_desc, n, family, 7 + family, 0, NULL) == 0,
	      "gen_fill_device");
	CHECK(xcsum_batch_device(c, d_umem, d_desc, n, d_out, mode, 0, 0, NULL) == 0,
	      "batch_device");
	CHECK(xcsum_sync(c, NULL) == 0, "sync");
	memset(got, 0, 2 * n);
	(void)hipMemcpy(got, d_out, 2 * n, hipMemcpyDeviceToHost);
	CHECK(count_diff(got, exp, n) == 0, "batch_device v%u: %u mismatches", family,
	      count_diff(got, exp, n));
	/* descriptor order must not matter */
	CHECK(xcsum_ctx_set_order(c, 3, 2) == 0, "set_order");
	CHECK(xcsum_batch_device(c, d_umem, d_desc, n, d_out, mode, 0, 1500, NULL) == 0,
	      "batch_device ordered");
	(void)hipMemcpy(got, d_out, 2 * n, hipMemcpyDeviceToHost);
	CHECK(count_diff(got, exp, n) == 0, "batch_device ordered v%u", family);
	CHECK(xcsum_ctx_set_order(c, -1, 0) == 0, "set_order auto");
	(void)hipFree(d_umem);
	(void)hipFree(d_desc);
	(void)hipFree(d_out);
	free(desc);
	if (xudp_map)
		munmap(umem, map_bytes);
	else
		free(umem);
	free(exp);
	free(got);
}

/* frames xudp_packet_udp_payload() builds
 * in the reference, byte for byte. */
static void check_packet_kats(void)
{
	unsigned char dmac[6] = {2, 0, 0, 0, 0, 2}, smac[6] = {2, 0, 0, 0, 0, 1};
	char buf[256];
	struct sockaddr_in to4 = {0}, from4 = {0};
	to4.sin_family = from4.sin_family = AF_INET;
	to4.sin_port = htons(40000);
	from4.sin_port = htons(3486);
	inet_pton(AF_INET, "10.0.35.1", &to4.sin_addr);
	inet_pton(AF_INET, "10.0.35.2", &from4.sin_addr);
	struct packet_info info;
	memset(&info, 0, sizeof(info));
	memset(buf, 0, sizeof(buf));
	info.family = AF_INET;
	info.dmac = dmac;
	info.smac = smac;
	info.to = &to4;
	info.from = &from4;
	info.head = buf;
	info.payload = "abcdef";
	info.payload_size = 6;
	xudp_packet_udp_payload(&info);
	CHECK(info.len == 48, "KAT4 len %d", info.len);
	CHECK(hex_eq((uint8_t *)info.packet,
		     "020000000002020000000001080045000022000040004011e0c80a0023020a0023010d9e"
		     "9c40000e0000616263646566"),
	      "KAT4 frame bytes");

	struct sockaddr_in6 to6 = {0}, from6 = {0};
	to6.sin6_family = from6.sin6_family = AF_INET6;
	to6.sin6_port = htons(40000);
	from6.sin6_port = htons(3487);
	inet_pton(AF_INET6, "1000:2000:3000:4000::1", &to6.sin6_addr);
	inet_pton(AF_INET6, "1000:2000:3000:4000::2", &from6.sin6_addr);
	memset(&info, 0, sizeof(info));
	memset(buf, 0, sizeof(buf));
	info.family = AF_INET6;
	info.dmac = dmac;
	info.smac = smac;
	info.to6 = &to6;
	info.from6 = &from6;
	info.head = buf;
	info.payload = "abcdef";
	info.payload_size = 6;
	xudp_packet_udp_payload(&info);
	CHECK(info.len == 68, "KAT3 len %d", info.len);
	CHECK(hex_eq((uint8_t *)info.packet,
		     "02000000000202000000000186dd60039f0d000e11401000200030004000000000000000"
		     "0002100020003000400000000000000000010d9f9c40000eebc1616263646566"),
	      "KAT3 frame bytes");
}

static void check_errors(xcsum_ctx *c)
{
	CHECK(xcsum_batch_device(NULL, NULL, NULL, 1, NULL, 0, 0, 0, NULL) == -XCSUM_ERR_INVAL,
	      "null ctx");
	CHECK(xcsum_batch_device(c, NULL, NULL, 5, NULL, 0, 0, 0, NULL) == -XCSUM_ERR_INVAL,
	      "null buffers");
	CHECK(xcsum_batch_device(c, NULL, NULL, 0, NULL, 0, 0, 0, NULL) == 0, "empty batch");
	CHECK(xcsum_ctx_set_geometry(c, 7, 1, 1) == -XCSUM_ERR_INVAL, "bad geometry");
	CHECK(xcsum_ctx_set_order(c, 13, 0) == -XCSUM_ERR_INVAL, "bad order");
	CHECK(xcsum_unregister_umem(c, (void *)0x1000) == -XCSUM_ERR_NOT_REGISTERED,
	      "unregister unknown");
	uint64_t e = 99;
	CHECK(xcsum_ctx_take_errors(c, &e) == 0 && e == 0, "error counter %llu",
	      (unsigned long long)e);
}

/* ---- fork: HIP initialised lazily, after fork, in each child ------------- */

/* one small batch through a fresh context, checked against the oracle;
 * returns the exit status for a child: 0 ok, 1 mismatch, 77 no GPU */
static int child_batch(uint32_t family, uint64_t seed)
{
	xcsum_ctx *c = NULL;
	int rc = xcsum_ctx_create(-1, &c);
	if (rc == -XCSUM_ERR_NODEV)
		return 77;
	if (rc)
		return 1;
	const uint32_t n = 1500;
	struct xcsum_desc *desc = calloc(n, sizeof(*desc));
	uint64_t bytes = 0;
	int ok = xcsum_gen_layout(n, family, 0, 1500, seed, 0, 8, 0, 0, desc, &bytes) == 0;
	uint8_t *umem = calloc(bytes + 64, 1);
	ok &= xcsum_gen_fill_host(umem, desc, n, family, seed, 0) == 0;
	uint16_t *exp = calloc(n, 2), *got = calloc(n, 2);
	const int mode = family == 6 ? XCSUM_MODE_V6 : XCSUM_MODE_V4_LEGACY;
	orc_batch(umem, desc, n, exp, mode, 0);
	ok &= xcsum_batch_host(c, umem, desc, n, got, (uint32_t)mode, 0) == 0;
	ok &= count_diff(got, exp, n) == 0;
	xcsum_ctx_destroy(c);
	free(desc);
	free(umem);
	free(exp);
	free(got);
	return ok ? 0 : 1;
}

/* Called first in main(), before this process has made any HIP call: two
 * workers forked like libxudp's (test/case/lib.c:169), both checksumming at
 * once; the parent initialises HIP only after they are done.  Returns 77
 * when no child found a GPU. */
static int check_fork(void)
{
	pid_t pid[2];
	for (int k = 0; k < 2; k++) {
		fflush(NULL);
		pid[k] = fork();
		if (pid[k] == 0)
			exit(child_batch(k ? 6 : 4, 100 + (uint64_t)k));
		CHECK(pid[k] > 0, "fork");
	}
	int nodev = 0;
	for (int k = 0; k < 2; k++) {
		int st = 0;
		if (pid[k] <= 0)
			continue;
		CHECK(waitpid(pid[k], &st, 0) == pid[k], "waitpid");
		CHECK(WIFEXITED(st), "worker %d did not exit normally (status 0x%x)", k, st);
		if (WIFEXITED(st) && WEXITSTATUS(st) == 77)
			nodev++;
		else
			CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0, "forked worker %d: status 0x%x", k,
			      st);
	}
	return nodev == 2 ? 77 : 0;
}

/* ---- two host threads, two contexts, two streams, device 0 --------------- */

struct thread_job {
	uint32_t family;
	uint64_t seed;
	int iters;
	int bad;        /* mismatching iterations */
	int err;        /* a call failed */
};

static void *thread_main(void *arg)
{
	struct thread_job *j = arg;
	xcsum_ctx *c = NULL;
	if (xcsum_ctx_create(0, &c) != 0) {
		j->err = 1;
		return NULL;
	}
	hipStream_t st = NULL;
	if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
		j->err = 1;
		xcsum_ctx_destroy(c);
		return NULL;
	}
	const uint32_t n = 20000;
	struct xcsum_desc *desc = calloc(n, sizeof(*desc));
	uint64_t bytes = 0;
	j->err |= xcsum_gen_layout(n, j->family, 0, 1472, j->seed, 0, 8, 0, 0, desc, &bytes) != 0;
	uint8_t *umem = calloc(bytes + 64, 1);
	uint16_t *exp = calloc(n, 2), *got = calloc(n, 2);
	const uint32_t mode = j->family == 6 ? XCSUM_MODE_V6 : XCSUM_MODE_V4_LEGACY;
	/* the same frames one per 4096-byte chunk (xudp's slots) in pageable
	 * memory: gathered frame by frame, the copies and the in-place stores
	 * split over the library's threads (>= 16384 frames) */
	struct xcsum_desc *sdesc = calloc(n, sizeof(*sdesc));
	uint64_t sbytes = 0;
	j->err |= xcsum_gen_layout(n, j->family, 0, 1472, j->seed, 0, 8, 4096,
				   j->family == 6 ? 322 : 342, sdesc, &sbytes) != 0;
	uint8_t *sumem = calloc(sbytes + 64, 1);
	uint16_t *sexp = calloc(n, 2);
	const uint32_t chk = j->family == 6 ? 60 : 40;
	uint8_t *d_umem = NULL;
	struct xcsum_desc *d_desc = NULL;
	uint16_t *d_out = NULL;
	j->err |= hipMalloc((void **)&d_umem, bytes + 64) != hipSuccess;
	j->err |= hipMalloc((void **)&d_desc, n * sizeof(*desc)) != hipSuccess;
	j->err |= hipMalloc((void **)&d_out, 2 * n) != hipSuccess;
	if (!j->err) {
		j->err |= hipMemcpyAsync(d_desc, desc, n * sizeof(*desc), hipMemcpyHostToDevice,
					 st) != hipSuccess;
		j->err |= xcsum_gen_fill_device(d_umem, d_desc, n, j->family, j->seed, 0, st) != 0;
		j->err |= xcsum_gen_fill_host(umem, desc, n, j->family, j->seed, 0) != 0;
		orc_batch(umem, desc, n, exp, (int)mode, 0);
		j->err |= xcsum_gen_fill_host(sumem, sdesc, n, j->family, j->seed, 0) != 0;
		orc_batch(sumem, sdesc, n, sexp, (int)mode, 0);
	}
	for (int it = 0; it < j->iters && !j->err; it++) {
		/* device-resident batch on this thread's stream ... */
		memset(got, 0, 2 * n);
		j->err |= hipMemsetAsync(d_out, 0, 2 * n, st) != hipSuccess;
		j->err |= xcsum_batch_device(c, d_umem, d_desc, n, d_out, mode, 0, 0, st) != 0;
		j->err |= hipMemcpyAsync(got, d_out, 2 * n, hipMemcpyDeviceToHost, st) != hipSuccess;
		j->err |= xcsum_sync(c, st) != 0;
		j->bad += count_diff(got, exp, n) != 0;
		/* ... and a host-resident one through the context's own staging */
		memset(got, 0, 2 * n);
		j->err |= xcsum_batch_host(c, umem, desc, n, got, mode, 0) != 0;
		j->bad += count_diff(got, exp, n) != 0;
		/* ... and the sparse frames in place (check fields zeroed after) */
		memset(got, 0, 2 * n);
		j->err |= xcsum_batch_host(c, sumem, sdesc, n, got, mode, XCSUM_F_INPLACE) != 0;
		uint32_t wrong = count_diff(got, sexp, n);
		for (uint32_t i = 0; i < n; i++) {
			uint16_t v;
			memcpy(&v, sumem + sdesc[i].addr + chk, 2);
			wrong += v != sexp[i];
			memset(sumem + sdesc[i].addr + chk, 0, 2);
		}
		j->bad += wrong != 0;
	}
	/* resident workgroups (xcsum_ctx_set_resident): both threads' servers
	 * live at once, libxudp-sized batches from different places, device
	 * batches on the thread's stream in between */
	j->err |= xcsum_ctx_set_resident(c, 8, 0) != 0;
	for (int it = 0; it < 4 * j->iters && !j->err; it++) {
		const uint32_t first = (uint32_t)(it * 997u) % (n - 100);
		memset(got, 0, 2 * 100);
		j->err |= xcsum_batch_host(c, umem, desc + first, 100, got, mode, 0) != 0;
		j->bad += count_diff(got, exp + first, 100) != 0;
		if (it % 8 == 7) {
			j->err |= xcsum_batch_device(c, d_umem, d_desc, n, d_out, mode, 0, 0, st) != 0;
			j->err |= xcsum_sync(c, st) != 0;
		}
	}
	(void)hipFree(d_umem);
	(void)hipFree(d_desc);
	(void)hipFree(d_out);
	(void)hipStreamDestroy(st);
	xcsum_ctx_destroy(c);
	free(desc);
	free(umem);
	free(exp);
	free(got);
	free(sdesc);
	free(sumem);
	free(sexp);
	return NULL;
}

static void check_threads(void)
{
	struct thread_job jobs[2] = {{4, 31, 25, 0, 0}, {6, 32, 25, 0, 0}};
	pthread_t th[2];
	for (int k = 0; k < 2; k++)
		CHECK(pthread_create(&th[k], NULL, thread_main, &jobs[k]) == 0, "pthread_create");
	for (int k = 0; k < 2; k++) {
		pthread_join(th[k], NULL);
		CHECK(!jobs[k].err, "thread %d: a call failed", k);
		CHECK(jobs[k].bad == 0, "thread %d: %d of %d iterations mismatched", k, jobs[k].bad,
		      3 * jobs[k].iters);
	}
}

/* ---- placement: 8 group threads, contexts under each policy ------------ */

struct place_job {
	int gid, ndev;
	int dev_auto, dev_group, dev_thread;
	int bad, err;
};

/* one 2000-frame host batch through ctx against the oracle */
static int place_batch(xcsum_ctx *c, uint32_t family, uint64_t seed)
{
	const uint32_t n = 2000;
	struct xcsum_desc *desc = calloc(n, sizeof(*desc));
	uint64_t bytes = 0;
	int bad = xcsum_gen_layout(n, family, 0, 1472, seed, 0, 8, 0, 0, desc, &bytes) != 0;
	uint8_t *umem = calloc(bytes + 64, 1);
	uint16_t *exp = calloc(n, 2), *got = calloc(n, 2);
	const int mode = family == 6 ? XCSUM_MODE_V6 : XCSUM_MODE_V4_LEGACY;
	bad |= xcsum_gen_fill_host(umem, desc, n, family, seed, 0) != 0;
	orc_batch(umem, desc, n, exp, mode, 0);
	bad |= xcsum_batch_host(c, umem, desc, n, got, (uint32_t)mode, 0) != 0;
	bad |= count_diff(got, exp, n) != 0;
	free(desc);
	free(umem);
	free(exp);
	free(got);
	return bad;
}

static void *place_main(void *arg)
{
	struct place_job *j = arg;
	xcsum_ctx *a = NULL, *g = NULL;
	/* XCSUM_DEVICE_AUTO: the process's round robin */
	if (xcsum_ctx_create(XCSUM_DEVICE_AUTO, &a) != 0) {
		j->err = 1;
		return NULL;
	}
	j->dev_auto = xcsum_ctx_device(a);
	j->bad += place_batch(a, 4, 500 + (uint64_t)j->gid);
	/* the group's own device, gid mod the device count */
	if (xcsum_ctx_create_for_group(j->gid, &g) != 0) {
		j->err = 1;
		xcsum_ctx_destroy(a);
		return NULL;
	}
	j->dev_group = xcsum_ctx_device(g);
	j->bad += place_batch(g, 6, 600 + (uint64_t)j->gid);
	/* the thread's default context (the packet.c mirrors'), placed at the
	 * worker's start-up */
	if (xcsum_thread_init(j->gid) != 0 || !xcsum_thread_ctx()) {
		j->err = 1;
	} else {
		j->dev_thread = xcsum_ctx_device(xcsum_thread_ctx());
		j->bad += place_batch(xcsum_thread_ctx(), 4, 700 + (uint64_t)j->gid);
	}
	xcsum_ctx_destroy(a);
	xcsum_ctx_destroy(g);
	return NULL;
}

static void check_placement(void)
{
	const int ndev = xcsum_device_count();
	CHECK(ndev >= 1, "xcsum_device_count %d", ndev);
	if (ndev < 1)
		return;
	struct place_job jobs[8];
	pthread_t th[8];
	for (int k = 0; k < 8; k++) {
		memset(&jobs[k], 0, sizeof(jobs[k]));
		jobs[k].gid = k;
		jobs[k].ndev = ndev;
		CHECK(pthread_create(&th[k], NULL, place_main, &jobs[k]) == 0, "pthread_create");
	}
	int per_dev[64] = {0};
	for (int k = 0; k < 8; k++) {
		pthread_join(th[k], NULL);
		CHECK(!jobs[k].err, "placement thread %d: a call failed", k);
		CHECK(jobs[k].bad == 0, "placement thread %d: %d batches mismatched", k, jobs[k].bad);
		CHECK(jobs[k].dev_group == k % ndev, "group %d on device %d, want %d", k,
		      jobs[k].dev_group, k % ndev);
		CHECK(jobs[k].dev_thread == k % ndev, "group %d default context on device %d", k,
		      jobs[k].dev_thread);
		CHECK(jobs[k].dev_auto >= 0 && jobs[k].dev_auto < ndev, "auto device %d",
		      jobs[k].dev_auto);
		if (jobs[k].dev_auto >= 0 && jobs[k].dev_auto < 64)
			per_dev[jobs[k].dev_auto]++;
	}
	/* 8 AUTO contexts over ndev devices: as even as a round robin makes them */
	for (int d = 0; d < ndev && d < 64; d++)
		CHECK(per_dev[d] >= 8 / ndev && per_dev[d] <= (8 + ndev - 1) / ndev,
		      "device %d got %d of 8 AUTO contexts", d, per_dev[d]);
	printf("capi_check: placement over %d device(s): 8 groups, auto/group/thread contexts ok\n",
	       ndev);
}

int main(int argc, char **argv)
{
	const int threads_only = argc > 1 && strcmp(argv[1], "--threads") == 0;
	if (!threads_only && check_fork() == 77) {
		printf("capi_check: no GPU, skipped\n");
		return 77;
	}
	xcsum_ctx *c = NULL;
	int rc = xcsum_ctx_create(-1, &c);
	if (rc == -XCSUM_ERR_NODEV) {
		printf("capi_check: no GPU, skipped\n");
		return 77;
	}
	if (rc != 0) {
		fprintf(stderr, "xcsum_ctx_create: %d\n", rc);
		return 1;
	}
	if (!threads_only) {
		check_batches(c, 4, 0, 0, 0);
		check_batches(c, 6, 0, 0, 0);
		check_batches(c, 4, 4096, 342, 0);   /* xudp TX UMEM layout, SURVEY a14 */
		check_batches(c, 4, 4096, 342, 1);   /* ... in xudp's own anon_map UMEM */
		check_batches(c, 6, 4096, 322, 1);
		check_packet_kats();
		check_errors(c);
	}
	check_threads();
	check_placement();   /* threaded too: in the TSan run as well */
	xcsum_ctx_destroy(c);
	printf("capi_check: %d checks, %d failures\n", checks, failures);
	return failures ? 1 : 0;
}
