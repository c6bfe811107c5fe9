/*
 * harness.h -- shared by the C test programs in tests/c (test infrastructure:
 * expected values come from the oracle restatement oracle/liboracle.so,
 * pinned to the reference by tests/test_oracle.py).
 */
#ifndef XCSUM_TEST_HARNESS_H
#define XCSUM_TEST_HARNESS_H

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>

#include "xcsum.h"

/* oracle/xcsum_oracle.c (struct orc_desc has the xdp_desc layout) */
void orc_batch(const uint8_t *umem, const struct xcsum_desc *desc, uint32_t n, uint16_t *out,
	       int mode, uint32_t flags);
uint16_t orc_ip_header_rfc(const uint8_t *iph);

static int failures;
static int checks;

#define CHECK(cond, ...)                                                   \
	do {                                                               \
		__atomic_add_fetch(&checks, 1, __ATOMIC_RELAXED);          \
		if (!(cond)) {                                             \
			__atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED); \
			fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
			fprintf(stderr, __VA_ARGS__);                      \
			fputc('\n', stderr);                               \
		}                                                          \
	} while (0)

static inline uint32_t count_diff(const uint16_t *a, const uint16_t *b, uint32_t n)
{
	uint32_t d = 0;
	for (uint32_t i = 0; i < n; i++)
		d += a[i] != b[i];
	return d;
}

/* xudp's UMEM allocation exactly: anon_map() of include/common.h:37-41, as
 * __umem_configure() maps the frame area (xudp/xsk.c:234).  MAP_LOCKED needs
 * RLIMIT_MEMLOCK headroom; when the kernel refuses it the map is retried
 * without MAP_LOCKED and *locked says so (the pages are still populated). */
static inline void *xudp_anon_map(size_t size, int *locked)
{
	void *p = mmap(NULL, size, PROT_READ | PROT_WRITE,
		       MAP_SHARED | MAP_ANONYMOUS | MAP_POPULATE | MAP_LOCKED, 0, 0);
	*locked = 1;
	if (p == MAP_FAILED && (errno == EAGAIN || errno == ENOMEM || errno == EPERM)) {
		struct rlimit rl = {0, 0};
		getrlimit(RLIMIT_MEMLOCK, &rl);
		fprintf(stderr, "anon_map: MAP_LOCKED refused for %zu bytes (%s, RLIMIT_MEMLOCK "
			"%llu): mapped MAP_SHARED|MAP_ANONYMOUS|MAP_POPULATE without it\n",
			size, strerror(errno), (unsigned long long)rl.rlim_cur);
		*locked = 0;
		p = mmap(NULL, size, PROT_READ | PROT_WRITE,
			 MAP_SHARED | MAP_ANONYMOUS | MAP_POPULATE, 0, 0);
	}
	return p == MAP_FAILED ? NULL : p;
}

#endif
