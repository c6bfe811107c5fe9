/* xcsum_stage.h -- host-side copies into the context's pinned stages
 * (xcsum_api.hip's host batches): the staged position of a
 * gathered frame, the range copy, and the frame-by-frame gather, both split
 * over up to STAGE_THREADS threads for large copies.  Plain C++ over
 * caller memory, so tests/test_stage_copy.py exercises it with g++ on the
 * CPU (thread splits, caps, phases); no HIP. */
#ifndef XCSUM_STAGE_H
#define XCSUM_STAGE_H

#include <stdint.h>
#include <string.h>
#include <thread>

#include "xcsum.h"

namespace xcsum {

/* staged offset of a gathered frame: packed, each at its UMEM 16-byte phase
 * (the kernel sees the same address parity and alignment) */
static inline uint64_t stage_off(uint64_t pos, uint64_t addr)
{
	return ((pos + 15) & ~(uint64_t)15) + (addr & 15);
}

/* memcpy into a pinned stage, split over up to STAGE_THREADS threads from
 * 4 MiB up: one thread copies ~25 GB/s here, under the ~57 GB/s PCIe moves
 * (config 2 frames, pageable, tools/bench_e2e.py: 23.0 GiB/s with one thread) */
static constexpr int STAGE_THREADS = 4;

/* threads for a host copy of n bytes in `pieces` memcpys (a gather of
 * small frames is bound by the latency of each frame's lines, not bytes) */
static int stage_threads(uint64_t n, uint32_t pieces = 1)
{
	const unsigned hw = std::thread::hardware_concurrency();
	int k = n >= (4u << 20) || pieces >= 16384u ? STAGE_THREADS : 1;
	if (hw && (int)hw < 2 * k)
		k = hw >= 4 ? (int)hw / 2 : 1;
	return k;
}

static void stage_copy(uint8_t *dst, const uint8_t *src, uint64_t n)
{
	const int k = stage_threads(n);
	if (k <= 1) {
		memcpy(dst, src, n);
		return;
	}
	const uint64_t part = ((n + k - 1) / k + 4095) & ~(uint64_t)4095;
	std::thread th[STAGE_THREADS];
	int started = 0;
	for (int t = 1; t < k; t++) {
		const uint64_t off = part * t;
		if (off >= n)
			break;
		const uint64_t len = n - off < part ? n - off : part;
		try {
			th[t] = std::thread(memcpy, dst + off, src + off, len);
			started = t;
		} catch (...) {
			memcpy(dst + off, src + off, len);   /* no thread: copy here */
		}
	}
	memcpy(dst, src, n < part ? n : part);
	for (int t = 1; t <= started; t++)
		if (th[t].joinable())
			th[t].join();
}

/* Frame-by-frame gather into a pinned stage: frame k at its 16-byte phase
 * (stage_off), at most `cap` bytes of it; ds[k] = its staged descriptor
 * (the frame's own length, for the kernel's rules).  From 4 MiB of staged
 * bytes or 16384 frames up the copies are split by staged bytes over up to
 * STAGE_THREADS threads (stage_threads).  Returns the staged bytes. */
static uint64_t gather_frames(uint8_t *stage, const uint8_t *umem, const struct xcsum_desc *d,
			      struct xcsum_desc *ds, uint32_t cnt, uint32_t cap)
{
	uint64_t pos = 0;
	for (uint32_t k = 0; k < cnt; k++) {
		const uint64_t off = stage_off(pos, d[k].addr);
		ds[k] = xcsum_desc{off, d[k].len, 0};
		pos = off + (d[k].len < cap ? d[k].len : cap);
	}
	auto copy = [stage, umem, d, ds, cap](uint32_t k0, uint32_t k1) {
		for (uint32_t k = k0; k < k1; k++)
			memcpy(stage + ds[k].addr, umem + d[k].addr, d[k].len < cap ? d[k].len : cap);
	};
	const int nt = stage_threads(pos, cnt);
	if (nt <= 1) {
		copy(0, cnt);
		return pos;
	}
	/* thread t copies the frames staged in [pos * t / nt, pos * (t+1) / nt) */
	uint32_t b[STAGE_THREADS + 1];
	b[0] = 0;
	b[nt] = cnt;
	for (int t = 1; t < nt; t++) {
		const uint64_t target = pos / nt * t;
		uint32_t lo = b[t - 1], hi = cnt;
		while (lo < hi) {   /* first frame staged at or after target */
			const uint32_t mid = lo + (hi - lo) / 2;
			if (ds[mid].addr < target)
				lo = mid + 1;
			else
				hi = mid;
		}
		b[t] = lo;
	}
	std::thread th[STAGE_THREADS];
	int started = 0;
	for (int t = 1; t < nt; t++) {
		try {
			th[t] = std::thread(copy, b[t], b[t + 1]);
			started = t;
		} catch (...) {
			copy(b[t], b[t + 1]);   /* no thread: copy here */
		}
	}
	copy(b[0], b[1]);
	for (int t = 1; t <= started; t++)
		if (th[t].joinable())
			th[t].join();
	return pos;
}

} /* namespace xcsum */

#endif
