/* xcsum_stage.h -- host-side copies into the context's pinned stages
 * (xcsum_api.hip's host batches): the staged position of a
 * gathered frame, the range copy, and the frame-by-frame gather, split over
 * up to STAGE_THREADS threads for large copies.  The threads are a small
 * pool each context keeps (StagePool: started on its first large copy,
 * parked between calls, joined by xcsum_ctx_destroy), and a copy uses only
 * as many as the calling thread's CPU budget allows -- its affinity mask and
 * the cgroup CPU quota, not the machine's CPU count: a libxudp TX worker
 * pinned to one core copies alone.  Plain C++ over caller
 * memory, so tests/test_stage_copy.py exercises it with g++ on the CPU
 * (thread splits, caps, phases, the budget); no HIP. */
#ifndef XCSUM_STAGE_H
#define XCSUM_STAGE_H

#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <functional>
#include <mutex>
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

/* CPUs of the cgroup quota (cgroup v2 cpu.max, else v1 cfs_quota/period),
 * rounded up; 0 = no quota.  Read once per process. */
static inline int cgroup_cpu_quota()
{
	static std::once_flag once;
	static int quota = 0;
	std::call_once(once, [] {
		long long q = -1, p = 0;
		if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
			char qs[32] = {0};
			if (fscanf(f, "%31s %lld", qs, &p) == 2 && strcmp(qs, "max") != 0)
				q = atoll(qs);
			fclose(f);
		} else if (FILE *f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
			if (fscanf(f1, "%lld", &q) != 1)
				q = -1;
			fclose(f1);
			if (FILE *f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
				if (fscanf(f2, "%lld", &p) != 1)
					p = 0;
				fclose(f2);
			}
		}
		if (q > 0 && p > 0)
			quota = (int)((q + p - 1) / p);
	});
	return quota;
}

/* CPUs the calling thread may run on: its affinity mask, capped by the
 * cgroup quota.  `mask_cpus` > 0 overrides the mask count (tests). */
static inline int usable_cpus(int mask_cpus = 0)
{
	int n = mask_cpus;
	if (n <= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
	}
	const int q = cgroup_cpu_quota();
	if (q > 0 && q < n)
		n = q;
	return n > 0 ? n : 1;
}

/* threads for a host copy of n bytes in `pieces` memcpys (a gather of
 * small frames is bound by the latency of each frame's lines, not bytes):
 * STAGE_THREADS for large copies when the caller may use at least twice as
 * many CPUs, else half of what it may use, and 1 below 4 usable CPUs */
static inline int stage_threads(uint64_t n, uint32_t pieces = 1, int cpus = 0)
{
	int k = n >= (4u << 20) || pieces >= 16384u ? STAGE_THREADS : 1;
	const int u = cpus > 0 ? cpus : usable_cpus();
	if (u < 2 * k)
		k = u >= 4 ? u / 2 : 1;
	return k;
}

/* The context's copy threads: STAGE_THREADS - 1 workers (the caller is the
 * other one), started on the first split copy, parked on a condition
 * variable between calls.  run(k, fn) calls fn(0..k-1), part 0 on the
 * caller, and returns when all k parts are done.  One caller at a time (one
 * context per host thread, include/xcsum.h).  If a worker cannot be
 * started, its parts run on the caller. */
struct StagePool {
	StagePool() = default;
	StagePool(const StagePool &) = delete;
	StagePool &operator=(const StagePool &) = delete;
	~StagePool() { stop(); }

	void run(int k, const std::function<void(int)> &fn)
	{
		if (k > STAGE_THREADS)
			k = STAGE_THREADS;
		if (k <= 1) {
			fn(0);
			return;
		}
		start(k - 1);
		const int w = k - 1 < nth_ ? k - 1 : nth_;   /* parts the workers take */
		{
			std::lock_guard<std::mutex> g(mu_);
			job_ = &fn;
			parts_ = w;
			pending_ = w;
			gen_++;
		}
		cv_work_.notify_all();
		fn(0);
		for (int t = w + 1; t < k; t++)   /* workers that did not start */
			fn(t);
		std::unique_lock<std::mutex> l(mu_);
		cv_done_.wait(l, [this] { return pending_ == 0; });
		job_ = nullptr;
	}

	int threads() const { return nth_; }   /* workers started */

	void stop()
	{
		{
			std::lock_guard<std::mutex> g(mu_);
			quit_ = true;
		}
		cv_work_.notify_all();
		for (int t = 0; t < nth_; t++)
			if (th_[t].joinable())
				th_[t].join();
		nth_ = 0;
	}

private:
	void start(int want)
	{
		while (nth_ < want && nth_ < STAGE_THREADS - 1) {
			const int id = nth_;
			/* the generation before the job this call posts: only run(),
			 * on the calling thread, moves gen_ */
			const uint64_t g0 = gen_;
			try {
				th_[id] = std::thread([this, id, g0] { worker(id, g0); });
			} catch (...) {
				return;
			}
			nth_++;
		}
	}

	void worker(int id, uint64_t seen)
	{
		std::unique_lock<std::mutex> l(mu_);
		for (;;) {
			cv_work_.wait(l, [&] { return quit_ || gen_ != seen; });
			if (quit_)
				return;
			seen = gen_;
			if (id >= parts_)
				continue;
			const std::function<void(int)> *fn = job_;
			l.unlock();
			(*fn)(id + 1);
			l.lock();
			if (--pending_ == 0)
				cv_done_.notify_one();
		}
	}

	std::mutex mu_;
	std::condition_variable cv_work_, cv_done_;
	std::thread th_[STAGE_THREADS - 1];
	int nth_ = 0;
	uint64_t gen_ = 0;
	int parts_ = 0, pending_ = 0;
	bool quit_ = false;
	const std::function<void(int)> *job_ = nullptr;
};

/* run fn over k parts on `pool`, or serially without one */
static inline void stage_run(StagePool *pool, int k, const std::function<void(int)> &fn)
{
	if (pool) {
		pool->run(k, fn);
		return;
	}
	for (int t = 0; t < k; t++)
		fn(t);
}

static void stage_copy(StagePool *pool, uint8_t *dst, const uint8_t *src, uint64_t n)
{
	const int k = stage_threads(n);
	if (k <= 1) {
		memcpy(dst, src, n);
		return;
	}
	const uint64_t part = ((n + k - 1) / k + 4095) & ~(uint64_t)4095;
	stage_run(pool, k, [=](int t) {
		const uint64_t off = part * (uint64_t)t;
		if (off < n)
			memcpy(dst + off, src + off, n - off < part ? n - off : part);
	});
}

/* Frame-by-frame gather into a pinned stage: frame k at its 16-byte phase
 * (stage_off), at most `cap` bytes of it; ds[k] = its staged descriptor
 * (the frame's own length, for the kernel's rules).  From 4 MiB of staged
 * bytes or 16384 frames up the copies are split by staged bytes over up to
 * STAGE_THREADS threads (stage_threads).  Returns the staged bytes. */
static uint64_t gather_frames(StagePool *pool, uint8_t *stage, const uint8_t *umem,
			      const struct xcsum_desc *d, struct xcsum_desc *ds, uint32_t cnt,
			      uint32_t cap)
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
	stage_run(pool, nt, [&](int t) { copy(b[t], b[t + 1]); });
	return pos;
}

} /* namespace xcsum */

#endif
