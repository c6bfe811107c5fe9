/*
 * latency_probe.hip -- measuring stick, not product code: what one small
 * host-path call costs on this MI355X, piece by piece, to decide how
 * libxudp's 100-frame TX batches (xudp.c:74 tx_batch_num) should reach the
 * GPU.  Frames and descriptors sit in pinned host memory (the registered
 * UMEM of the drop-in); results go back to pinned host memory.
 *
 *   launch floors   empty kernel + hipStreamSynchronize / hipEventSynchronize
 *                   / a host spin on a flag the kernel stores
 *   per-call work   one launch per batch that reads the batch over PCIe
 *                   (the DIRECT path's shape), completion by sync or by spin
 *   resident        W workgroups stay resident and poll a doorbell in host
 *                   memory; a batch is a doorbell store and a spin on W done
 *                   words.  Every wave leaves when the host says stop or after
 *                   IDLE_MS without a request (wall clock), so the grid always
 *                   drains.
 *
 * The per-frame work is a byte sum (one wave per frame, 16-byte loads): the
 * point is the latency around it.  usage: latency_probe [iters]
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>

#define CHK(x)                                                                     \
	do {                                                                       \
		hipError_t e_ = (x);                                               \
		if (e_ != hipSuccess) {                                            \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorName(e_)); \
			exit(2);                                                   \
		}                                                                  \
	} while (0)

struct Desc {
	uint64_t addr;
	uint32_t len, opt;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static double now_us()
{
	timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static __device__ __forceinline__ uint32_t ld_sys(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static __device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* frames [w, w + W, ...) of the batch, one wave each */
static __device__ void work(const uint8_t *umem, const Desc *desc, uint32_t n, uint16_t *out,
			    uint32_t wave, uint32_t nwaves)
{
	const uint32_t lane = threadIdx.x & 63;
	for (uint32_t i = wave; i < n; i += nwaves) {
		const Desc d = desc[i];
		const uint8_t *e = umem + d.addr;
		uint32_t s = 0;
		for (uint32_t o = lane * 16; o + 16 <= d.len; o += 1024) {
			const u32x4 v = *(const u32x4 *)(e + o);
			s += (v.x & 0xffff) + (v.x >> 16) + (v.y & 0xffff) + (v.y >> 16) +
			     (v.z & 0xffff) + (v.z >> 16) + (v.w & 0xffff) + (v.w >> 16);
		}
		for (int m = 32; m; m >>= 1)
			s += __shfl_xor(s, m);
		if (lane == 0)
			out[i] = (uint16_t)(s + (s >> 16));
	}
}

__global__ void empty_kernel() {}

__global__ void flag_kernel(uint32_t *flag, uint32_t v)
{
	if (threadIdx.x == 0)
		st_sys(flag, v);
}

/* one launch per batch (the DIRECT path's shape); block 0 of a 1-block grid
 * or the last block to finish raises the flag */
__global__ void __launch_bounds__(256) call_kernel(const uint8_t *umem, const Desc *desc, uint32_t n,
						   uint16_t *out, uint32_t *flag, uint32_t v,
						   uint32_t *dcount)
{
	work(umem, desc, n, out, blockIdx.x * 4 + (threadIdx.x >> 6), gridDim.x * 4);
	if (!flag)
		return;
	__syncthreads();
	if (threadIdx.x == 0) {
		__atomic_thread_fence(__ATOMIC_RELEASE);
		const uint32_t k = __hip_atomic_fetch_add(dcount, 1u, __ATOMIC_ACQ_REL,
							  __HIP_MEMORY_SCOPE_AGENT);
		if (k == gridDim.x - 1) {
			__hip_atomic_store(dcount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			st_sys(flag, v);
		}
	}
}

struct Doorbell {
	uint32_t seq;           /* host: request number */
	uint32_t n;
	uint32_t stop;
	uint32_t pad[29];
	uint32_t done[64 * 32]; /* workgroup w: done[32 * w] = seq served */
};

/* W resident workgroups; every wave polls, so no barrier is needed */
__global__ void __launch_bounds__(256) server_kernel(const uint8_t *umem, const Desc *desc,
						     uint16_t *out, Doorbell *db, uint32_t idle_ms)
{
	const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
	uint32_t served = 0;
	uint64_t last = wall_clock64();
	const uint64_t idle = (uint64_t)idle_ms * 100000ull;  /* 100 MHz */
	for (;;) {
		const uint32_t seq = __builtin_amdgcn_readfirstlane(ld_sys(&db->seq));
		if (ld_sys(&db->stop))
			break;
		if (seq == served) {
			if (wall_clock64() - last > idle)
				break;
			__builtin_amdgcn_s_sleep(2);
			continue;
		}
		const uint32_t n = __builtin_amdgcn_readfirstlane(ld_sys(&db->n));
		work(umem, desc, n, out, wave, nwaves);
		served = seq;
		last = wall_clock64();
		/* every wave of the workgroup done, then one system-scope release */
		__syncthreads();
		if (threadIdx.x == 0)
			st_sys(&db->done[32 * blockIdx.x], seq);
	}
}

static inline uint32_t vload(const uint32_t *p)
{
	return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

int main(int argc, char **argv)
{
	const int iters = argc > 1 ? atoi(argv[1]) : 2000;
	/* LP_SCHED=spin|yield|blocking: the runtime's wait policy */
	if (const char *e = getenv("LP_SCHED"))
		CHK(hipSetDeviceFlags(strcmp(e, "spin") == 0    ? hipDeviceScheduleSpin
				      : strcmp(e, "yield") == 0 ? hipDeviceScheduleYield
								: hipDeviceScheduleBlockingSync));
	const uint32_t NMAX = 4096, FRAME = 1514, SLOT = 4096;
	uint8_t *umem;
	Desc *desc;
	uint16_t *out;
	uint32_t *flag, *dcount;
	Doorbell *db;
	CHK(hipHostMalloc((void **)&umem, (size_t)NMAX * SLOT, hipHostMallocCoherent | hipHostMallocMapped));
	CHK(hipHostMalloc((void **)&desc, NMAX * sizeof(Desc), hipHostMallocCoherent | hipHostMallocMapped));
	CHK(hipHostMalloc((void **)&out, NMAX * 2, hipHostMallocCoherent | hipHostMallocMapped));
	CHK(hipHostMalloc((void **)&flag, 256, hipHostMallocCoherent | hipHostMallocMapped));
	CHK(hipHostMalloc((void **)&db, sizeof(Doorbell), hipHostMallocCoherent | hipHostMallocMapped));
	CHK(hipMalloc((void **)&dcount, 4));
	CHK(hipMemset(dcount, 0, 4));
	memset(db, 0, sizeof(Doorbell));
	for (uint32_t i = 0; i < NMAX * SLOT; i++)
		umem[i] = (uint8_t)(i * 131u + 7u);
	for (uint32_t i = 0; i < NMAX; i++)
		desc[i] = Desc{(uint64_t)i * SLOT + 384 - 42, FRAME, 0};
	/* device copies for the HBM-resident variant */
	uint8_t *d_umem;
	Desc *d_desc;
	uint16_t *d_out;
	CHK(hipMalloc((void **)&d_umem, (size_t)NMAX * SLOT));
	CHK(hipMalloc((void **)&d_desc, NMAX * sizeof(Desc)));
	CHK(hipMalloc((void **)&d_out, NMAX * 2));
	CHK(hipMemcpy(d_umem, umem, (size_t)NMAX * SLOT, hipMemcpyHostToDevice));
	CHK(hipMemcpy(d_desc, desc, NMAX * sizeof(Desc), hipMemcpyHostToDevice));

	hipStream_t s;
	hipEvent_t ev;
	CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));

	auto report = [&](const char *what, uint32_t n, double us) {
		printf("{\"probe\": \"%s\", \"frames\": %u, \"us_per_call\": %.2f}\n", what, n, us);
		fflush(stdout);
	};

	/* ---- launch floors ---- */
	for (int k = 0; k < 100; k++) {
		hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
		CHK(hipStreamSynchronize(s));
	}
	double t0 = now_us();
	for (int k = 0; k < iters; k++) {
		hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
		CHK(hipStreamSynchronize(s));
	}
	report("empty+streamsync", 0, (now_us() - t0) / iters);
	t0 = now_us();
	for (int k = 0; k < iters; k++) {
		hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
		CHK(hipEventRecord(ev, s));
		CHK(hipEventSynchronize(ev));
	}
	report("empty+eventsync", 0, (now_us() - t0) / iters);
	t0 = now_us();
	for (int k = 0; k < iters; k++) {
		hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
		CHK(hipEventRecord(ev, s));
		while (hipEventQuery(ev) == hipErrorNotReady)
			_mm_pause();
	}
	report("empty+eventquery_spin", 0, (now_us() - t0) / iters);
	*flag = 0;
	t0 = now_us();
	for (int k = 1; k <= iters; k++) {
		hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, flag, (uint32_t)k);
		while (vload(flag) != (uint32_t)k)
			_mm_pause();
	}
	report("flag+hostspin", 0, (now_us() - t0) / iters);
	CHK(hipStreamSynchronize(s));
	/* launch rate alone: back to back, one sync at the end */
	t0 = now_us();
	for (int k = 0; k < iters; k++)
		hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
	CHK(hipStreamSynchronize(s));
	report("empty_back_to_back", 0, (now_us() - t0) / iters);

	/* ---- one launch per batch, frames in pinned host memory ---- */
	const uint32_t sizes[] = {1, 16, 100, 1024};
	for (uint32_t n : sizes) {
		const int blocks = (int)((n + 3) / 4 < 64 ? (n + 3) / 4 : 64);
		char name[96];
		t0 = now_us();
		for (int k = 0; k < iters; k++) {
			hipLaunchKernelGGL(call_kernel, dim3(blocks), dim3(256), 0, s, umem, desc, n, out,
					   (uint32_t *)nullptr, 0u, dcount);
			CHK(hipStreamSynchronize(s));
		}
		snprintf(name, sizeof name, "call_host_frames+streamsync(%d blocks)", blocks);
		report(name, n, (now_us() - t0) / iters);
		*flag = 0;
		t0 = now_us();
		for (int k = 1; k <= iters; k++) {
			hipLaunchKernelGGL(call_kernel, dim3(blocks), dim3(256), 0, s, umem, desc, n, out, flag,
					   (uint32_t)k, dcount);
			while (vload(flag) != (uint32_t)k)
				_mm_pause();
		}
		snprintf(name, sizeof name, "call_host_frames+hostspin(%d blocks)", blocks);
		report(name, n, (now_us() - t0) / iters);
		CHK(hipStreamSynchronize(s));
		t0 = now_us();
		for (int k = 0; k < iters; k++) {
			hipLaunchKernelGGL(call_kernel, dim3(blocks), dim3(256), 0, s, d_umem, d_desc, n, d_out,
					   (uint32_t *)nullptr, 0u, dcount);
			CHK(hipStreamSynchronize(s));
		}
		snprintf(name, sizeof name, "call_hbm_frames+streamsync(%d blocks)", blocks);
		report(name, n, (now_us() - t0) / iters);
	}

	/* ---- resident workgroups polling a doorbell ---- */
	const int wgs[] = {1, 8, 32};
	for (int W : wgs) {
		for (int hbm = 0; hbm < 2; hbm++) {
			memset(db, 0, sizeof(Doorbell));
			hipLaunchKernelGGL(server_kernel, dim3(W), dim3(256), 0, s, hbm ? d_umem : umem,
					   hbm ? d_desc : desc, hbm ? d_out : out, db, 500u);
			CHK(hipGetLastError());
			uint32_t seq = 0;
			bool dead = false;
			for (uint32_t n : sizes) {
				auto one = [&]() {
					seq++;
					db->n = n;
					__atomic_store_n(&db->seq, seq, __ATOMIC_RELEASE);
					const double tw = now_us();
					for (int w = 0; w < W; w++)
						while (vload(&db->done[32 * w]) != seq) {
							_mm_pause();
							if (now_us() - tw > 200000.0)
								return false;
						}
					return true;
				};
				for (int k = 0; k < 50 && !dead; k++)
					dead = !one();
				t0 = now_us();
				for (int k = 0; k < iters && !dead; k++)
					dead = !one();
				char name[96];
				snprintf(name, sizeof name, "resident_%s(%d wg)", hbm ? "hbm_frames" : "host_frames", W);
				if (dead) {
					printf("{\"probe\": \"%s\", \"frames\": %u, \"error\": \"no answer in 200 ms\"}\n",
					       name, n);
					break;
				}
				report(name, n, (now_us() - t0) / iters);
			}
			__atomic_store_n(&db->stop, 1u, __ATOMIC_RELEASE);
			CHK(hipStreamSynchronize(s));
			if (dead)
				return 1;
		}
	}
	/* check: the last resident pass (HBM frames, 1024) against one launch on
	 * the host frames (the same bytes) */
	hipLaunchKernelGGL(call_kernel, dim3(64), dim3(256), 0, s, umem, desc, 1024u, out,
			   (uint32_t *)nullptr, 0u, dcount);
	CHK(hipStreamSynchronize(s));
	static uint16_t ref[1024];
	CHK(hipMemcpy(ref, d_out, sizeof ref, hipMemcpyDeviceToHost));
	int bad = 0;
	for (int i = 0; i < 1024; i++)
		bad += ref[i] != out[i];
	printf("{\"probe\": \"done\", \"mismatch\": %d}\n", bad);
	return 0;
}
