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

struct alignas(64) Doorbell {
	uint32_t seq;           /* host: request number */
	uint32_t stop;          /* next to seq: one 8-byte poll reads both */
	uint32_t n;
	uint32_t pad[29];
	uint32_t done[64 * 32]; /* workgroup w: done[32 * w] = seq served */
};

/* W resident workgroups; wave 0 of each polls, the workgroup follows.
 * MODE 0: every poll a system-scope acquire load (L2 invalidate per poll);
 * MODE 1: relaxed system-scope polls (no cache maintenance), one acquire
 *         fence per request, release store of done;
 * MODE 2: relaxed polls, no cache maintenance at all (fine-grained memory
 *         only: nothing of it is cached), relaxed store of done after the
 *         workgroup's stores have completed;
 * MODE 3: MODE 1 with the doorbell (seq, stop, n) in fine-grained DEVICE
 *         memory the host writes through the BAR: polls stay on the card. */
template <int MODE>
__global__ void __launch_bounds__(256) server_kernel(const uint8_t *umem, const Desc *desc,
						     uint16_t *out, Doorbell *db, uint32_t idle_ms,
						     Doorbell *bell)
{
	__shared__ uint32_t cmd[2];
	const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
	uint32_t served = 0;
	uint64_t last = wall_clock64();
	const uint64_t idle = (uint64_t)idle_ms * 100000ull;  /* 100 MHz */
	for (;;) {
		if (threadIdx.x < 64) {
			uint32_t seq = served, go = 0;
			for (;;) {
				uint64_t w;
				if (MODE == 0) {
					seq = ld_sys(&bell->seq);
					w = ((uint64_t)ld_sys(&bell->stop) << 32) | seq;
				} else {
					w = __hip_atomic_load((const uint64_t *)__builtin_assume_aligned(&bell->seq, 8), __ATOMIC_RELAXED,
							      __HIP_MEMORY_SCOPE_SYSTEM);
				}
				w = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)) << 32) |
				    __builtin_amdgcn_readfirstlane((uint32_t)w);
				seq = (uint32_t)w;
				if (w >> 32)
					break;
				if (seq != served) {
					go = 1;
					break;
				}
				if (wall_clock64() - last > idle)
					break;
				__builtin_amdgcn_s_sleep(1);
			}
			if ((MODE == 1 || MODE == 3) && go)
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
			uint32_t n = 0;
			if (go)
				n = __hip_atomic_load(&bell->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			if (threadIdx.x == 0) {
				cmd[0] = go ? seq : 0u;
				cmd[1] = n;
			}
		}
		__syncthreads();
		const uint32_t seq = __builtin_amdgcn_readfirstlane(cmd[0]);
		const uint32_t n = __builtin_amdgcn_readfirstlane(cmd[1]);
		if (!seq)
			break;
		work(umem, desc, n, out, wave, nwaves);
		if (MODE == 2)
			__builtin_amdgcn_s_waitcnt(0);   /* this wave's stores done */
		else
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
		__syncthreads();
		if (threadIdx.x == 0) {
			if (MODE == 2)
				__hip_atomic_store(&db->done[32 * blockIdx.x], seq, __ATOMIC_RELAXED,
						   __HIP_MEMORY_SCOPE_SYSTEM);
			else
				st_sys(&db->done[32 * blockIdx.x], seq);
		}
		served = seq;
		last = wall_clock64();
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
	Doorbell *dbell = nullptr;   /* fine-grained device memory, host-writable */
	CHK(hipExtMallocWithFlags((void **)&dbell, sizeof(Doorbell) + (64u << 10), hipDeviceMallocFinegrained));
	{
		hipPointerAttribute_t at;
		memset(&at, 0, sizeof at);
		const hipError_t e = hipPointerGetAttributes(&at, dbell);
		printf("{\"probe\": \"finegrained_device_attr\", \"rc\": %d, \"type\": %d, "
		       "\"host_ptr_is_dev_ptr\": %d, \"host_ptr_null\": %d}\n", (int)e, (int)at.type,
		       at.hostPointer == (void *)dbell, at.hostPointer == nullptr);
		/* host stores into it through the BAR: descriptor-sized copies */
		static uint8_t src[64u << 10];
		memset(src, 7, sizeof src);
		for (uint32_t bytes : {1600u, 16384u, 65536u}) {
			uint8_t *dst = (uint8_t *)(dbell + 1);
			memcpy(dst, src, bytes);
			_mm_sfence();
			const double t = now_us();
			for (int k = 0; k < 200; k++) {
				memcpy(dst, src, bytes);
				_mm_sfence();
			}
			printf("{\"probe\": \"host_memcpy_to_finegrained_device\", \"bytes\": %u, "
			       "\"us\": %.2f}\n", bytes, (now_us() - t) / 200);
		}
	}
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
	const int wgs[] = {1, 4, 8, 16};
	for (int mode = 0; mode < 4; mode++)
	for (int W : wgs) {
		for (int hbm = 0; hbm < 2; hbm++) {
			memset(db, 0, sizeof(Doorbell));
			Doorbell *bell = mode == 3 ? dbell : db;
			if (mode == 3) {
				CHK(hipMemset(dbell, 0, sizeof(Doorbell)));
				CHK(hipDeviceSynchronize());
			}
#define SRV(M) hipLaunchKernelGGL(server_kernel<M>, dim3(W), dim3(256), 0, s, hbm ? d_umem : umem, \
				  hbm ? d_desc : desc, hbm ? d_out : out, db, 500u, bell)
			if (mode == 0) SRV(0); else if (mode == 1) SRV(1); else if (mode == 2) SRV(2); else SRV(3);
#undef SRV
			CHK(hipGetLastError());
			uint32_t seq = 0;
			bool dead = false;
			for (uint32_t n : sizes) {
				auto one = [&]() {
					seq++;
					bell->n = n;
					__atomic_store_n(&bell->seq, seq, __ATOMIC_RELEASE);
					_mm_sfence();
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
				snprintf(name, sizeof name, "resident_m%d_%s(%d wg)", mode,
					 hbm ? "hbm_frames" : "host_frames", W);
				if (dead) {
					printf("{\"probe\": \"%s\", \"frames\": %u, \"error\": \"no answer in 200 ms\"}\n",
					       name, n);
					break;
				}
				report(name, n, (now_us() - t0) / iters);
			}
			__atomic_store_n(&bell->stop, 1u, __ATOMIC_RELEASE);
			_mm_sfence();
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
