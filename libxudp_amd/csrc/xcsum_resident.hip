/*
 * xcsum_resident.hip -- resident checksum workgroups for small host batches.
 *
 * libxudp sends in batches of tx_batch_num = 100 frames (xudp/xudp.c:74); each
 * batch is one trip through xudp_frame_send (tx.c:673-734).  As a kernel
 * launch per batch, a call costs a launch and a completion (~17-20 us,
 * DESIGN.md 5.8) for microseconds of work.  A resident server removes both:
 * W workgroups stay on the device and poll a doorbell in pinned host memory
 * (xcsum_resident.h); a batch is the request and its descriptors written
 * there, a sequence number stored after them, and a host spin on one "done"
 * word per workgroup.
 *
 * The work is the frame-group checksum loop itself (csum_loop<16, 2, 6, 2>
 * of xcsum_csum.h: every mode and flag, bit-exact with the launched kernels),
 * over frames the host gathered into the context's pinned stage, each
 * descriptor checked against the request's bounds inside the loop.
 *
 * Memory ordering (all vector memory operations):
 *   - wave 0 of a workgroup polls `seq` (and `stop`, the same 8 bytes) with
 *     relaxed system-scope loads, then, once per request, a system-scope
 *     acquire fence: it invalidates the CU's L1 and the L2's non-coherent
 *     lines, so the request, descriptors and frame bytes the host wrote
 *     before `seq` are read fresh by every wave after the workgroup barrier
 *     that follows;
 *   - every wave ends a request with a system-scope release fence (its
 *     results and in-place stores written back to host memory), then the
 *     workgroup barrier, then thread 0 stores done[w] = seq;
 *   - descriptor and frame loads are vector loads (G = 16: one descriptor per
 *     lane), never through the scalar cache, which the acquire does not
 *     invalidate.
 *
 * Lifetime: a workgroup leaves when the host sets `stop`, after idle_ticks
 * of the 100 MHz wall clock without a request, or once it has lived
 * life_ticks (checked between requests), so the grid always drains on its
 * own and a busy server gives its hardware queue back every few ms.  The host relaunches on the next batch (see resident_call in
 * xcsum_api.hip, which also covers a workgroup that left at the idle deadline
 * while a request was on its way: it is relaunched with a mask of the
 * workgroups that already served that request, so no frame is done twice --
 * an in-place frame summed twice would sum its own check field).
 */
#include "xcsum_csum.h"
#include "xcsum_resident.h"

namespace xcsum {

static __device__ __forceinline__ uint32_t ld_relaxed_sys(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static __device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi)
{
	return ((uint64_t)hi << 32) | lo;
}

/* The resident loop's arguments: a request's frames must lie inside
 * [bias, bias + limit) of its buffer; csum_loop checks every descriptor before
 * any load of its frame (resolve) and hands a bad one to desc_bad, which keeps
 * the workgroup's lowest bad index in LDS.  The check rides on the loop's own
 * descriptor loads, so it costs no round trip of its own. */
struct ResidentArgs : CsumArgs {
	static constexpr bool kChecked = true;
	uint64_t limit;
	uint32_t *first_bad;   /* LDS */
	const uint32_t *inl;   /* LDS: the request's inline descriptors, or null */
};

static __device__ __forceinline__ u32x4 desc_inline(const ResidentArgs &a, uint32_t q)
{
	const uint32_t *w = a.inl + 4u * q;
	return u32x4{w[0], w[1], w[2], w[3]};
}

static __device__ __forceinline__ bool desc_ok(const ResidentArgs &a, u32x4 d)
{
	const uint64_t ad = ((uint64_t)d.y << 32) | d.x;
	return !(ad < a.bias || ad - a.bias > a.limit || d.z > a.limit - (ad - a.bias));
}

static __device__ __forceinline__ void desc_bad(const ResidentArgs &a, uint32_t p)
{
	atomicMin(a.first_bad, p);
}

/* served0: the sequence number every workgroup has served at launch, except
 * the workgroups of skip_mask (bit w), which served skip_seq already
 * (relaunch after a partial service, see the file comment) */
template <int G, int U, int K>
__global__ void __launch_bounds__(256) resident_kernel(const ResidentBell *bell, ResidentDone *done,
						       unsigned long long *err, uint32_t gen,
						       uint32_t served0, uint32_t skip_seq,
						       uint64_t skip_mask, uint64_t idle_ticks,
						       uint64_t life_ticks)
{
	__shared__ uint32_t cmd[RB_REQ_WORDS + 1];
	__shared__ uint32_t first_bad_lds;   /* ResidentArgs::first_bad */
	__shared__ uint32_t inl_lds[4 * RB_INLINE];   /* ResidentArgs::inl */
	__shared__ uint32_t inl_on;
#ifdef XCSUM_DEBUG_BOUNDS
	__shared__ uint32_t allow_lds[2 * RB_ALLOW_N];
#endif
	const uint32_t lane = threadIdx.x & 63;
	uint32_t served = served0;
	if (blockIdx.x < 64 && ((skip_mask >> blockIdx.x) & 1ull))
		served = skip_seq;
	uint64_t last = wall_clock64();
	const uint64_t born = last;
	for (;;) {
		if (threadIdx.x < 64) {
			/* one load of the doorbell's first 256 bytes per poll: lane i
			 * reads word i -- seq (0), stop (1), the request (16...) and
			 * the inline descriptors (32...), each 64-byte line with its
			 * own echo of the sequence number (written after the line's
			 * other words, xcsum_api.hip resident_call) saying the words
			 * read with it belong to that request.  Relaxed: no cache
			 * maintenance per poll (an acquire load per poll invalidated the
			 * L2 every time: 12-55 us per request, tools/latency_probe). */
			const uint32_t *words = (const uint32_t *)bell;
			uint32_t s = served, go = 0, v = 0, inl = 0;
			for (;;) {
				v = ld_relaxed_sys(words + lane);
				s = __builtin_amdgcn_readlane(v, 0);
				if (__builtin_amdgcn_readlane(v, 1))
					break;   /* stop */
				if (s != served && __builtin_amdgcn_readlane(v, 16 + RB_SEQ) == s) {
					/* inline descriptors only if their lines are this
					 * request's; else the ones in desc[] (always written) */
					const uint32_t n = __builtin_amdgcn_readlane(v, 16 + RB_N);
					inl = n <= RB_INLINE &&
					      __builtin_amdgcn_readlane(v, 32 + RB_INL_ECHO) == s &&
					      (n <= 3 || __builtin_amdgcn_readlane(v, 48 + RB_INL_ECHO) == s);
					go = 1;
					break;
				}
				/* idle, or alive for life_ticks: leave (the next batch
				 * relaunches).  The life bound caps how long a busy
				 * server holds its hardware queue, which other streams
				 * of the process may share (GPU_MAX_HW_QUEUES): their
				 * work waits behind this grid */
				const uint64_t now = wall_clock64();
				if (now - last > idle_ticks || now - born > life_ticks)
					break;
				__builtin_amdgcn_s_sleep(1);
			}
			/* one acquire per request: the descriptors and frames the host
			 * wrote before seq are read fresh from here on */
			if (go)
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
			if (lane >= 16 && lane < 16 + RB_REQ_WORDS)
				cmd[1 + lane - 16] = v;
#ifdef XCSUM_DEBUG_BOUNDS
			if (lane >= 2 && lane < 2 + 2 * RB_ALLOW_N)
				allow_lds[lane - 2] = v;
#endif
			if (lane >= 32 && (lane & 15) < RB_INL_ECHO)   /* 3 descriptors a line */
				inl_lds[(lane >> 4 == 3 ? 12 : 0) + (lane & 15)] = v;
			if (lane == 0) {
				cmd[0] = go ? s : 0u;
				first_bad_lds = ~0u;
				inl_on = go && inl;
			}
		}
		__syncthreads();
		const uint32_t s = __builtin_amdgcn_readfirstlane(cmd[0]);
		if (s != 0u && __builtin_amdgcn_readfirstlane(cmd[1 + RB_SEQ]) != s) {
			/* the request read is not the one announced (never seen; a
			 * guard against serving stale words): poll again */
			__syncthreads();
			continue;
		}
		if (s == 0u) {
			/* stop or idle: the whole workgroup leaves (sequence numbers
			 * skip 0), and says so */
			if (threadIdx.x == 0)
				__hip_atomic_store(&done->done[RB_DONE_STRIDE * blockIdx.x + RB_LEFT], gen,
						   __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
			break;
		}
		uint32_t r[RB_REQ_WORDS];
#pragma unroll
		for (int k = 0; k < RB_REQ_WORDS; k++)
			r[k] = __builtin_amdgcn_readfirstlane(cmd[1 + k]);
		ResidentArgs a;
		a.umem = (uint8_t *)(uintptr_t)u64_of(r[RB_UMEM], r[RB_UMEM + 1]);
		a.desc = (const struct xcsum_desc *)(uintptr_t)u64_of(r[RB_DESC], r[RB_DESC + 1]);
		a.out = (uint16_t *)(uintptr_t)u64_of(r[RB_OUT], r[RB_OUT + 1]);
		a.out_ip = (uint16_t *)(uintptr_t)u64_of(r[RB_OUT_IP], r[RB_OUT_IP + 1]);
		a.bias = u64_of(r[RB_BIAS], r[RB_BIAS + 1]);
		a.n = r[RB_N];
		a.mode = r[RB_MODE];
		a.flags = r[RB_FLAGS];
		a.err = err;
		a.ord = order_identity(a.n);
		a.dense = a.ord;
		a.limit = u64_of(r[RB_LIMIT], r[RB_LIMIT + 1]);
		a.first_bad = &first_bad_lds;
		a.inl = __builtin_amdgcn_readfirstlane(inl_on) ? inl_lds : nullptr;
#ifdef XCSUM_DEBUG_BOUNDS
		{
			/* the request's pointers against the context's own buffers:
			 * frames [umem, umem + limit) in the stage, n descriptors in
			 * the doorbell (unless inline), n (2n with IPHDR) results in
			 * the result slot; a request outside them is not served */
			auto al = [&](int k) {
				return u64_of(allow_lds[2 * k], allow_lds[2 * k + 1]);
			};
			const uint64_t um = (uint64_t)(uintptr_t)a.umem;
			const uint64_t ds = (uint64_t)(uintptr_t)a.desc;
			const uint64_t ot = (uint64_t)(uintptr_t)a.out;
			const uint64_t oi = (uint64_t)(uintptr_t)a.out_ip;
			bool ok = xb_in(um, a.limit, al(RB_ALLOW_STAGE), al(RB_ALLOW_STAGE + 1), XB_RES_REQ,
					s);
			ok = ok && (a.inl || xb_in(ds, 16ull * a.n, al(RB_ALLOW_DESC), al(RB_ALLOW_DESC + 1),
						   XB_RES_REQ, s));
			ok = ok && xb_in(ot, 2ull * a.n, al(RB_ALLOW_OUT), al(RB_ALLOW_OUT + 1), XB_RES_REQ, s);
			ok = ok && (!oi || xb_in(oi, 2ull * a.n, al(RB_ALLOW_OUT), al(RB_ALLOW_OUT + 1),
						 XB_RES_REQ, s));
			if (!ok)
				a.n = 0;
			if (threadIdx.x == 0) {
				uint32_t *cr = &done->done[RB_DONE_STRIDE * blockIdx.x + RB_CRUMB];
				cr[1] = (uint32_t)um;
				cr[2] = (uint32_t)(um >> 32);
				cr[3] = a.n;
				cr[4] = (uint32_t)ds;
				cr[5] = (uint32_t)(ds >> 32);
				__hip_atomic_store(&cr[0], s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
			}
		}
#endif
		csum_loop<G, U, K, false, 2>(a);
		/* a descriptor outside the request's bounds: its frame was not
		 * read; report the workgroup's first (the host fails the call) */
		__syncthreads();
		const uint32_t first_bad = __builtin_amdgcn_readfirstlane(first_bad_lds);
		if (first_bad != ~0u && threadIdx.x == 0) {
			const u32x4 d = *((gu32x4 *)(a.desc + first_bad));
			uint32_t *o = &done->done[RB_DONE_STRIDE * blockIdx.x + RB_BAD];
			o[1] = first_bad;
			o[2] = d.x;
			o[3] = d.y;
			o[4] = d.z;
			__hip_atomic_store(&o[0], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		}
		/* this wave's results and in-place stores reach host memory ... */
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
		/* ... for every wave, before done[w] says so */
		__syncthreads();
		if (threadIdx.x == 0)
			__hip_atomic_store(&done->done[RB_DONE_STRIDE * blockIdx.x], s, __ATOMIC_RELEASE,
					   __HIP_MEMORY_SCOPE_SYSTEM);
		served = s;
		last = wall_clock64();
	}
}

hipError_t launch_resident(ResidentBell *v_bell, ResidentDone *v_done, unsigned long long *err,
			   int wg, uint32_t gen, uint32_t served0, uint32_t skip_seq,
			   uint64_t skip_mask, uint32_t idle_us, uint32_t life_us, hipStream_t s)
{
	if (wg <= 0 || wg > RB_MAX_WG)
		return hipErrorInvalidValue;
	(void)hipGetLastError();
	hipLaunchKernelGGL((resident_kernel<16, 2, 6>), dim3((unsigned)wg), dim3(256), 0, s, v_bell, v_done,
			   err, gen, served0, skip_seq, skip_mask, (uint64_t)idle_us * 100ull,
			   (uint64_t)life_us * 100ull);
	return hipGetLastError();
}

} /* namespace xcsum */
