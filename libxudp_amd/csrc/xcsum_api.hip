/*
 * xcsum_api.hip -- host side of libxcsum.so: the C ABI of include/xcsum.h.
 *
 * Error behaviour follows the reference (include/xudp.h:67-140): negative
 * codes, never abort, errno untouched except by the packet.c mirrors.
 */
#include <errno.h>
#include <sys/prctl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <new>
#include <chrono>
#include <mutex>
#include <thread>

#include <hsa/hsa_ext_amd.h>

#include "xcsum_internal.h"
#include "xcsum_gen.h"
#include "xcsum_thp.h"
#include "xcsum_stage.h"

using namespace xcsum;

/* the last failing HIP call of this thread, for xcsum_last_hip_error() */
static thread_local int t_hip_err = 0, t_hip_line = 0;

#define HIPCHK(x)                                           \
	do {                                                \
		const hipError_t e_ = (x);                  \
		if (e_ != hipSuccess) {                     \
			t_hip_err = (int)e_;                \
			t_hip_line = __LINE__;              \
			return -XCSUM_ERR_HIP;              \
		}                                           \
	} while (0)

extern "C" int xcsum_last_hip_error(int *line, const char **name)
{
	if (line)
		*line = t_hip_line;
	if (name)
		*name = t_hip_err ? hipGetErrorName((hipError_t)t_hip_err) : "hipSuccess";
	return t_hip_err;
}

/* resident server defaults (xcsum_ctx_set_resident) */
static constexpr uint32_t RES_IDLE_US = 20000;     /* workgroups leave after 20 ms idle */
/* ... and after 2 ms alive even when busy: a live resident grid blocks the
 * work of any stream that shares its hardware queue (GPU_MAX_HW_QUEUES is 4;
 * streams beyond that share queues), so its life is bounded; the next batch
 * relaunches (~10 us, once per 2 ms of service) */
static constexpr uint32_t RES_LIFE_US = 2000;
static constexpr uint32_t RES_MAX_FRAMES = 4096;   /* larger batches are launched */
static constexpr int RES_TIMEOUT_S = 30;           /* no answer: the call fails */

#ifdef XCSUM_DEBUG_BOUNDS
namespace xcsum {
BoundsReader *&bounds_readers()
{
	static BoundsReader *head = nullptr;
	return head;
}
} /* namespace xcsum */

/* Debug build only (make -C libxudp_amd debug): synchronise the device, then
 * collect and clear the bounds-violation logs of every kernel translation
 * unit.  *count = violations since the last call; recs (may be null) gets up
 * to max_recs records of 4 u64 each: {site << 32 | index, addr, lo, hi}. */
extern "C" int xcsum_debug_bounds(uint64_t *count, uint64_t *recs, int max_recs)
{
	if (!count)
		return -XCSUM_ERR_INVAL;
	if (hipDeviceSynchronize() != hipSuccess)
		return -XCSUM_ERR_HIP;
	uint64_t total = 0;
	int k = 0;
	for (BoundsReader *r = bounds_readers(); r; r = r->next) {
		BoundsLog log;
		if (r->take(&log))
			return -XCSUM_ERR_HIP;
		total += log.count;
		for (unsigned i = 0; i < log.count && i < (unsigned)BOUNDS_RECS; i++, k++) {
			if (!recs || k >= max_recs)
				continue;
			recs[4 * k] = ((uint64_t)log.rec[i].site << 32) | log.rec[i].index;
			recs[4 * k + 1] = log.rec[i].addr;
			recs[4 * k + 2] = log.rec[i].lo;
			recs[4 * k + 3] = log.rec[i].hi;
		}
	}
	*count = total;
	return 0;
}
#endif

/* $XCSUM_GEOMETRY="G,U,K" forces a geometry for every new context (sweeps) */
static Geometry env_geometry()
{
	const char *s = getenv("XCSUM_GEOMETRY");
	int G, U, K;
	if (s && sscanf(s, "%d,%d,%d", &G, &U, &K) == 3 && geometry_supported(Geometry{G, U, K, 0}))
		return Geometry{G, U, K, 0};
	return Geometry{0, 0, 0, 0};
}

/* XCSUM_ORDER="R,T": log2 regions, log2 frames per tile (tuning only) */
static void env_order(xcsum_ctx *c)
{
	c->order_rlog = -1;
	c->order_tlog = 0;
	const char *e = getenv("XCSUM_ORDER");
	int r = 0, t = 0;
	if (e && sscanf(e, "%d,%d", &r, &t) == 2 && r >= 0 && r <= 12 && t >= 0 && t <= 16) {
		c->order_rlog = r;
		c->order_tlog = t;
	}
}

/* XCSUM_RESIDENT="W[,idle_us[,max_frames]]": resident workgroups for every
 * new context (xcsum_ctx_set_resident), e.g. for the packet.c mirror's
 * default context */
static void env_resident(xcsum_ctx *c)
{
	c->res_wg = 0;
	c->res_idle_us = RES_IDLE_US;
	c->res_max_frames = RES_MAX_FRAMES;
	c->res_bell = nullptr;
	c->res_vbell = nullptr;
	c->res_done = nullptr;
	c->res_vdone = nullptr;
	c->res_stream = nullptr;
	c->res_live = false;
	c->res_seq = 0;
	c->res_gen = 0;
	c->res_trace = getenv("XCSUM_RESIDENT_TRACE") != nullptr;   /* diagnostic */
	c->res_life_us = RES_LIFE_US;       /* xcsum_ctx_set_resident_life */
	c->res_limit_cut = 0;               /* XCSUM_TUNE_RESIDENT_LIMIT_CUT */
	c->res_inline = true;               /* XCSUM_TUNE_RESIDENT_INLINE */
	c->res_calls = 0;
	c->res_spin_us = c->res_call_us = 0;
	const char *e = getenv("XCSUM_RESIDENT");
	int w = 0;
	unsigned idle = RES_IDLE_US, maxf = RES_MAX_FRAMES;
	if (e && sscanf(e, "%d,%u,%u", &w, &idle, &maxf) >= 1 && w >= 0 && w <= RB_MAX_WG) {
		c->res_wg = w;
		c->res_idle_us = idle ? idle : RES_IDLE_US;
		c->res_max_frames = maxf < RB_DESC_CAP ? maxf : RB_DESC_CAP;
	}
}

static void tuning_defaults(xcsum_ctx *c)
{
	Tuning &t = c->tune;
	t.iphdr_fpt = 4;
	t.build_hdr = true;
	t.build_G = t.build_K = 0;
	t.rx_G = t.rx_K = t.rx_U = t.rx_B = 0;
	t.rx_rlog = -1;
	t.rx_tlog = 0;
	t.gather_ratio = 2;
	t.claim_static_64 = 64;
	t.claim_steps = 16;
	c->inplace_block = 0;
	c->inplace_tl = 1;
}

extern "C" int xcsum_ctx_set_tuning(xcsum_ctx *c, int knob, int a, int b, int cc, int d)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	Tuning &t = c->tune;
	switch (knob) {
	case XCSUM_TUNE_IPHDR_FPT:
		if (a != 1 && a != 2 && a != 4 && a != 8)
			return -XCSUM_ERR_INVAL;
		t.iphdr_fpt = a;
		return 0;
	case XCSUM_TUNE_BUILD_HDR:
		t.build_hdr = a != 0;
		return 0;
	case XCSUM_TUNE_BUILD_GEOMETRY:
		if (a && !build_geometry_supported(a, b))
			return -XCSUM_ERR_INVAL;
		t.build_G = a;
		t.build_K = a ? b : 0;
		return 0;
	case XCSUM_TUNE_RX_GEOMETRY:
		if (a && (!rx_geometry_supported(a, b, cc) || d < 0 || d > 32))
			return -XCSUM_ERR_INVAL;
		t.rx_G = a;
		t.rx_K = a ? b : 0;
		t.rx_U = a ? cc : 0;
		t.rx_B = a ? d : 0;
		return 0;
	case XCSUM_TUNE_RX_ORDER:
		if (a < -1 || a > 12 || (a > 0 && (b < 0 || b > 16)))
			return -XCSUM_ERR_INVAL;
		t.rx_rlog = a;
		t.rx_tlog = a > 0 ? b : 0;
		return 0;
	case XCSUM_TUNE_GATHER_RATIO:
		if (a < 0)
			return -XCSUM_ERR_INVAL;
		t.gather_ratio = a ? (uint32_t)a : 2u;
		return 0;
	case XCSUM_TUNE_INPLACE_BLOCK:
		if (a != 0 && a != 32 && a != 64)
			return -XCSUM_ERR_INVAL;
		c->inplace_block = (uint32_t)a;
		return 0;
	case XCSUM_TUNE_INPLACE_TL:
		c->inplace_tl = a != 0;
		return 0;
	case XCSUM_TUNE_RESIDENT_INLINE:
		c->res_inline = a != 0;
		return 0;
	case XCSUM_TUNE_RESIDENT_LIMIT_CUT:
		if (a < 0)
			return -XCSUM_ERR_INVAL;
		c->res_limit_cut = (uint64_t)a;
		return 0;
	case XCSUM_TUNE_CLAIM:
		/* the claimed-tail kernels are in the A/B build only */
		if (a < 0 || a > 64 || b < 0 || b > 4096 || (a < 64 && !launch_csum_claim_f0))
			return -XCSUM_ERR_INVAL;
		t.claim_static_64 = (uint32_t)a;
		t.claim_steps = b ? (uint32_t)b : 16u;
		return 0;
	default:
		return -XCSUM_ERR_INVAL;
	}
}

#ifdef XCSUM_ENV_TUNING
/* `make variant` only (A/B sweeps by tools/ scripts): the tuning knobs from
 * XCSUM_<KNOB> at context creation.  libxcsum.so itself takes them through
 * xcsum_ctx_set_tuning alone. */
static void read_env_tuning(xcsum_ctx *c)
{
	int a = 0, b = 0, cc = 0, d = 0;
	const char *e;
	if ((e = getenv("XCSUM_IPHDR_FPT")))
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_IPHDR_FPT, atoi(e), 0, 0, 0);
	if ((e = getenv("XCSUM_BUILD_HDR")))
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_BUILD_HDR, atoi(e), 0, 0, 0);
	if ((e = getenv("XCSUM_BUILD_GEOMETRY")) && sscanf(e, "%d,%d", &a, &b) == 2)
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_BUILD_GEOMETRY, a, b, 0, 0);
	a = b = 0;
	if ((e = getenv("XCSUM_RX_GEOMETRY"))) {
		cc = 1;
		d = 0;
		if (sscanf(e, "%d,%d,%d,%d", &a, &b, &cc, &d) >= 2)
			(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_RX_GEOMETRY, a, b, cc, d);
	}
	a = b = 0;
	if ((e = getenv("XCSUM_RX_ORDER"))) {
		b = 6;
		if (sscanf(e, "%d,%d", &a, &b) >= 1)
			(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_RX_ORDER, a, b, 0, 0);
	}
	if ((e = getenv("XCSUM_GATHER_RATIO")))
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_GATHER_RATIO, atoi(e), 0, 0, 0);
	if ((e = getenv("XCSUM_INPLACE_BLOCK")))
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_INPLACE_BLOCK, atoi(e), 0, 0, 0);
	if ((e = getenv("XCSUM_INPLACE_TL")))
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_INPLACE_TL, atoi(e), 0, 0, 0);
	if ((e = getenv("XCSUM_RESIDENT_INLINE")))
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_RESIDENT_INLINE, atoi(e), 0, 0, 0);
	if ((e = getenv("XCSUM_RESIDENT_LIFE_US")) && atoi(e) > 0)
		c->res_life_us = (uint32_t)atoi(e);
	a = 64;
	b = 0;
	if ((e = getenv("XCSUM_CLAIM")) && sscanf(e, "%d,%d", &a, &b) >= 1)
		(void)xcsum_ctx_set_tuning(c, XCSUM_TUNE_CLAIM, a, b, 0, 0);
}
#endif

/* ---- resident server (xcsum_resident.hip) ----------------------------------
 * W workgroups poll a doorbell in pinned host memory; a small host batch is a
 * request written there and a spin on the workgroups' done words instead of
 * a launch and its completion. */

/* A doorbell word, visible to the device after everything written before it
 * (the request and the descriptors): a release store between store fences. */
static inline void bell_store(uint32_t *p, uint32_t v)
{
	__builtin_ia32_sfence();
	__atomic_store_n(p, v, __ATOMIC_RELEASE);
	__builtin_ia32_sfence();
}

/* Ask the workgroups to leave and wait until they have (a no-op when none
 * run).  Every path that synchronises the whole device calls this first:
 * resident workgroups end only on `stop` or after res_idle_us without work. */
static int resident_stop(xcsum_ctx *c)
{
	if (!c->res_bell || !c->res_stream)
		return 0;
	bell_store(&c->res_bell->stop, 1u);
	const hipError_t e = hipStreamSynchronize(c->res_stream);
	bell_store(&c->res_bell->stop, 0u);
	c->res_live = false;
	if (e != hipSuccess) {
		t_hip_err = (int)e;
		t_hip_line = __LINE__;
		return -XCSUM_ERR_HIP;
	}
	return 0;
}

/* A caller stream a device entry point launched this context's work on. */
static void note_stream(xcsum_ctx *c, void *s)
{
	for (void *x : c->streams_used)
		if (x == s)
			return;
	c->streams_used.push_back(s);
}

static void drain_slots(xcsum_ctx *c);
static void reg_trace(const char *what, const void *base, size_t size, const void *dev,
		      int known_before);

/* Wait for everything this context started: its resident workgroups (asked
 * to leave), its host-path slots, and the caller streams its device entry
 * points launched on.  Not hipDeviceSynchronize: another context's resident
 * workgroups leave only after their idle time without a batch, so a
 * device-wide wait lasts as long as that context stays busy.
 * A caller stream destroyed since is skipped (the runtime refuses the
 * handle); any other error is returned. */
static int drain_ctx(xcsum_ctx *c)
{
	int rc = resident_stop(c);
	drain_slots(c);
	for (void *s : c->streams_used) {
		const hipError_t e = hipStreamSynchronize((hipStream_t)s);
		if (e == hipErrorContextIsDestroyed || e == hipErrorInvalidHandle ||
		    e == hipErrorInvalidResourceHandle) {
			(void)hipGetLastError();
			continue;
		}
		if (e != hipSuccess && !rc) {
			t_hip_err = (int)e;
			t_hip_line = __LINE__;
			rc = -XCSUM_ERR_HIP;
		}
	}
	return rc;
}

/* Doorbell memory: the doorbell (request + descriptors) and the done words in
 * pinned, coherent host memory, which the workgroups read over PCIe.  (A
 * doorbell in device memory written through the BAR was measured and
 * dropped: DESIGN.md 5.10.)  Allocated once per process and device and kept
 * for later contexts: contexts come and go (one per test), the memory a
 * resident kernel polls is never freed and reallocated under it. */
struct BellMem {
	int device;
	ResidentBell *h, *d;     /* as the host writes it, as the kernel reads it */
	ResidentDone *done_h, *done_d;
	uint32_t seq, gen;       /* last sequence number / generation issued on it:
				    a later owner continues from there, so no
				    stale view of seq can announce a request */
};
static std::mutex g_bell_mu;
static std::vector<BellMem> g_bell_pool;   /* free doorbells */
static std::vector<ResidentBell *> g_bell_all;   /* every doorbell (host view) */

/* At process exit, every resident workgroup still polling is told to leave
 * (they would anyway, after their idle time): no kernel outlives the
 * process's last call by more than one poll.  Registered after HIP's own
 * initialisation (at the first doorbell), so it runs before HIP's teardown. */
static void bells_stop_at_exit()
{
	/* a thread still inside resident_ensure at exit holds the lock: skip
	 * rather than wait (the workgroups leave after their idle time anyway) */
	if (!g_bell_mu.try_lock())
		return;
	for (ResidentBell *b : g_bell_all)
		bell_store(&b->stop, 1u);
	g_bell_mu.unlock();
}

static int bell_alloc(int device, BellMem *m)
{
	void *d = nullptr, *h = nullptr, *v = nullptr;
	m->device = device;
	if (hipHostMalloc(&h, sizeof(ResidentBell), hipHostMallocCoherent | hipHostMallocMapped) !=
		    hipSuccess)
		return -XCSUM_ERR_NOMEM;
	if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
		(void)hipHostFree(h);
		return -XCSUM_ERR_HIP;
	}
	m->h = (ResidentBell *)h;
	m->d = (ResidentBell *)d;
	h = nullptr;
	if (hipHostMalloc(&h, sizeof(ResidentDone), hipHostMallocCoherent | hipHostMallocMapped) !=
		    hipSuccess ||
	    hipHostGetDevicePointer(&v, h, 0) != hipSuccess) {
		if (h)
			(void)hipHostFree(h);
		(void)hipHostFree(m->h);
		return -XCSUM_ERR_NOMEM;
	}
	m->done_h = (ResidentDone *)h;
	m->done_d = (ResidentDone *)v;
	m->seq = 0;
	m->gen = 0;
	memset(m->h, 0, sizeof(ResidentBell));
	std::lock_guard<std::mutex> g(g_bell_mu);
	if (g_bell_all.empty())
		(void)atexit(bells_stop_at_exit);
	g_bell_all.push_back(m->h);
	return 0;
}

static void resident_free(xcsum_ctx *c)
{
	if (c->res_stream)
		(void)hipStreamDestroy(c->res_stream);
	if (c->res_bell) {
		/* back to the pool; its kernel has left (resident_stop first) */
		std::lock_guard<std::mutex> g(g_bell_mu);
		g_bell_pool.push_back(BellMem{c->device, c->res_bell, c->res_vbell, c->res_done,
					      c->res_vdone, c->res_seq, c->res_gen});
	}
	c->res_stream = nullptr;
	c->res_bell = nullptr;
	c->res_vbell = nullptr;
	c->res_done = nullptr;
	c->res_vdone = nullptr;
	c->res_live = false;
}

static int resident_ensure(xcsum_ctx *c)
{
	if (c->res_bell)
		return 0;
	BellMem m;
	bool have = false;
	{
		std::lock_guard<std::mutex> g(g_bell_mu);
		for (size_t i = 0; i < g_bell_pool.size(); i++)
			if (g_bell_pool[i].device == c->device) {
				m = g_bell_pool[i];
				g_bell_pool.erase(g_bell_pool.begin() + (long)i);
				have = true;
				break;
			}
	}
	if (!have) {
		const int rc = bell_alloc(c->device, &m);
		if (rc)
			return rc;
	}
	if (hipStreamCreateWithFlags(&c->res_stream, hipStreamNonBlocking) != hipSuccess) {
		c->res_stream = nullptr;
		std::lock_guard<std::mutex> g(g_bell_mu);
		g_bell_pool.push_back(m);
		return -XCSUM_ERR_HIP;
	}
	c->res_bell = m.h;
	c->res_vbell = m.d;
	c->res_done = m.done_h;
	c->res_vdone = m.done_d;
	/* no answers or left words of the previous owner (its kernel has
	 * left); sequence numbers and generations continue from its last */
	memset(c->res_done, 0, sizeof(ResidentDone));
	c->res_seq = m.seq;
	c->res_gen = m.gen;
	c->res_live = false;
	return 0;
}

extern "C" int xcsum_ctx_set_resident(xcsum_ctx *c, int workgroups, uint32_t idle_us)
{
	if (!c || workgroups < 0 || workgroups > RB_MAX_WG)
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	/* the running workgroups leave; the next batch launches the new count */
	const int rc = resident_stop(c);
	c->res_wg = workgroups;
	c->res_idle_us = idle_us ? idle_us : RES_IDLE_US;
	if (!workgroups)
		resident_free(c);
	return rc;
}

extern "C" int xcsum_ctx_set_resident_life(xcsum_ctx *c, uint32_t life_us)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	/* the running workgroups leave; the next batch launches them with it */
	const int rc = resident_stop(c);
	c->res_life_us = life_us ? life_us : RES_LIFE_US;
	return rc;
}

/* One request: the batch `a` describes (device addresses of the frames,
 * descriptors and result slots) served by the resident workgroups.  Returns
 * when every workgroup has answered.  A workgroup that left at its idle
 * deadline while the request was on its way is relaunched with the mask of
 * those that did answer (they skip it), so every frame is served once. */
static hipError_t resident_launch(xcsum_ctx *c, uint32_t served0, uint32_t skip_seq,
				  uint64_t skip_mask)
{
	c->res_gen = c->res_gen + 1u ? c->res_gen + 1u : 1u;
	const hipError_t e = launch_resident(c->res_vbell, c->res_vdone, c->d_err, c->res_wg,
					     c->res_gen, served0, skip_seq, skip_mask, c->res_idle_us,
					     c->res_life_us,
					     c->res_stream);
	c->res_live = e == hipSuccess;
	return e;
}

static inline uint32_t done_word(const xcsum_ctx *c, int w, int k)
{
	return __atomic_load_n(&c->res_done->done[RB_DONE_STRIDE * w + k], __ATOMIC_ACQUIRE);
}

/* After every workgroup answered request seq: did one refuse it (a
 * descriptor outside the request's limit, RB_BAD)?  Then the call fails --
 * -XCSUM_ERR_INVAL, the frames' descriptors are the caller's -- and says
 * which on stderr. */
static int resident_bad(const xcsum_ctx *c, uint32_t seq)
{
	for (int w = 0; w < c->res_wg; w++) {
		const uint32_t *o = &c->res_done->done[RB_DONE_STRIDE * w + RB_BAD];
		if (__atomic_load_n(&o[0], __ATOMIC_ACQUIRE) == seq) {
			fprintf(stderr, "xcsum resident: request %u: descriptor %u {addr %#llx, len %u} "
				"outside the frames' buffer\n", seq, o[1],
				(unsigned long long)(((uint64_t)o[3] << 32) | o[2]), o[4]);
			return -XCSUM_ERR_INVAL;
		}
	}
	return 0;
}

static int resident_call(xcsum_ctx *c, const CsumArgs &a, uint64_t limit)
{
	ResidentBell *b = c->res_bell;
	const int W = c->res_wg;
	const uint32_t prev = c->res_seq;
	const uint32_t seq = prev + 1u ? prev + 1u : 1u;
	auto put64 = [&](int k, uint64_t v) {
		b->req[k] = (uint32_t)v;
		b->req[k + 1] = (uint32_t)(v >> 32);
	};
	put64(RB_UMEM, (uint64_t)(uintptr_t)a.umem);
	put64(RB_DESC, (uint64_t)(uintptr_t)a.desc);
	put64(RB_OUT, (uint64_t)(uintptr_t)a.out);
	put64(RB_OUT_IP, (uint64_t)(uintptr_t)a.out_ip);
	put64(RB_BIAS, a.bias);
	b->req[RB_N] = a.n;
	b->req[RB_MODE] = a.mode;
	b->req[RB_FLAGS] = a.flags;
	put64(RB_LIMIT, limit);
	/* the buffers the request may point into (checked by the debug build) */
	b->allow[RB_ALLOW_STAGE] = (uint64_t)(uintptr_t)c->v_stage[0];
	b->allow[RB_ALLOW_STAGE + 1] = (uint64_t)(uintptr_t)c->v_stage[0] + c->frame_cap + 64;
	b->allow[RB_ALLOW_DESC] = (uint64_t)(uintptr_t)c->res_vbell->desc;
	b->allow[RB_ALLOW_DESC + 1] = (uint64_t)(uintptr_t)(c->res_vbell->desc + RB_DESC_CAP);
	b->allow[RB_ALLOW_OUT] = (uint64_t)(uintptr_t)c->v_out[0];
	b->allow[RB_ALLOW_OUT + 1] = (uint64_t)(uintptr_t)c->v_out[0] + 2 * c->desc_cap * sizeof(uint16_t);
	/* a small batch's descriptors also go into the lines the workgroups
	 * poll (three a line, the line's echo after them) */
	if (a.n <= RB_INLINE && c->res_inline)
		for (uint32_t l = 0; l * 3 < a.n; l++) {
			memcpy(b->inl[l], &b->desc[3 * l], 3 * sizeof(struct xcsum_desc));
			bell_store(&b->inl[l][RB_INL_ECHO], seq);
		}
	/* the echo last, after everything else of the request has left the
	 * write-combining buffers: a workgroup that reads the echo equal to seq
	 * has the whole request in the same 64-byte read */
	bell_store(&b->req[RB_SEQ], seq);
	/* a workgroup that left after its idle time says so in its left word:
	 * the others leave at about the same moment -- wait for them, then a
	 * fresh launch (no HIP call while they stay) */
	if (c->res_live)
		for (int w = 0; w < W; w++)
			if (done_word(c, w, RB_LEFT) == c->res_gen) {
				/* the rest are told to leave at once (seq is not
				 * out yet), or they would poll to their deadline */
				const int rc = resident_stop(c);
				if (rc)
					return rc;
				break;
			}
	if (!c->res_live)
		HIPCHK(resident_launch(c, prev, 0u, 0ull));
	bell_store(&b->seq, seq);
	c->res_seq = seq;
	struct SpinTimer {   /* XCSUM_RESIDENT_TRACE */
		xcsum_ctx *c;
		std::chrono::steady_clock::time_point t;
		~SpinTimer()
		{
			if (c->res_trace)
				c->res_spin_us += std::chrono::duration<double, std::micro>(
							  std::chrono::steady_clock::now() - t).count();
		}
	} spin_timer{c, c->res_trace ? std::chrono::steady_clock::now()
				     : std::chrono::steady_clock::time_point()};

	const uint64_t all = W == 64 ? ~0ull : (1ull << W) - 1;
	uint64_t pending = all;
	const auto t0 = std::chrono::steady_clock::now();
	for (uint64_t spin = 1;; spin++) {
		uint64_t gone = 0;
		for (int w = 0; w < W; w++) {
			if (!((pending >> w) & 1ull))
				continue;
			if (done_word(c, w, 0) == seq)
				pending &= ~(1ull << w);
			else if (done_word(c, w, RB_LEFT) == c->res_gen)
				gone |= 1ull << w;
		}
		if (!pending)
			return resident_bad(c, seq);
		if (gone == pending) {
			/* every workgroup still owing an answer left before it saw
			 * the request: once all are gone (and done[] is final),
			 * relaunch; those that answered skip it.  The ones that
			 * answered are told to leave first, or they would poll
			 * until their idle deadline */
			{
				const int rc = resident_stop(c);
				if (rc)
					return rc;
			}
			for (int w = 0; w < W; w++)
				if (((pending >> w) & 1ull) && done_word(c, w, 0) == seq)
					pending &= ~(1ull << w);
			if (!pending)
				return resident_bad(c, seq);
			HIPCHK(resident_launch(c, prev, seq, all & ~pending));
			continue;
		}
		__builtin_ia32_pause();
		if (spin % 65536 == 0) {
			/* a fault, or a device that stopped answering: give up after
			 * RES_TIMEOUT_S rather than spin forever */
			const hipError_t q = hipStreamQuery(c->res_stream);
			if (q != hipErrorNotReady && q != hipSuccess) {
#ifdef XCSUM_DEBUG_BOUNDS
				/* what each workgroup was serving when the grid died */
				for (int w = 0; w < W; w++) {
					const uint32_t *cr = &c->res_done->done[RB_DONE_STRIDE * w + RB_CRUMB];
					fprintf(stderr, "xcsum resident: fault: workgroup %d last request %u "
						"umem %#llx n %u desc %#llx (this request %u)\n", w, cr[0],
						(unsigned long long)(((uint64_t)cr[2] << 32) | cr[1]), cr[3],
						(unsigned long long)(((uint64_t)cr[5] << 32) | cr[4]), seq);
				}
#endif
				c->res_live = false;
				t_hip_err = (int)q;
				t_hip_line = __LINE__;
				return -XCSUM_ERR_HIP;
			}
			if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(RES_TIMEOUT_S)) {
				(void)resident_stop(c);
				t_hip_err = (int)hipErrorLaunchTimeOut;
				t_hip_line = __LINE__;
				return -XCSUM_ERR_HIP;
			}
		}
	}
}

/* ---- device placement (include/xcsum.h) ---------------------------------- */

static std::atomic<unsigned> g_auto_turn{0};   /* XCSUM_DEVICE_AUTO round robin */

extern "C" int xcsum_device_count(void)
{
	int count = 0;
	if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
		return -XCSUM_ERR_NODEV;
	return count;
}

extern "C" int xcsum_device_resolve(int device, int ndev)
{
	if (ndev <= 0) {
		ndev = xcsum_device_count();
		if (ndev < 0)
			return ndev;
	}
	if (device == XCSUM_DEVICE_ENV) {
		/* read when a context is created, never on a batch path */
		const char *e = getenv("XCSUM_DEVICE");
		device = e ? atoi(e) : 0;
		if (device < 0)
			return -XCSUM_ERR_NODEV;
	} else if (device == XCSUM_DEVICE_AUTO) {
		device = (int)(g_auto_turn.fetch_add(1u, std::memory_order_relaxed) % (unsigned)ndev);
	} else if (device <= XCSUM_DEVICE_GROUP(0) && device >= XCSUM_DEVICE_GROUP(1000000)) {
		device = (XCSUM_DEVICE_GROUP(0) - device) % ndev;
	} else if (device < 0) {
		return -XCSUM_ERR_INVAL;
	}
	return device < ndev ? device : -XCSUM_ERR_NODEV;
}

extern "C" int xcsum_ctx_create(int device, xcsum_ctx **out)
{
	if (!out)
		return -XCSUM_ERR_INVAL;
	*out = nullptr;
	const int count = xcsum_device_count();
	if (count < 0)
		return count;
	device = xcsum_device_resolve(device, count);
	if (device < 0)
		return device;
	HIPCHK(hipSetDevice(device));
	xcsum_ctx *c = new (std::nothrow) xcsum_ctx();
	if (!c)
		return -XCSUM_ERR_NOMEM;
	c->device = device;
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
		delete c;
		return -XCSUM_ERR_HIP;
	}
	c->cus = prop.multiProcessorCount;
	c->max_blocks = c->cus * 8;
	c->d_err = nullptr;
	c->d_rx_part = nullptr;
	/* two counters: [0] the caller's (xcsum_ctx_take_errors), [1] where
	 * xcsum_ctx_calibrate_order's calls count theirs */
	if (hipMalloc(&c->d_err, 2 * sizeof(unsigned long long)) != hipSuccess ||
	    hipMalloc(&c->d_rx_part, RX_PART_MAX * sizeof(uint32_t)) != hipSuccess) {
		if (c->d_err)
			(void)hipFree(c->d_err);
		delete c;
		return -XCSUM_ERR_NOMEM;
	}
	(void)hipMemset(c->d_err, 0, 2 * sizeof(unsigned long long));
	for (int s = 0; s < Ctx::NSLOT; s++) {
		c->streams[s] = nullptr;
		c->done[s] = nullptr;
		c->d_frames[s] = nullptr;
		c->d_desc[s] = nullptr;
		c->d_out[s] = nullptr;
		c->h_out[s] = nullptr;
		c->d_rx_msgs[s] = nullptr;
		c->h_rx_msgs[s] = nullptr;
		c->h_stage[s] = nullptr;
		c->h_dstage[s] = nullptr;
		c->v_stage[s] = nullptr;
		c->v_dstage[s] = nullptr;
		c->v_out[s] = nullptr;
		c->v_rx_msgs[s] = nullptr;
	}
	c->frame_cap = 0;
	c->desc_cap = 0;
	c->inplace_sched = XCSUM_INPLACE_AUTO;
	if (const char *e = getenv("XCSUM_INPLACE"))
		c->inplace_sched = strcmp(e, "fused") == 0      ? XCSUM_INPLACE_FUSED
				   : strcmp(e, "two_pass") == 0 ? XCSUM_INPLACE_TWO_PASS
								: XCSUM_INPLACE_AUTO;
	/* XCSUM_TUNE_INPLACE_BLOCK 0|32|64: the second pass's store width (A/B);
	 * 2-byte stores measured fastest in every case (config 2 0.348 vs
	 * 0.364 / 0.353 ms for 32 / 64, config 4 0.332 vs 0.342 / 0.345, xudp's
	 * slots likewise; profiles/r04/inplace/r04wxy_two_pass_widths.txt): the
	 * whole-block variants load the block first */
	tuning_defaults(c);
	c->d_inplace = nullptr;
	c->inplace_cap = 0;
	c->inplace_done = nullptr;
	c->inplace_stream = nullptr;
	c->inplace_recorded = false;
	c->geom = env_geometry();
	c->blocks_per_cu = 0;
	env_order(c);
	env_resident(c);
#ifdef XCSUM_ENV_TUNING
	read_env_tuning(c);
#endif
	c->stage_pool = new (std::nothrow) StagePool();   /* threads start on first use */
	*out = c;
	return 0;
}

static void free_staging(xcsum_ctx *c)
{
	for (int s = 0; s < Ctx::NSLOT; s++) {
		if (c->streams[s]) (void)hipStreamDestroy(c->streams[s]);
		if (c->done[s]) (void)hipEventDestroy(c->done[s]);
		if (c->d_frames[s]) (void)hipFree(c->d_frames[s]);
		if (c->d_desc[s]) (void)hipFree(c->d_desc[s]);
		if (c->d_out[s]) (void)hipFree(c->d_out[s]);
		if (c->h_out[s]) (void)hipHostFree(c->h_out[s]);
		if (c->d_rx_msgs[s]) (void)hipFree(c->d_rx_msgs[s]);
		if (c->h_rx_msgs[s]) (void)hipHostFree(c->h_rx_msgs[s]);
		if (c->h_stage[s]) (void)hipHostFree(c->h_stage[s]);
		if (c->h_dstage[s]) (void)hipHostFree(c->h_dstage[s]);
		c->h_stage[s] = nullptr;
		c->h_dstage[s] = nullptr;
		c->v_stage[s] = nullptr;
		c->v_dstage[s] = nullptr;
		c->v_out[s] = nullptr;
		c->v_rx_msgs[s] = nullptr;
		c->d_rx_msgs[s] = nullptr;
		c->h_rx_msgs[s] = nullptr;
		c->streams[s] = nullptr;
		c->done[s] = nullptr;
		c->d_frames[s] = nullptr;
		c->d_desc[s] = nullptr;
		c->d_out[s] = nullptr;
		c->h_out[s] = nullptr;
	}
	c->frame_cap = 0;
	c->desc_cap = 0;
}

extern "C" int xcsum_ctx_create_for_group(int gid, xcsum_ctx **out)
{
	if (gid < 0 || gid > 1000000)
		return -XCSUM_ERR_INVAL;
	return xcsum_ctx_create(XCSUM_DEVICE_GROUP(gid), out);
}

extern "C" void xcsum_ctx_destroy(xcsum_ctx *c)
{
	if (!c)
		return;
	delete c->stage_pool;   /* joins its copy threads */
	c->stage_pool = nullptr;
	(void)hipSetDevice(c->device);
	if (c->res_trace && c->res_calls)
		fprintf(stderr, "xcsum resident: %llu calls, %.2f us per call, %.2f us of it "
			"from the doorbell store to the last answer\n",
			(unsigned long long)c->res_calls, c->res_call_us / c->res_calls,
			c->res_spin_us / c->res_calls);
	(void)drain_ctx(c);
	resident_free(c);
	free_staging(c);
	for (auto &r : c->regions) {
		if (r.mapped)
			(void)hipHostUnregister(r.reg);
		reg_trace("unregister", r.host, r.size, r.dev, 0);
	}
	if (c->d_err)
		(void)hipFree(c->d_err);
	if (c->d_rx_part)
		(void)hipFree(c->d_rx_part);
	if (c->d_inplace)
		(void)hipFree(c->d_inplace);
	if (c->d_claim)
		(void)hipFree(c->d_claim);
	if (c->inplace_done)
		(void)hipEventDestroy(c->inplace_done);
	delete c;
}

extern "C" int xcsum_ctx_device(const xcsum_ctx *c)
{
	return c ? c->device : -XCSUM_ERR_INVAL;
}

extern "C" int xcsum_ctx_take_errors(xcsum_ctx *c, uint64_t *count)
{
	unsigned long long v = 0;
	if (!c || !count)
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	{
		const int rc = drain_ctx(c);
		if (rc)
			return rc;
	}
	HIPCHK(hipMemcpy(&v, c->d_err, sizeof(v), hipMemcpyDeviceToHost));
	HIPCHK(hipMemset(c->d_err, 0, sizeof(v)));
	*count = v;
	return 0;
}

/* Visiting order of a checksum launch.  Forced (xcsum_ctx_set_order), or
 * automatic: 32 regions of 16-frame tiles if the kernel finds the batch
 * sparse in the UMEM (profiles/r01/order_*.log), else the dense order of
 * the geometry, measured in round 2 (profiles/r02/session2/order_dense/):
 * MTU frames (16,2,6) 8 regions of 16-frame tiles, in the bench config 2
 * 0.2408 -> 0.2338 ms and config 4 0.2415 -> 0.2344 ms (16 regions: 0.2349
 * / 0.2342, 4 regions 0.2375 / 0.2417); mixed sizes (64,1,9) 16 regions of
 * 4-frame tiles, config 5 6.01 -> 5.86 ms; 400-760-byte frames (16,1,2) /
 * (16,1,3) 32 regions of 16-frame tiles, -5 %; 150-byte frames (8,1,2)
 * lose under it and keep descriptor order.  Frames spread over 8-32 places
 * of the batch keep more HBM channels busy than one contiguous window.
 * (Round 1 measured forced region orders 1-4 % slower on packed frames,
 * with the kernel of that time.)  Other geometries keep descriptor order
 * for dense batches. */
static void set_order(const xcsum_ctx *c, CsumArgs &a, const Geometry &g)
{
	if (c->order_rlog >= 0) {
		a.ord = order_regions(a.n, c->order_rlog, c->order_tlog);
		a.dense = a.ord;
		return;
	}
	a.ord = order_regions(a.n, 5, 4);
	/* in place over a sparse batch (libxudp's TX call on its slots): fewer
	 * regions -- in place + IPHDR 16 regions of 32-frame tiles, IPv6 and
	 * IPv4 without IPHDR 8 of 16: 0.3522 -> 0.3467, 0.3533 -> 0.3440 and
	 * 0.3537 -> 0.3472 ms (plain: no order better than 32 x 16; same box,
	 * alternating, profiles/r04/check/r04so_slot_orders.txt) */
	if ((a.flags & XCSUM_F_INPLACE) && g.G == 16 && g.U == 2 && g.K == 6)
		a.ord = (a.flags & XCSUM_F_IPHDR) ? order_regions(a.n, 4, 5) : order_regions(a.n, 3, 4);
	/* VERIFY (dense): descriptor order, config 2 0.2406 -> 0.2382 ms, config
	 * 4 0.2404 -> 0.2378 (alternating, three pairs each; the plain and
	 * in-place passes keep 8 x 16; profiles/r04/check/r04do_dense_orders.txt) */
	if (g.G == 16 && g.U == 2 && g.K == 6 && (a.flags & XCSUM_F_VERIFY))
		a.dense = order_identity(a.n);
	else if (g.G == 16 && g.U == 2 && g.K == 6)
		a.dense = order_regions(a.n, 3, 4);
	else if (g.G == 16 && g.U == 1 && (g.K == 2 || g.K == 3))
		a.dense = order_regions(a.n, 5, 4);   /* 400 / 700-byte payloads:
							 0.0888 -> 0.0842 ms,
							 0.1408 -> 0.1343 ms (s24) */
	else if (g.G == 64 && g.U == 1)
		a.dense = order_regions(a.n, 4, 2);
	else
		a.dense = order_identity(a.n);
	/* resolved in the kernel whenever either order is not the identity: a
	 * batch of 128-511 frames is too small for 32 regions of 16-frame
	 * tiles but still gets its dense order */
	a.ord.sparse_only = a.ord.rshift != 0 || a.dense.rshift != 0;
}

static Geometry geometry_for(const xcsum_ctx *c, uint32_t len_hint, uint32_t flags)
{
	Geometry g = c->geom.G ? c->geom : pick_geometry(len_hint);
	/* MTU frames with the IPv4 header (its own instantiation, 234 VGPRs):
	 * two blocks per CU instead of one, INPLACE | IPHDR 0.383 -> 0.343 ms
	 * packed, 0.404 -> 0.361 on xudp's slots (profiles/r02/flags_bpc/) */
	if (!c->geom.G && (flags & XCSUM_F_IPHDR) && g.G == 16 && g.U == 2 && g.K == 6)
		g.B = 2;
	if (c->blocks_per_cu > 0)
		g.B = c->blocks_per_cu;
	return g;
}

extern "C" int xcsum_ctx_set_geometry(xcsum_ctx *c, int G, int U, int K)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	if (G == 0) {
		c->geom = Geometry{0, 0, 0, 0};
		return 0;
	}
	if (!geometry_supported(Geometry{G, U, K, 0}))
		return -XCSUM_ERR_INVAL;
	c->geom = pick_geometry(0);
	c->geom.G = G;
	c->geom.U = U;
	c->geom.K = K;
	c->geom.B = 0;
	return 0;
}

extern "C" int xcsum_ctx_set_order(xcsum_ctx *c, int region_log2, int tile_log2)
{
	if (!c || region_log2 < -1 || region_log2 > 12 || tile_log2 < 0 || tile_log2 > 16)
		return -XCSUM_ERR_INVAL;
	c->order_rlog = region_log2;
	c->order_tlog = tile_log2;
	return 0;
}

extern "C" int xcsum_ctx_set_launch(xcsum_ctx *c, int blocks_per_cu)
{
	if (!c || blocks_per_cu < 0 || blocks_per_cu > 32)
		return -XCSUM_ERR_INVAL;
	c->blocks_per_cu = blocks_per_cu;
	return 0;
}

/* XCSUM_F_INPLACE in two passes (xcsum_scatter.hip): the checksum pass
 * without INPLACE into d_out (or the context's scratch) and, with IPHDR, the
 * scratch's iph->check half; then the scatter launch stores the fields.
 * *done = false: the caller runs the fused pass instead (a call under
 * stream capture that would need the scratch, see below). */
static int inplace_two_pass(xcsum_ctx *c, const CsumArgs &a, const Geometry &g, hipStream_t s,
			    bool *done)
{
	const bool iph = (a.flags & XCSUM_F_IPHDR) != 0;
	const bool scratch = !a.out || iph;
	hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
	HIPCHK(hipStreamIsCapturing(s, &cs));
	const bool capturing = cs != hipStreamCaptureStatusNone;
	/* A captured graph never references the context's scratch: it would keep
	 * a pointer an eager call may free when the scratch grows, and
	 * its replays could not be ordered against eager two-pass calls through
	 * the context's event.  So a call under capture that needs scratch runs
	 * the fused pass (same bytes); with the caller's d_out and no IPHDR the
	 * two passes need no scratch and are captured as they are. */
	if (scratch && capturing)
		return 0;
	if (scratch && c->inplace_cap < a.n) {
		uint32_t cap = 1u << 16;
		while (cap < a.n)
			cap = cap >= (1u << 31) ? a.n : cap * 2;
		uint16_t *p = nullptr;
		/* hipFree waits for the device: the previous array is idle */
		if (c->d_inplace)
			HIPCHK(hipFree(c->d_inplace));
		c->d_inplace = nullptr;
		c->inplace_cap = 0;
		if (hipMalloc(&p, (size_t)cap * 2 * sizeof(uint16_t)) != hipSuccess)
			return -XCSUM_ERR_NOMEM;
		c->d_inplace = p;
		c->inplace_cap = cap;
	}
	if (scratch) {
		if (!c->inplace_done)
			HIPCHK(hipEventCreateWithFlags(&c->inplace_done, hipEventDisableTiming));
		/* the scratch is the context's: a call on another stream waits for
		 * the last one's second pass */
		if (c->inplace_recorded && c->inplace_stream != (void *)s)
			HIPCHK(hipStreamWaitEvent(s, c->inplace_done, 0));
	}
	CsumArgs b = a;
	b.flags &= ~XCSUM_F_INPLACE;
	b.out = a.out ? a.out : c->d_inplace;
	b.out_ip = iph ? c->d_inplace + c->inplace_cap : nullptr;
	HIPCHK(launch_csum(b, g, c->cus, s));
	ScatterArgs t;
	t.umem = a.umem;
	t.desc = a.desc;
	t.n = a.n;
	t.mode = a.mode;
	t.res = b.out;
	t.res_ip = b.out_ip;
	t.bias = a.bias;
	t.block = c->inplace_block;
	HIPCHK(launch_scatter(t, c->cus, s));
	if (scratch) {
		HIPCHK(hipEventRecord(c->inplace_done, s));
		c->inplace_stream = (void *)s;
		c->inplace_recorded = true;
	}
	*done = true;
	return 0;
}

extern "C" int xcsum_batch_device(xcsum_ctx *c, uint8_t *d_umem, const struct xcsum_desc *d_desc,
				  uint32_t n, uint16_t *d_out, uint32_t mode, uint32_t flags,
				  uint32_t len_hint, void *stream)
{
	if (!c || mode > XCSUM_MODE_AUTO)
		return -XCSUM_ERR_INVAL;
	if (n == 0)
		return 0;
	if (!d_umem || !d_desc || (!d_out && !(flags & XCSUM_F_INPLACE)))
		return -XCSUM_ERR_INVAL;
	if ((flags & XCSUM_F_IPHDR_ONLY) && mode == XCSUM_MODE_V6)
		return -XCSUM_ERR_INVAL;   /* IPv6 has no header checksum */
	HIPCHK(hipSetDevice(c->device));
	note_stream(c, stream);
	CsumArgs a;
	a.umem = d_umem;
	a.desc = d_desc;
	a.n = n;
	a.out = d_out;
	a.out_ip = nullptr;
	a.mode = mode;
	if (flags & XCSUM_F_IPHDR_ONLY) {
		/* libxudp's IPv4 TX call: iph->check alone, no payload byte read
		 * (xcsum_iphdr.hip).  Automatic order: descriptor order, packed
		 * and in xudp's slots alike -- in place, 1M frames, one box, three
		 * interleaved rounds (profiles/r05/iphdr/r05c_sweep.log): slots
		 * 40.4 us vs 43.2-49.3 with 8-32 regions, packed 48.5 vs 49.5-49.9 */
		a.flags = flags & (XCSUM_F_INPLACE | XCSUM_F_VERIFY | XCSUM_F_IPHDR_ONLY);
		a.bias = 0;
		a.err = c->d_err;
		a.ord = c->order_rlog >= 0 ? order_regions(n, c->order_rlog, c->order_tlog)
					   : order_identity(n);
		a.dense = a.ord;
		HIPCHK(launch_iphdr(a, c->tune.iphdr_fpt, (hipStream_t)stream));
		return 0;
	}
	a.flags = flags & (XCSUM_F_INPLACE | XCSUM_F_IPHDR | XCSUM_F_V4_RFC | XCSUM_F_VERIFY);
	if (a.flags & XCSUM_F_VERIFY)
		a.flags &= ~XCSUM_F_INPLACE; /* verifying never writes frames */
	if (mode == XCSUM_MODE_V6)
		a.flags &= ~XCSUM_F_IPHDR;   /* IPv4 only; the lighter kernel */
	a.bias = 0;
	a.err = c->d_err;
	const Geometry g = geometry_for(c, len_hint, a.flags);
	set_order(c, a, g);
	/* AUTO is FUSED: the two-pass schedule measured slower */
	if ((a.flags & XCSUM_F_INPLACE) && c->inplace_sched == XCSUM_INPLACE_TWO_PASS) {
		bool done = false;
		const int rc = inplace_two_pass(c, a, g, (hipStream_t)stream, &done);
		if (rc || done)
			return rc;
	}
	/* in place without the IPv4 header at MTU: temporal loads of the chunks
	 * that hold udp->check (xcsum_csum_tl.hip: config 4 -1.5 %) */
	if ((a.flags & XCSUM_F_INPLACE) && !(a.flags & XCSUM_F_IPHDR) && c->inplace_tl &&
	    g.G == 16 && g.U == 2 && g.K == 6) {
		HIPCHK(launch_csum_inplace_tl(a, g, c->cus, (hipStream_t)stream));
		return 0;
	}
	ClaimParams cp{nullptr, c->tune.claim_static_64, c->tune.claim_steps};
	if (cp.static_64 < 64) {
		/* the claimed tail: a counter pair of the context's ring, zero on
		 * allocation and reset by the last wave of each launch */
		if (!c->d_claim) {
			HIPCHK(hipMalloc((void **)&c->d_claim, 2 * CLAIM_SLOTS * sizeof(uint32_t)));
			HIPCHK(hipMemset(c->d_claim, 0, 2 * CLAIM_SLOTS * sizeof(uint32_t)));
		}
		cp.claim = c->d_claim + 2 * (c->claim_seq++ % CLAIM_SLOTS);
	}
	HIPCHK(launch_csum(a, g, c->cus, (hipStream_t)stream, &cp));
	return 0;
}

/* Calibrate the visiting order once per context, on the caller's own batch
 * (a box whose HBM prefers another order than the ones
 * measured here).  First the clocks are brought up (>= CAL_WARM_MS of
 * back-to-back calls: a cold GPU runs its first ~100 ms slow, which would
 * reward whichever order happens to run later).  Then the automatic order
 * and six forced ones (descriptor order; 8, 16, 4, 32 and 16 regions of
 * 16/16/32/16/32-frame tiles) are timed in CAL_ROUNDS rounds, each round in a
 * rotated sequence; a time is the median of CAL_REPS samples of >= CAL_SAMPLE_MS
 * of back-to-back calls between two events.  A forced order is kept only if
 * it beats the automatic one by CAL_MARGIN in every round (noise between
 * repeats is ~0.3 %; a kernel the order does not affect, like the
 * small-frame stream kernel, never qualifies).  The calls are ordinary
 * xcsum_batch_device calls with the caller's arguments: results and
 * in-place fields are what any call writes.  Synchronous. */
static const int CAL_ROUNDS = 3, CAL_REPS = 3;
static const float CAL_WARM_MS = 60.0f, CAL_SAMPLE_MS = 2.0f;
static const float CAL_MARGIN = 0.99f;

extern "C" int xcsum_ctx_calibrate_order(xcsum_ctx *c, uint8_t *d_umem,
					 const struct xcsum_desc *d_desc, uint32_t n, uint16_t *d_out,
					 uint32_t mode, uint32_t flags, uint32_t len_hint, void *stream,
					 int *region_log2, int *tile_log2)
{
	if (!c || !d_umem || !d_desc || n == 0)
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
	HIPCHK(hipStreamIsCapturing((hipStream_t)stream, &cs));
	if (cs != hipStreamCaptureStatusNone)
		return -XCSUM_ERR_INVAL;   /* timing inside a capture means nothing */
	static const int cand[][2] = {{-1, 0}, {0, 0}, {3, 4}, {4, 4}, {2, 5}, {5, 4}, {4, 5}};
	constexpr int NC = (int)(sizeof(cand) / sizeof(cand[0]));
	const int old_r = c->order_rlog, old_t = c->order_tlog;
	/* the calls' malformed frames go to the calibration counter, not the
	 * caller's (thousands of repeats inflated take_errors) */
	unsigned long long *const err_keep = c->d_err;
	c->d_err = err_keep + 1;
	struct ErrRestore {
		xcsum_ctx *c;
		unsigned long long *keep;
		~ErrRestore() { c->d_err = keep; }
	} err_restore{c, err_keep};
	hipEvent_t e0 = nullptr, e1 = nullptr;
	int rc = 0;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
		rc = -XCSUM_ERR_HIP;
	/* ms per call over `per` back-to-back calls */
	auto sample = [&](int per, float *ms) -> int {
		if (hipEventRecord(e0, (hipStream_t)stream) != hipSuccess)
			return -XCSUM_ERR_HIP;
		for (int i = 0; i < per; i++) {
			const int r = xcsum_batch_device(c, d_umem, d_desc, n, d_out, mode, flags,
							 len_hint, stream);
			if (r)
				return r;
		}
		float t = 0;
		if (hipEventRecord(e1, (hipStream_t)stream) != hipSuccess ||
		    hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t, e0, e1) != hipSuccess)
			return -XCSUM_ERR_HIP;
		*ms = t / (float)per;
		return 0;
	};
	float t1 = 0;
	int per = 1;
	c->order_rlog = -1;
	c->order_tlog = 0;
	if (!rc)
		rc = sample(3, &t1);
	if (!rc) {
		t1 = std::max(t1, 1e-4f);
		per = (int)std::min(2000.0f, std::max(3.0f, CAL_SAMPLE_MS / t1 + 1.0f));
		const int warm = (int)std::min(20000.0f, CAL_WARM_MS / t1 + 1.0f);
		rc = sample(warm, &t1);
	}
	float ms[CAL_ROUNDS][NC];
	for (int round = 0; round < CAL_ROUNDS && !rc; round++)
		for (int j = 0; j < NC && !rc; j++) {
			const int k = (j + round) % NC;
			c->order_rlog = cand[k][0];
			c->order_tlog = cand[k][1];
			float rep[CAL_REPS];
			rc = sample(1, &rep[0]);   /* the new order's first call */
			for (int r = 0; r < CAL_REPS && !rc; r++)
				rc = sample(per, &rep[r]);
			if (!rc) {
				std::sort(rep, rep + CAL_REPS);
				ms[round][k] = rep[CAL_REPS / 2];
			}
		}
	if (e0)
		(void)hipEventDestroy(e0);
	if (e1)
		(void)hipEventDestroy(e1);
	if (rc) {
		c->order_rlog = old_r;
		c->order_tlog = old_t;
		return rc;
	}
	int pick = 0;
	float pick_sum = 0;
	for (int k = 1; k < NC; k++) {
		bool wins = true;
		float sum = 0;
		for (int round = 0; round < CAL_ROUNDS; round++) {
			wins = wins && ms[round][k] < CAL_MARGIN * ms[round][0];
			sum += ms[round][k];
		}
		if (wins && (!pick || sum < pick_sum)) {
			pick = k;
			pick_sum = sum;
		}
	}
	c->order_rlog = cand[pick][0];
	c->order_tlog = cand[pick][1];
	if (region_log2)
		*region_log2 = c->order_rlog;
	if (tile_log2)
		*tile_log2 = c->order_tlog;
	return 0;
}

extern "C" int xcsum_ctx_set_inplace(xcsum_ctx *c, int schedule)
{
	if (!c || schedule < XCSUM_INPLACE_AUTO || schedule > XCSUM_INPLACE_TWO_PASS)
		return -XCSUM_ERR_INVAL;
	c->inplace_sched = schedule;
	return 0;
}

extern "C" int xcsum_rx_device(xcsum_ctx *c, const uint8_t *d_umem, const struct xcsum_desc *d_desc,
			       uint32_t n, struct xcsum_rx_msg *d_msgs, uint32_t *d_count,
			       uint32_t flags, uint32_t len_hint, void *stream)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	if (n && (!d_umem || !d_desc || !d_msgs))
		return -XCSUM_ERR_INVAL;
	if ((uintptr_t)d_umem & 3u)   /* chunk grid: see xcsum_rx.hip */
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	if (n == 0) {
		if (d_count)
			HIPCHK(hipMemsetAsync(d_count, 0, sizeof(uint32_t), (hipStream_t)stream));
		return 0;
	}
	RxArgs a;
	a.umem = d_umem;
	a.desc = d_desc;
	a.n = n;
	a.flags = flags & (XCSUM_F_VERIFY | XCSUM_F_IPHDR);
	a.msgs = d_msgs;
	a.count = d_count;
	a.part = c->d_rx_part;
	note_stream(c, stream);
	HIPCHK(launch_rx(a, len_hint, c->cus, c->tune, (hipStream_t)stream));
	return 0;
}

/* The 64-byte header template of a batch: every header byte that does not
 * depend on the frame (packet.c:141-150 eth_build, :68-84 iph_build,
 * :92-103 iph_build6, :119-126 udp_build), length and check fields 0.  Plain
 * field stores, no checksum arithmetic. */
static void header_template(const struct xcsum_route *r, uint8_t t[64])
{
	memset(t, 0, 64);
	memcpy(t, r->dmac, 6);
	memcpy(t + 6, r->smac, 6);
	if (r->family == 6) {
		t[12] = 0x86;
		t[13] = 0xDD;
		/* ip6_flow_hdr(iph6, 0, (0x3 << 16) + sin6_port), packet.c:96 */
		uint32_t flow = 0x60000000u | ((0x3u << 16) + r->sport_be);
		t[14] = (uint8_t)(flow >> 24);
		t[15] = (uint8_t)(flow >> 16);
		t[16] = (uint8_t)(flow >> 8);
		t[17] = (uint8_t)flow;
		t[20] = 17;  /* nexthdr */
		t[21] = 64;  /* hop_limit */
		memcpy(t + 22, r->saddr, 16);
		memcpy(t + 38, r->daddr, 16);
		memcpy(t + 54, &r->sport_be, 2);
		memcpy(t + 56, &r->dport_be, 2);
	} else {
		t[12] = 0x08;
		t[14] = 0x45;  /* IP_VIT */
		t[20] = 0x40;  /* IP_DF */
		t[22] = 64;    /* IP_XUDP_TTL */
		t[23] = 17;    /* IPPROTO_UDP */
		memcpy(t + 26, r->saddr, 4);
		memcpy(t + 30, r->daddr, 4);
		memcpy(t + 34, &r->sport_be, 2);
		memcpy(t + 36, &r->dport_be, 2);
	}
}

extern "C" int xcsum_build_device(xcsum_ctx *c, const struct xcsum_route *route,
				  const uint8_t *d_src, const struct xcsum_msg *d_msgs, uint32_t n,
				  uint8_t *d_umem, uint32_t frame_size, uint32_t data_off,
				  struct xcsum_desc *d_desc_out, uint16_t *d_out, uint32_t flags,
				  uint32_t len_hint, void *stream)
{
	if (!c || !route || (route->family != 4 && route->family != 6))
		return -XCSUM_ERR_INVAL;
	if (n == 0)
		return 0;
	const uint32_t hdr = route->family == 6 ? 62u : 42u;
	if (!d_msgs || !d_umem || !d_desc_out || (((uintptr_t)d_umem) & 15) ||
	    (frame_size & 15) || (data_off & 15) || data_off < hdr || data_off >= frame_size ||
	    (!(flags & XCSUM_F_BUILD_INPLACE) && !d_src))
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	BuildArgs a;
	a.umem = d_umem;
	a.src = d_src;
	a.msgs = d_msgs;
	a.n = n;
	a.frame_size = frame_size;
	a.data_off = data_off;
	a.flags = flags & (XCSUM_F_V4_RFC | XCSUM_F_BUILD_INPLACE | XCSUM_F_SRC_ALIGNED);
	a.desc_out = d_desc_out;
	a.out = d_out;
	a.err = c->d_err;
	a.family = route->family;
	header_template(route, (uint8_t *)a.tmpl);
	if (c->order_rlog >= 0) {
		a.ord = order_regions(n, c->order_rlog, c->order_tlog);
	} else {
		/* automatic: the frames are sparse when a slot is at least twice
		 * the frame (xudp: 4096-byte chunks, ~1.5 KB frames) -- then 32
		 * regions of 16-message tiles, as for the checksum kernel */
		const uint32_t typ = hdr + (len_hint ? len_hint : 1472u);
		a.ord = frame_size >= 2u * typ ? order_regions(n, 5, 4) : order_identity(n);
	}
	note_stream(c, stream);
	HIPCHK(launch_build(a, len_hint, c->cus, c->tune, (hipStream_t)stream));
	return 0;
}

extern "C" int xcsum_sync(xcsum_ctx *c, void *stream)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipStreamSynchronize((hipStream_t)stream));
	return 0;
}

/* ---- UMEM registration --------------------------------------------------- */

/* XCSUM_REG_TRACE=<file>: one line per registration and unregistration
 * (diagnostic of the registered-memory faults): the host range,
 * its page range, the device alias the runtime returned, whether the runtime
 * already knew the address before the call, the VMA flags of the pages
 * (locked "lo", THP "hg"/"nh", from /proc/self/smaps), and whether the device
 * alias overlaps one handed out by an earlier, since unregistered,
 * registration of this process (a recycled GPU virtual range). */
static std::mutex g_reg_mu;
struct DevRange {
	uintptr_t lo, hi;
};
static std::vector<DevRange> g_reg_freed;   /* device ranges of past registrations */

static void vma_flags(uintptr_t lo, uintptr_t hi, char *out, size_t cap)
{
	out[0] = 0;
	FILE *f = fopen("/proc/self/smaps", "r");
	if (!f)
		return;
	char line[512];
	uintptr_t s = 0, e = 0;
	unsigned long thp_kb = 0;
	size_t used = 0;
	while (fgets(line, sizeof line, f)) {
		unsigned long a, b;
		if (sscanf(line, "%lx-%lx ", &a, &b) == 2 && strchr(line, '-') < strchr(line, ' ')) {
			s = a;
			e = b;
			thp_kb = 0;
			continue;
		}
		(void)sscanf(line, "AnonHugePages: %lu kB", &thp_kb);
		if (strncmp(line, "VmFlags:", 8) == 0 && s < hi && e > lo) {
			line[strcspn(line, "\n")] = 0;
			const int k = snprintf(out + used, cap - used, "[%lx-%lx:%s thp_kb=%lu]",
					       (unsigned long)s, (unsigned long)e, line + 8, thp_kb);
			if (k > 0 && used + (size_t)k < cap)
				used += (size_t)k;
		}
	}
	fclose(f);
}

/* What ROCr knows about the allocation holding p: its type, host base and
 * size ("%d:%p+%zu"), for the trace; *lo / *sz get the locked extent. */
static int rocr_extent(const void *p, uintptr_t *lo, size_t *sz)
{
	hsa_amd_pointer_info_t info;
	memset(&info, 0, sizeof info);
	info.size = sizeof info;
	if (hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS)
		return -1;
	*lo = (uintptr_t)info.hostBaseAddress;
	*sz = info.sizeInBytes;
	return (int)info.type;
}

static void reg_trace(const char *what, const void *base, size_t size, const void *dev,
		      int known_before)
{
	const char *path = getenv("XCSUM_REG_TRACE");
	std::lock_guard<std::mutex> g(g_reg_mu);
	const uintptr_t plo = (uintptr_t)base & ~(uintptr_t)4095;
	const uintptr_t phi = ((uintptr_t)base + size + 4095) & ~(uintptr_t)4095;
	const uintptr_t dlo = (uintptr_t)dev & ~(uintptr_t)4095;
	const uintptr_t dhi = dlo + (phi - plo);
	bool recycled = false;
	if (what[0] == 'r')
		for (const DevRange &r : g_reg_freed)
			recycled |= r.lo < dhi && r.hi > dlo;
	else if (dev) {
		g_reg_freed.push_back(DevRange{dlo, dhi});
		if (g_reg_freed.size() > 4096)
			g_reg_freed.erase(g_reg_freed.begin());
	}
	if (!path)
		return;
	char flags[1024];
	vma_flags(plo, phi, flags, sizeof flags);
	uintptr_t xl = 0;
	size_t xs = 0;
	const int xt = rocr_extent(base, &xl, &xs);
	if (FILE *f = fopen(path, "a")) {
		fprintf(f, "%s host=%p size=%zu pages=[%#lx,%#lx) dev=%p known_before=%d "
			   "recycled_dev=%d rocr_now=%d:%#lx+%zu vma=%s\n",
			what, base, size, (unsigned long)plo, (unsigned long)phi, dev, known_before,
			(int)recycled, xt, (unsigned long)xl, xs, flags);
		fclose(f);
	}
}

/* Can the kernel move the pages of [lo, hi) under a GPU mapping?  The
 * policy and its smaps parser are in xcsum_thp.h; here the process-wide
 * inputs: THP disabled for the process (PR_GET_THP_DISABLE), the sysfs
 * modes, /proc/self/smaps.  Read once per registration (include/xcsum.h). */
/* the bracketed word of a THP sysfs setting ("always", "never", ...) */
static bool thp_mode_is(const char *path, const char *word)
{
	char buf[160] = {0}, want[32];
	snprintf(want, sizeof want, "[%s]", word);
	FILE *f = fopen(path, "r");
	if (!f)
		return false;
	const bool got = fgets(buf, sizeof buf, f) != nullptr;
	fclose(f);
	return got && strstr(buf, want) != nullptr;
}

static bool thp_eligible(uintptr_t lo, uintptr_t hi)
{
	if (prctl(PR_GET_THP_DISABLE, 0, 0, 0, 0) == 1)
		return false;
	/* private anonymous memory: "enabled"; shared (shmem, anon_map's
	 * MAP_SHARED | MAP_ANONYMOUS): "shmem_enabled" */
	const char *en = "/sys/kernel/mm/transparent_hugepage/enabled";
	const char *sh = "/sys/kernel/mm/transparent_hugepage/shmem_enabled";
	ThpModes m;
	m.never = thp_mode_is(en, "never");
	m.always = thp_mode_is(en, "always");
	m.sh_always = thp_mode_is(sh, "always") || thp_mode_is(sh, "force") ||
		      thp_mode_is(sh, "within_size");
	m.sh_advise = thp_mode_is(sh, "advise");
	FILE *f = fopen("/proc/self/smaps", "r");
	if (!f)
		return true;   /* cannot tell: assume the worst */
	const bool eligible = thp_eligible_smaps(f, lo, hi, m);   /* xcsum_thp.h */
	fclose(f);
	return eligible;
}

extern "C" int xcsum_register_umem(xcsum_ctx *c, void *base, size_t size)
{
	void *dev = nullptr;
	if (!c || !base || !size)
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	/* did the runtime know this address already (a registration or pinning
	 * that was never released)?  Trace only. */
	hipPointerAttribute_t pa;
	const bool known = hipPointerGetAttributes(&pa, base) == hipSuccess &&
			   pa.type != hipMemoryTypeUnregistered;
	(void)hipGetLastError();
	const uintptr_t plo = (uintptr_t)base & ~(uintptr_t)4095;
	const uintptr_t phi = ((uintptr_t)base + size + 4095) & ~(uintptr_t)4095;
	const char *force = getenv("XCSUM_REG_ALLOW_THP");   /* diagnostic */
	if (!(force && strcmp(force, "1") == 0) && thp_eligible(plo, phi)) {
		/* kept for bookkeeping, never mapped: batches in it are staged */
		reg_trace("register_staged", base, size, nullptr, known);
		c->regions.push_back(Region{(uint8_t *)base, size, nullptr, nullptr, false});
		return 0;
	}
	if (hipHostRegister(base, size, hipHostRegisterMapped) != hipSuccess)
		return -XCSUM_ERR_HIP;
	if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
		(void)hipHostUnregister(base);
		return -XCSUM_ERR_HIP;
	}
	reg_trace("register", base, size, dev, known);
	c->regions.push_back(Region{(uint8_t *)base, size, (uint8_t *)dev, (uint8_t *)base, true});
	return 0;
}

extern "C" int xcsum_umem_mapped(xcsum_ctx *c, const void *base)
{
	if (!c || !base)
		return -XCSUM_ERR_INVAL;
	for (auto &r : c->regions)
		if (r.host == (const uint8_t *)base)
			return r.mapped ? 1 : 0;
	return -XCSUM_ERR_NOT_REGISTERED;
}

extern "C" int xcsum_unregister_umem(xcsum_ctx *c, void *base)
{
	if (!c || !base)
		return -XCSUM_ERR_INVAL;
	for (size_t i = 0; i < c->regions.size(); i++) {
		if (c->regions[i].host == (uint8_t *)base) {
			HIPCHK(hipSetDevice(c->device));
			/* no kernel or copy of this context may still read or write
			 * the region once it is unmapped: its resident workgroups,
			 * its host-path streams and the streams its device entry
			 * points ran on (the region's device alias may have been
			 * handed to them) */
			(void)drain_ctx(c);
			if (c->regions[i].mapped)
				(void)hipHostUnregister(c->regions[i].reg);
			reg_trace("unregister", base, c->regions[i].size, c->regions[i].dev, 0);
			c->regions.erase(c->regions.begin() + i);
			return 0;
		}
	}
	return -XCSUM_ERR_NOT_REGISTERED;
}

/* the GPU-mapped registered region holding [lo, hi), or null */
static const Region *find_region(const xcsum_ctx *c, const uint8_t *lo, const uint8_t *hi)
{
	for (auto &r : c->regions)
		if (r.mapped && lo >= r.host && hi <= r.host + r.size)
			return &r;
	return nullptr;
}

/* any registered region holding [lo, hi), mapped or staged */
static bool in_any_region(const xcsum_ctx *c, const uint8_t *lo, const uint8_t *hi)
{
	for (auto &r : c->regions)
		if (lo >= r.host && hi <= r.host + r.size)
			return true;
	return false;
}

/* ---- host-resident batches ----------------------------------------------- */

/* Gathered batches of at most this many staged bytes skip the copies: the
 * kernel reads the pinned stage and writes the pinned result slot over PCIe,
 * so a call is one launch and one wait instead of three transfers, a launch
 * and a wait.  TX ring harness, same call (profiles/r02/session2/host_direct):
 * 1 frame 24.5 -> 20.4 us per call (IPv6 26.7 -> 21.3), 100 frames 24.4 ->
 * 21.5 us (IPv6 37.7 -> 30.5), 1024 IPv4 header-only frames 53 -> 38 us.
 * A launch plus its completion is the floor (~19 us here, zero-copy calls of
 * one frame).  0 disables. */
#ifndef XCSUM_DIRECT_MAX
#define XCSUM_DIRECT_MAX (256u << 10)
#endif
static constexpr uint64_t DIRECT_MAX = XCSUM_DIRECT_MAX;
static constexpr bool DIRECT_ON = DIRECT_MAX != 0;

/* a slot's completion (polling the event instead measured no faster,
 * profiles/r02/session2/host_direct) */
static hipError_t wait_slot(hipEvent_t e)
{
	return hipEventSynchronize(e);
}

/* The pinned stage, its descriptors and the result slots are read and
 * written by kernels directly on the copy-free path: allocate them coherent
 * (uncached on the GPU side), so that a slot reused by the next call never
 * serves lines a previous kernel cached, whatever HIP_HOST_COHERENT says. */
#define PINNED_FLAGS hipHostMallocCoherent

static int ensure_staging(xcsum_ctx *c)
{
	if (c->frame_cap)
		return 0;
	const size_t frame_cap = 32u << 20;   /* bytes of UMEM per chunk */
	const uint32_t desc_cap = 1u << 16;   /* frames per chunk */
	for (int s = 0; s < Ctx::NSLOT; s++) {
		if (hipStreamCreateWithFlags(&c->streams[s], hipStreamNonBlocking) != hipSuccess ||
		    hipEventCreateWithFlags(&c->done[s], hipEventDisableTiming) != hipSuccess ||
		    hipMalloc(&c->d_frames[s], frame_cap + 64) != hipSuccess ||
		    hipMalloc(&c->d_desc[s], desc_cap * sizeof(struct xcsum_desc)) != hipSuccess ||
		    hipMalloc(&c->d_out[s], 2 * desc_cap * sizeof(uint16_t)) != hipSuccess ||
		    hipHostMalloc(&c->h_out[s], 2 * desc_cap * sizeof(uint16_t), PINNED_FLAGS) != hipSuccess) {
			free_staging(c);
			return -XCSUM_ERR_NOMEM;
		}
	}
	c->frame_cap = frame_cap;
	c->desc_cap = desc_cap;
	return 0;
}

/* Pinned stage for gathered frames and their descriptors, and the device
 * addresses the copy-free path hands the kernel (stage, descriptors, result
 * slot).  After ensure_staging. */
static int ensure_gather(xcsum_ctx *c)
{
	for (int s = 0; s < Ctx::NSLOT; s++) {
		/* + 64: a range copy is up to frame_cap + 15 bytes (16-aligned start) */
		if (!c->h_stage[s] && hipHostMalloc(&c->h_stage[s], c->frame_cap + 64, PINNED_FLAGS) != hipSuccess)
			return -XCSUM_ERR_NOMEM;
		if (!c->h_dstage[s] &&
		    hipHostMalloc(&c->h_dstage[s], c->desc_cap * sizeof(struct xcsum_desc), PINNED_FLAGS) !=
			    hipSuccess)
			return -XCSUM_ERR_NOMEM;
		if (DIRECT_ON && !c->v_stage[s] &&
		    (hipHostGetDevicePointer((void **)&c->v_stage[s], c->h_stage[s], 0) != hipSuccess ||
		     hipHostGetDevicePointer((void **)&c->v_dstage[s], c->h_dstage[s], 0) != hipSuccess ||
		     hipHostGetDevicePointer((void **)&c->v_out[s], c->h_out[s], 0) != hipSuccess)) {
			c->v_stage[s] = nullptr;
			return -XCSUM_ERR_HIP;
		}
	}
	return 0;
}

/* Gather a host batch frame by frame (one host memcpy per frame into the
 * pinned stage, gather_frames) instead of copying the UMEM range it spans,
 * when the frames fill less than half of that range and the UMEM is
 * pageable.  A registered UMEM keeps the range copy (pure DMA, no host
 * memcpy).  Measured on xudp's 4096-byte chunks, pageable
 * (tools/bench_e2e.py --layout umem): round 2, one thread
 * (profiles/r02/session2/rx_gather/): 64-byte frames 23.3 -> 6.9 ms per
 * 256K-frame receive batch, MTU frames 22.7 -> 33.6 ms, hence a 1/8 rule;
 * round 5, the copies and the in-place stores split over STAGE_THREADS
 * threads, same-run A/B against the one-thread library
 * (profiles/r05/host/r05v_*): 256K MTU frames gathered instead of
 * range-copied, TX 20.3 -> 14.3 ms, in place 24.2 -> 12.2, receive 23.2 ->
 * 11.4; 64-byte frames TX 4.7 -> 3.8, in place 9.5 -> 4.9, receive 5.8 ->
 * 3.9; the ratio is the context's Tuning::gather_ratio (2; A/B through
 * XCSUM_TUNE_GATHER_RATIO). */
static bool gather_pays(const xcsum_ctx *c, const uint8_t *h_umem, uint64_t lo, uint64_t hi,
			uint64_t frame_bytes)
{
	return hi - lo > (uint64_t)c->tune.gather_ratio * frame_bytes + 4096 &&
	       !find_region(c, h_umem + lo, h_umem + hi);
}

/* A sparse batch in a registered UMEM (the frames fill less than half of
 * the range they span) is read in place (zero-copy) even without
 * XCSUM_F_ZEROCOPY: the range copy moves the gaps over PCIe too.  Results
 * are the same bytes either way.  256K frames in 4096-byte chunks
 * (profiles/r02/session2/rx_gather/): 64-byte frames 20 ms copied, 1.5 ms in
 * place (checksum), 22.5 / 2.9 ms (receive); MTU frames 19.6 / 7.6-8.5 ms,
 * 22.6 / 9.5 ms.  Dense batches keep the copy (packed MTU frames: 31.9 ms
 * copied, 39.2 ms in place).  Returns the region, or null. */
static const Region *zerocopy_pays(const xcsum_ctx *c, const uint8_t *h_umem,
				   const struct xcsum_desc *h_desc, uint32_t n)
{
	uint64_t lo = UINT64_MAX, hi = 0, sum = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (h_desc[i].addr < lo) lo = h_desc[i].addr;
		if (h_desc[i].addr + h_desc[i].len > hi) hi = h_desc[i].addr + h_desc[i].len;
		sum += h_desc[i].len;
	}
	if (n == 0 || hi - lo <= 2 * sum + 4096)
		return nullptr;
	return find_region(c, h_umem + lo, h_umem + hi);
}

/* The source of a host-to-device copy of caller memory [p, p + n): the
 * memory itself when it lies in a registered region (page-locked by
 * xcsum_register_umem: the DMA reads it in place), else a copy in the slot's
 * pinned stage.  Unregistered (pageable) caller memory is never handed to
 * the copy engine: for copies of 1 MiB and more the HIP runtime pins such
 * memory in place (tools/diag_pinning.py: "HSA Copy Using Pinned resource"
 * from 1.5 MB up), and a pinning that outlives the caller's buffer -- freed,
 * its addresses handed to another buffer -- is the likely cause of the
 * illegal-address faults of DESIGN.md 6.  The slot's
 * previous copy has completed (its event was waited for) before the stage
 * is overwritten. */
static const void *host_dma_src(xcsum_ctx *c, int slot, const uint8_t *p, uint64_t n)
{
	if (find_region(c, p, p + n))
		return p;
	stage_copy(c->stage_pool, c->h_stage[slot], p, n);
	return c->h_stage[slot];
}

/* the same for a descriptor range (up to 1 MiB per chunk) */
static const void *host_desc_src(xcsum_ctx *c, int slot, const struct xcsum_desc *d, uint32_t n)
{
	const uint8_t *p = (const uint8_t *)d;
	if (find_region(c, p, p + (uint64_t)n * sizeof(*d)))
		return d;
	memcpy(c->h_dstage[slot], d, (size_t)n * sizeof(*d));
	return c->h_dstage[slot];
}

/* udp->check / iph->check offsets of a frame for the resolved family */
static int host_family(const uint8_t *eth, uint32_t mode)
{
	if (mode == XCSUM_MODE_V6)
		return 6;
	if (mode != XCSUM_MODE_AUTO)
		return 4;
	uint32_t proto = ((uint32_t)eth[12] << 8) | eth[13];
	return proto == 0x86DDu ? 6 : (proto == 0x0800u ? 4 : 0);
}

struct Pending {
	uint32_t first, count;
	bool busy;
	bool gathered;   /* receive: records hold staged offsets, to be fixed up */
};

/* results of one finished chunk -> caller arrays / host frames.  The
 * in-place stores touch one line per frame: from 16384 frames up they are
 * split over up to STAGE_THREADS threads, as the gathers. */
static void retire(StagePool *pool, const Pending &pd, const uint16_t *h_res, uint8_t *h_umem,
		   const struct xcsum_desc *h_desc, uint16_t *h_out, uint16_t *h_out_ip,
		   uint32_t mode, uint32_t flags)
{
	const uint16_t *res = h_res, *res_ip = h_res + pd.count;
	if (h_out)
		memcpy(h_out + pd.first, res, pd.count * sizeof(uint16_t));
	if (h_out_ip)
		memcpy(h_out_ip + pd.first, res_ip, pd.count * sizeof(uint16_t));
	if (!(flags & XCSUM_F_INPLACE))
		return;
	auto store = [&](uint32_t i0, uint32_t i1) {
		for (uint32_t i = i0; i < i1; i++) {
			const struct xcsum_desc &d = h_desc[pd.first + i];
			uint8_t *eth = h_umem + d.addr;
			int fam = host_family(eth, mode);
			/* frames the kernel rejects as malformed (resolve(): too short
			 * for the headers, or a UDP length past 16 bits) are left
			 * untouched, as on the device path: for a truncated frame the
			 * check field's offset may lie in the next frame */
			const uint32_t hdr = fam == 6 ? 54u : 34u;
			if (d.len < hdr + 8u || d.len - hdr > 65535u)
				continue;
			if (flags & XCSUM_F_IPHDR_ONLY) {
				if (fam == 4)                    /* iph->check only */
					memcpy(eth + 24, &res[i], 2);
			} else if (fam == 6) {
				memcpy(eth + 60, &res[i], 2);
			} else if (fam == 4) {
				memcpy(eth + 40, &res[i], 2);
				if (flags & XCSUM_F_IPHDR)
					memcpy(eth + 24, &res_ip[i], 2);
			}
		}
	};
	const int nt = stage_threads(0, pd.count);
	if (nt <= 1) {
		store(0, pd.count);
		return;
	}
	const uint32_t part = (pd.count + nt - 1) / nt;
	stage_run(pool, nt, [&](int t) {
		const uint32_t i0 = part * t < pd.count ? part * t : pd.count;
		const uint32_t i1 = part * (t + 1) < pd.count ? part * (t + 1) : pd.count;
		store(i0, i1);
	});
}

/* Wait for everything the host path queued on the context's streams.  Every
 * host entry point calls it before an error return: a slot still in flight
 * reads the caller's UMEM (registered, or pinned in place by the copy) or the
 * pinned stage, and writes the pinned result slot -- the caller may unmap
 * the UMEM, and the next call reuses the slots, as soon as we return.
 * Errors are ignored: the caller already gets the first one. */
static void drain_slots(xcsum_ctx *c)
{
	for (int s = 0; s < Ctx::NSLOT; s++)
		if (c->streams[s])
			(void)hipStreamSynchronize(c->streams[s]);
}

extern "C" int xcsum_ctx_pending(xcsum_ctx *c)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -XCSUM_ERR_HIP;
	int busy = 0;
	for (int s = 0; s < Ctx::NSLOT; s++)
		if (c->streams[s] && hipStreamQuery(c->streams[s]) == hipErrorNotReady)
			busy++;
	return busy;
}

/* A host batch through the resident workgroups (xcsum_ctx_set_resident):
 * the frames are read where the kernel can reach them without a copy
 *   - in a registered UMEM: in place through its device alias (in-place
 *     writes land in the frames directly);
 *   - else staged into the pinned stage of slot 0 (gathered frame by frame,
 *     or the 16-byte aligned range), up to XCSUM_DIRECT_MAX bytes;
 * descriptors go to the pinned descriptor stage, results come back in the
 * pinned result slot.  Returns RES_DECLINE when the batch does not fit (the
 * launched path takes it). */
static constexpr int RES_DECLINE = 1;

static int batch_host_resident(xcsum_ctx *c, uint8_t *h_umem, const struct xcsum_desc *h_desc,
			       uint32_t n, uint16_t *h_out, uint16_t *h_out_ip, uint32_t mode,
			       uint32_t flags, const Region *zc, bool gather)
{
	if (n > c->res_max_frames || n > RB_DESC_CAP || !c->v_stage[0])
		return RES_DECLINE;
	const auto t_call = c->res_trace ? std::chrono::steady_clock::now()
					 : std::chrono::steady_clock::time_point();
	/* The resident kernel reads only the library's own pinned stage, never
	 * the caller's registered UMEM in place: reading it in place faulted 4 of
	 * 12 GPU suite runs, always in a test whose resident workgroups read a
	 * registered UMEM; reading the stage never did.  A
	 * sparse registered UMEM's frames are gathered like a pageable one's. */
	if (zc)
		gather = true;
	uint64_t lo = UINT64_MAX, hi = 0, staged = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (h_desc[i].addr < lo) lo = h_desc[i].addr;
		if (h_desc[i].addr + h_desc[i].len > hi) hi = h_desc[i].addr + h_desc[i].len;
		staged = stage_off(staged, h_desc[i].addr) + h_desc[i].len;
	}
	const uint64_t alo = lo & ~(uint64_t)15;
	if ((gather ? staged : hi - alo) > DIRECT_MAX)
		return RES_DECLINE;
	int rc = resident_ensure(c);
	if (rc)
		return rc;
	/* the descriptors go into the doorbell */
	struct xcsum_desc *ds = c->res_bell->desc;
	CsumArgs a;
	a.umem = c->v_stage[0];
	a.desc = c->res_vbell->desc;
	a.n = n;
	a.out = c->v_out[0];
	a.out_ip = (flags & XCSUM_F_IPHDR) ? c->v_out[0] + n : nullptr;
	a.mode = mode;
	/* in-place fields are written on the host (retire) */
	a.flags = flags & (XCSUM_F_IPHDR | XCSUM_F_V4_RFC | XCSUM_F_VERIFY);
	a.err = c->d_err;
	a.bias = 0;
	a.ord = order_identity(n);
	a.dense = a.ord;
	if (gather) {
		/* each frame copied on its own, at its 16-byte phase (stage_off) */
		uint64_t pos = 0;
		for (uint32_t k = 0; k < n; k++) {
			const struct xcsum_desc &d = h_desc[k];
			const uint64_t off = stage_off(pos, d.addr);
			memcpy(c->h_stage[0] + off, h_umem + d.addr, d.len);
			ds[k] = xcsum_desc{off, d.len, 0};
			pos = off + d.len;
		}
	} else {
		/* 16-byte aligned copy of [lo, hi): every frame keeps its address
		 * parity and phase */
		memcpy(c->h_stage[0], h_umem + alo, hi - alo);
		memcpy(ds, h_desc, (size_t)n * sizeof(*ds));
		a.bias = alo;
	}
	{
		const uint64_t lim = gather ? staged : hi - alo;
		rc = resident_call(c, a, lim - (c->res_limit_cut < lim ? c->res_limit_cut : lim));
	}
	if (rc)
		return rc;
	Pending pd;
	pd.first = 0;
	pd.count = n;
	retire(c->stage_pool, pd, c->h_out[0], h_umem, h_desc, h_out, h_out_ip, mode, flags);
	if (c->res_trace) {
		c->res_calls++;
		c->res_call_us += std::chrono::duration<double, std::micro>(
					  std::chrono::steady_clock::now() - t_call).count();
	}
	return 0;
}

static int batch_host_run(xcsum_ctx *c, uint8_t *h_umem, const struct xcsum_desc *h_desc,
			  uint32_t n, uint16_t *h_out, uint16_t *h_out_ip, uint32_t mode,
			  uint32_t flags, bool gather)
{
	if (!c || mode > XCSUM_MODE_AUTO)
		return -XCSUM_ERR_INVAL;
	if (n == 0)
		return 0;
	if (!h_desc || (!h_out && !h_out_ip && !(flags & XCSUM_F_INPLACE)))
		return -XCSUM_ERR_INVAL;
	/* libxudp's IPv4 call (XCSUM_F_IPHDR_ONLY): the header kernel, on the
	 * frames' first 42 bytes -- gathered from unregistered memory, read in
	 * place over PCIe from a mapped UMEM */
	const bool hdr_only = (flags & XCSUM_F_IPHDR_ONLY) != 0;
	if (hdr_only && mode == XCSUM_MODE_V6)
		return -XCSUM_ERR_INVAL;
	/* the header kernel's one result per frame goes to h_out (it is
	 * iph->check): a second array would only get stale slot contents
	 *  */
	if (hdr_only && h_out_ip)
		return -XCSUM_ERR_INVAL;
	if (hdr_only)
		flags &= XCSUM_F_IPHDR_ONLY | XCSUM_F_INPLACE | XCSUM_F_VERIFY | XCSUM_F_ZEROCOPY;
	if (flags & XCSUM_F_VERIFY)
		flags &= ~XCSUM_F_INPLACE; /* verifying never writes frames */
	HIPCHK(hipSetDevice(c->device));
	int rc = ensure_staging(c);
	if (rc)
		return rc;
	const bool want_ip = (flags & XCSUM_F_IPHDR) != 0;

	/* zero-copy: the kernel reads frames where they are (registered UMEM) */
	const Region *zc = nullptr;
	if (flags & XCSUM_F_ZEROCOPY) {
		uint64_t lo = UINT64_MAX, hi = 0;
		for (uint32_t i = 0; i < n; i++) {
			if (h_desc[i].addr < lo) lo = h_desc[i].addr;
			if (h_desc[i].addr + h_desc[i].len > hi) hi = h_desc[i].addr + h_desc[i].len;
		}
		zc = find_region(c, h_umem + lo, h_umem + hi);
		/* a registered region the GPU does not map is staged instead */
		if (!zc && !in_any_region(c, h_umem + lo, h_umem + hi))
			return -XCSUM_ERR_NOT_REGISTERED;
	} else if (hdr_only) {
		/* one header line per frame: read in place from a mapped UMEM
		 * whatever the density (1M packed frames: 5.7 ms in place vs
		 * 18.6 ms gathered, profiles/r05/iphdr/r05q_e2e_iphdr_packed.log) */
		uint64_t lo = UINT64_MAX, hi = 0;
		for (uint32_t i = 0; i < n; i++) {
			if (h_desc[i].addr < lo) lo = h_desc[i].addr;
			if (h_desc[i].addr + h_desc[i].len > hi) hi = h_desc[i].addr + h_desc[i].len;
		}
		zc = find_region(c, h_umem + lo, h_umem + hi);
	} else {
		zc = zerocopy_pays(c, h_umem, h_desc, n);
	}

	if (zc)
		gather = false;
	else if (hdr_only)
		gather = true;
	/* the pinned stages: every byte that crosses PCIe from unregistered
	 * caller memory goes through them (see host_dma_src) */
	if ((rc = ensure_gather(c)))
		return rc;

	/* small batches: the resident workgroups, if the context has them (they
	 * run the checksum kernel: header-only batches are launched) */
	if (c->res_wg > 0) {
		rc = hdr_only ? RES_DECLINE
			      : batch_host_resident(c, h_umem, h_desc, n, h_out, h_out_ip, mode,
						    flags, zc, gather);
		if (rc != RES_DECLINE)
			return rc;
		/* the launched path's slot streams may share a hardware queue
		 * with the live grid, and would wait behind it: stop it first */
		if (c->res_live && (rc = resident_stop(c)))
			return rc;
	}

	/* zero-copy + INPLACE: the kernel already wrote the host frames */
	const uint32_t rflags = zc ? (flags & ~XCSUM_F_INPLACE) : flags;
	/* bytes gathered per frame: the header kernel reads inside [eth+9,
	 * eth+40), the descriptor keeps the frame's length for its rules */
	auto glen = [hdr_only](const struct xcsum_desc &d) -> uint64_t {
		return hdr_only && d.len > 42u ? 42u : d.len;
	};
	Pending pend[Ctx::NSLOT];
	for (int s = 0; s < Ctx::NSLOT; s++)
		pend[s].busy = false;

	uint32_t i = 0;
	int slot = 0;
	while (i < n) {
		/* grow a chunk: <= desc_cap frames, UMEM range (or gathered bytes)
		 * <= frame_cap */
		uint64_t lo = h_desc[i].addr, hi = h_desc[i].addr + h_desc[i].len;
		uint64_t gpos = stage_off(0, lo) + glen(h_desc[i]);   /* gathered bytes so far */
		/* the first frame must fit a stage: gathered, only its glen() bytes
		 * are staged (42 of a header-only frame), else its range */
		if (!zc && (gather ? gpos > c->frame_cap : hi - lo > c->frame_cap - 16))
			return -XCSUM_ERR_INVAL;
		uint32_t cnt = 1;
		while (gather && i + cnt < n && cnt < c->desc_cap) {
			const struct xcsum_desc &d = h_desc[i + cnt];
			const uint64_t e = stage_off(gpos, d.addr) + glen(d);
			if (e > c->frame_cap)
				break;
			gpos = e;
			cnt++;
		}
		while (!gather && i + cnt < n && cnt < c->desc_cap) {
			const struct xcsum_desc &d = h_desc[i + cnt];
			uint64_t nlo = d.addr < lo ? d.addr : lo;
			uint64_t nhi = d.addr + d.len > hi ? d.addr + d.len : hi;
			if (!zc && nhi - nlo > c->frame_cap)
				break;
			lo = nlo;
			hi = nhi;
			cnt++;
		}
		if (pend[slot].busy) {
			HIPCHK(wait_slot(c->done[slot]));
			retire(c->stage_pool, pend[slot], c->h_out[slot], h_umem, h_desc, h_out, h_out_ip, mode, rflags);
			pend[slot].busy = false;
		}
		hipStream_t st = c->streams[slot];
		bool direct = false;
		CsumArgs a;
		a.desc = c->d_desc[slot];
		a.n = cnt;
		a.ord = order_identity(cnt);
		a.dense = a.ord;
		a.out = c->d_out[slot];
		a.out_ip = want_ip ? c->d_out[slot] + cnt : nullptr;
		a.mode = mode;
		a.err = c->d_err;
		if (zc) {
			a.umem = zc->dev + (h_umem - zc->host);
			a.bias = 0;
			a.flags = flags & (XCSUM_F_INPLACE | XCSUM_F_IPHDR | XCSUM_F_V4_RFC |
					   XCSUM_F_VERIFY);
#ifdef XCSUM_DEBUG_BOUNDS
			a.reg_lo = (uint64_t)(uintptr_t)zc->dev;
			a.reg_hi = a.reg_lo + zc->size;
#endif
		} else if (gather) {
			/* each frame copied on its own into the pinned stage, then
			 * one DMA of the packed bytes and one of their descriptors */
			const uint64_t pos = gather_frames(c->stage_pool, c->h_stage[slot], h_umem, h_desc + i,
							   c->h_dstage[slot], cnt,
							   hdr_only ? 42u : UINT32_MAX);
			a.bias = 0;
			a.flags = flags & (XCSUM_F_IPHDR | XCSUM_F_V4_RFC | XCSUM_F_VERIFY);
			if (DIRECT_ON && pos <= DIRECT_MAX) {
				/* small batch: no copies -- the kernel reads the pinned
				 * stage over PCIe and writes the pinned result slot; the
				 * call's latency is one launch, not three transfers and
				 * a launch */
				direct = true;
				a.umem = c->v_stage[slot];
				a.desc = c->v_dstage[slot];
				a.out = c->v_out[slot];
				a.out_ip = want_ip ? c->v_out[slot] + cnt : nullptr;
			} else {
				HIPCHK(hipMemcpyAsync(c->d_frames[slot], c->h_stage[slot], pos,
						      hipMemcpyHostToDevice, st));
				a.umem = c->d_frames[slot];
			}
		} else {
			/* 16-byte aligned copy of [lo, hi) keeps every frame's address
			 * parity and 16-byte phase identical to the host UMEM */
			uint64_t alo = lo & ~(uint64_t)15;
			HIPCHK(hipMemcpyAsync(c->d_frames[slot],
					      host_dma_src(c, slot, h_umem + alo, hi - alo), hi - alo,
					      hipMemcpyHostToDevice, st));
			a.umem = c->d_frames[slot];
			a.bias = alo;
			/* the device copy is scratch: in-place writes happen on the host */
			a.flags = flags & (XCSUM_F_IPHDR | XCSUM_F_V4_RFC | XCSUM_F_VERIFY);
		}
		if (!direct)
			HIPCHK(hipMemcpyAsync(c->d_desc[slot], gather ? c->h_dstage[slot]
							       : host_desc_src(c, slot, h_desc + i, cnt),
					      cnt * sizeof(struct xcsum_desc), hipMemcpyHostToDevice, st));
		uint32_t avg = (uint32_t)((gather ? gpos : hi - lo) / cnt);
		if (hdr_only)
			HIPCHK(launch_iphdr(a, c->tune.iphdr_fpt, st));
		else
			HIPCHK(launch_csum(a, geometry_for(c, avg, a.flags), c->cus, st));
		if (!direct)
			HIPCHK(hipMemcpyAsync(c->h_out[slot], c->d_out[slot],
					      (want_ip ? 2 : 1) * cnt * sizeof(uint16_t),
					      hipMemcpyDeviceToHost, st));
		HIPCHK(hipEventRecord(c->done[slot], st));
		pend[slot].first = i;
		pend[slot].count = cnt;
		pend[slot].busy = true;
		i += cnt;
		slot = (slot + 1) % Ctx::NSLOT;
	}
	for (int k = 0; k < Ctx::NSLOT; k++) {
		int s = (slot + k) % Ctx::NSLOT;
		if (pend[s].busy) {
			HIPCHK(wait_slot(c->done[s]));
			retire(c->stage_pool, pend[s], c->h_out[s], h_umem, h_desc, h_out, h_out_ip, mode, rflags);
			pend[s].busy = false;
		}
	}
	return 0;
}

namespace xcsum {

int batch_host_impl(xcsum_ctx *c, uint8_t *h_umem, const struct xcsum_desc *h_desc, uint32_t n,
		    uint16_t *h_out, uint16_t *h_out_ip, uint32_t mode, uint32_t flags, bool gather)
{
	const int rc = batch_host_run(c, h_umem, h_desc, n, h_out, h_out_ip, mode, flags, gather);
	if (rc && c)
		drain_slots(c);
	return rc;
}

} /* namespace xcsum */

extern "C" int xcsum_batch_host(xcsum_ctx *c, uint8_t *h_umem, const struct xcsum_desc *h_desc,
				uint32_t n, uint16_t *h_out, uint32_t mode, uint32_t flags)
{
	/* small frames spread over a pageable UMEM: gathered (gather_pays) */
	bool gather = false;
	if (c && h_umem && h_desc && n && !(flags & XCSUM_F_ZEROCOPY)) {
		uint64_t lo = UINT64_MAX, hi = 0, sum = 0;
		for (uint32_t i = 0; i < n; i++) {
			if (h_desc[i].addr < lo) lo = h_desc[i].addr;
			if (h_desc[i].addr + h_desc[i].len > hi) hi = h_desc[i].addr + h_desc[i].len;
			sum += h_desc[i].len;
		}
		gather = gather_pays(c, h_umem, lo, hi, sum);
	}
	return batch_host_impl(c, h_umem, h_desc, n, h_out, nullptr, mode, flags, gather);
}

/* Receive batch on host-resident frames: the chunking of batch_host_impl
 * (<= desc_cap frames, <= frame_cap bytes per chunk, two slots in flight),
 * the receive kernel per chunk, records back through pinned staging.  Record
 * addresses are UMEM offsets, as from xcsum_rx_device.
 * Three ways to the frames:
 *   - zero-copy (XCSUM_F_ZEROCOPY, registered UMEM): read in place;
 *   - a dense batch: one copy of the UMEM range per chunk, the kernel's base
 *     biased by the chunk's offset so addresses stay UMEM offsets;
 *   - a sparse batch in a pageable UMEM (the frames cover less than half
 *     the range they span, as an RX ring's frames do, one per 2-4 KB UMEM
 *     chunk): gathered frame by frame into the pinned stage, so only frame
 *     bytes are copied (a pageable range copy memcpy's the gaps too); up to
 *     XCSUM_DIRECT_MAX staged bytes the kernel reads the stage and writes the
 *     pinned records in place (no copies).  The kernel then sees staged
 *     offsets: `frame` and `body` are moved back to UMEM offsets on the host
 *     as the records are collected. */
static int rx_host_run(xcsum_ctx *c, const uint8_t *h_umem, const struct xcsum_desc *h_desc,
		       uint32_t n, struct xcsum_rx_msg *h_msgs, uint32_t *h_count, uint32_t flags);

extern "C" int xcsum_rx_host(xcsum_ctx *c, const uint8_t *h_umem, const struct xcsum_desc *h_desc,
			     uint32_t n, struct xcsum_rx_msg *h_msgs, uint32_t *h_count,
			     uint32_t flags)
{
	const int rc = rx_host_run(c, h_umem, h_desc, n, h_msgs, h_count, flags);
	if (rc && c)
		drain_slots(c);   /* see batch_host_impl */
	return rc;
}

static int rx_host_run(xcsum_ctx *c, const uint8_t *h_umem, const struct xcsum_desc *h_desc,
		       uint32_t n, struct xcsum_rx_msg *h_msgs, uint32_t *h_count, uint32_t flags)
{
	if (!c)
		return -XCSUM_ERR_INVAL;
	if (h_count)
		*h_count = 0;
	if (n == 0)
		return 0;
	if (!h_umem || !h_desc || !h_msgs || ((uintptr_t)h_umem & 3u))
		return -XCSUM_ERR_INVAL;
	HIPCHK(hipSetDevice(c->device));
	int rc = ensure_staging(c);
	if (rc)
		return rc;
	for (int s = 0; s < Ctx::NSLOT; s++) {
		if (!c->d_rx_msgs[s] &&
		    hipMalloc(&c->d_rx_msgs[s], c->desc_cap * sizeof(struct xcsum_rx_msg)) != hipSuccess)
			return -XCSUM_ERR_NOMEM;
		if (!c->h_rx_msgs[s] &&
		    hipHostMalloc(&c->h_rx_msgs[s], c->desc_cap * sizeof(struct xcsum_rx_msg),
				  PINNED_FLAGS) != hipSuccess)
			return -XCSUM_ERR_NOMEM;
		if (DIRECT_ON && !c->v_rx_msgs[s] &&
		    hipHostGetDevicePointer((void **)&c->v_rx_msgs[s], c->h_rx_msgs[s], 0) != hipSuccess) {
			c->v_rx_msgs[s] = nullptr;
			return -XCSUM_ERR_HIP;
		}
	}
	uint64_t blo = UINT64_MAX, bhi = 0, bsum = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (h_desc[i].addr < blo) blo = h_desc[i].addr;
		if (h_desc[i].addr + h_desc[i].len > bhi) bhi = h_desc[i].addr + h_desc[i].len;
		bsum += h_desc[i].len;
	}
	const Region *zc = nullptr;
	if (flags & XCSUM_F_ZEROCOPY) {
		zc = find_region(c, h_umem + blo, h_umem + bhi);
		if (!zc && !in_any_region(c, h_umem + blo, h_umem + bhi))
			return -XCSUM_ERR_NOT_REGISTERED;
		if (zc && ((uintptr_t)zc->dev & 3u) != ((uintptr_t)zc->host & 3u))
			return -XCSUM_ERR_NOT_REGISTERED;
	} else {
		zc = zerocopy_pays(c, h_umem, h_desc, n);
		if (zc && ((uintptr_t)zc->dev & 3u) != ((uintptr_t)zc->host & 3u))
			zc = nullptr;
	}
	const bool gather = !zc && gather_pays(c, h_umem, blo, bhi, bsum);
	if ((rc = ensure_gather(c)))   /* the pinned stages (host_dma_src) */
		return rc;
	Pending pend[Ctx::NSLOT];
	for (int s = 0; s < Ctx::NSLOT; s++)
		pend[s].busy = false;
	uint32_t delivered = 0;
	auto finish = [&](int s) -> int {
		HIPCHK(wait_slot(c->done[s]));
		struct xcsum_rx_msg *m = h_msgs + pend[s].first;
		memcpy(m, c->h_rx_msgs[s], (size_t)pend[s].count * sizeof(struct xcsum_rx_msg));
		for (uint32_t k = 0; k < pend[s].count; k++) {
			delivered += m[k].status == XCSUM_RX_OK;
			if (pend[s].gathered) {
				/* staged offset -> UMEM offset */
				const uint64_t st = c->h_dstage[s][k].addr;
				const uint64_t ua = h_desc[pend[s].first + k].addr;
				m[k].frame = ua;
				if (m[k].body)
					m[k].body = m[k].body - st + ua;
			}
		}
		pend[s].busy = false;
		return 0;
	};
	uint32_t i = 0;
	int slot = 0;
	while (i < n) {
		uint64_t lo = h_desc[i].addr, hi = h_desc[i].addr + h_desc[i].len;
		uint32_t cnt = 1;
		uint64_t gpos = stage_off(0, lo) + h_desc[i].len;   /* gathered bytes so far */
		if (gather ? gpos > c->frame_cap : (!zc && hi - lo > c->frame_cap))
			return -XCSUM_ERR_INVAL;
		while (gather && i + cnt < n && cnt < c->desc_cap) {
			const struct xcsum_desc &d = h_desc[i + cnt];
			const uint64_t e = stage_off(gpos, d.addr) + d.len;
			if (e > c->frame_cap)
				break;
			gpos = e;
			cnt++;
		}
		while (!gather && i + cnt < n && cnt < c->desc_cap) {
			const struct xcsum_desc &d = h_desc[i + cnt];
			uint64_t nlo = d.addr < lo ? d.addr : lo;
			uint64_t nhi = d.addr + d.len > hi ? d.addr + d.len : hi;
			if (!zc && nhi - nlo > c->frame_cap)
				break;
			lo = nlo;
			hi = nhi;
			cnt++;
		}
		if (pend[slot].busy && (rc = finish(slot)))
			return rc;
		hipStream_t st = c->streams[slot];
		bool direct = false;
		RxArgs a;
		a.desc = c->d_desc[slot];
		a.msgs = c->d_rx_msgs[slot];
		if (zc) {
			a.umem = zc->dev + (h_umem - zc->host);
		} else if (gather) {
			const uint64_t pos = gather_frames(c->stage_pool, c->h_stage[slot], h_umem, h_desc + i,
							   c->h_dstage[slot], cnt, UINT32_MAX);
			if (DIRECT_ON && pos <= DIRECT_MAX) {
				direct = true;
				a.umem = c->v_stage[slot];
				a.desc = c->v_dstage[slot];
				a.msgs = c->v_rx_msgs[slot];
			} else {
				HIPCHK(hipMemcpyAsync(c->d_frames[slot], c->h_stage[slot], pos,
						      hipMemcpyHostToDevice, st));
				a.umem = c->d_frames[slot];
			}
		} else {
			/* 16-byte aligned copy of [lo, hi): every frame keeps its
			 * address phase; the kernel sees umem + addr inside it */
			const uint64_t alo = lo & ~(uint64_t)15;
			HIPCHK(hipMemcpyAsync(c->d_frames[slot],
					      host_dma_src(c, slot, h_umem + alo, hi - alo), hi - alo,
					      hipMemcpyHostToDevice, st));
			a.umem = (const uint8_t *)((uintptr_t)c->d_frames[slot] - (uintptr_t)alo);
		}
		if (!direct)
			HIPCHK(hipMemcpyAsync(c->d_desc[slot], gather ? c->h_dstage[slot]
							       : host_desc_src(c, slot, h_desc + i, cnt),
					      cnt * sizeof(struct xcsum_desc), hipMemcpyHostToDevice, st));
		a.n = cnt;
		a.flags = flags & (XCSUM_F_VERIFY | XCSUM_F_IPHDR);
		a.count = nullptr;
		a.part = c->d_rx_part;
		HIPCHK(launch_rx(a, (uint32_t)((gather ? gpos : hi - lo) / cnt), c->cus, c->tune, st));
		if (!direct)
			HIPCHK(hipMemcpyAsync(c->h_rx_msgs[slot], c->d_rx_msgs[slot],
					      (size_t)cnt * sizeof(struct xcsum_rx_msg),
					      hipMemcpyDeviceToHost, st));
		HIPCHK(hipEventRecord(c->done[slot], st));
		pend[slot].first = i;
		pend[slot].count = cnt;
		pend[slot].busy = true;
		pend[slot].gathered = gather;
		i += cnt;
		slot = (slot + 1) % Ctx::NSLOT;
	}
	for (int k = 0; k < Ctx::NSLOT; k++) {
		const int s = (slot + k) % Ctx::NSLOT;
		if (pend[s].busy && (rc = finish(s)))
			return rc;
	}
	if (h_count)
		*h_count = delivered;
	return 0;
}

/* ---- synthetic frames ---------------------------------------------------- */

extern "C" int xcsum_gen_layout(uint32_t n, uint32_t family, uint32_t pmin, uint32_t pmax,
				uint64_t seed, uint64_t first_index, uint32_t align,
				uint32_t stride, uint32_t offset, struct xcsum_desc *h_desc,
				uint64_t *umem_bytes)
{
	if ((family != 4 && family != 6) || pmin > pmax || (n && !h_desc) || !umem_bytes)
		return -XCSUM_ERR_INVAL;
	const uint32_t hdr = family == 6 ? XG_HDR6 : XG_HDR4;
	if ((uint64_t)pmax + hdr > 0xffffffffull)
		return -XCSUM_ERR_INVAL;
	if (align == 0)
		align = 8;
	uint64_t off = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint32_t len = hdr + xg_payload_size(seed, first_index + i, pmin, pmax);
		if (stride) {
			if ((uint64_t)offset + len > stride)
				return -XCSUM_ERR_INVAL;
			h_desc[i].addr = (uint64_t)i * stride + offset;
		} else {
			h_desc[i].addr = off;
			off = (off + len + align - 1) / align * align;
		}
		h_desc[i].len = len;
		h_desc[i].options = 0;
	}
	*umem_bytes = stride ? (uint64_t)n * stride : off;
	return 0;
}

extern "C" int xcsum_gen_fill_host(uint8_t *h_umem, const struct xcsum_desc *h_desc, uint32_t n,
				   uint32_t family, uint64_t seed, uint64_t first_index)
{
	if ((family != 4 && family != 6) || (n && (!h_umem || !h_desc)))
		return -XCSUM_ERR_INVAL;
	const uint32_t hdr = family == 6 ? XG_HDR6 : XG_HDR4;
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *eth = h_umem + h_desc[i].addr;
		uint32_t len = h_desc[i].len;
		uint64_t key = xg_key(seed, first_index + i);
		if (len < hdr)
			return -XCSUM_ERR_INVAL;
		for (uint32_t o = 0; o < hdr; o++)
			eth[o] = xg_header_byte(family, key, len, o);
		uint8_t *pl = eth + hdr;
		uint32_t plen = len - hdr;
		for (uint32_t q = 0; q < plen; q += 8) {
			uint64_t w = xg_payload_word(key, q >> 3);
			uint32_t k = plen - q < 8 ? plen - q : 8;
			memcpy(pl + q, &w, k); /* little-endian host: byte i = bits 8i.. */
		}
	}
	return 0;
}

extern "C" int xcsum_gen_fill_device(uint8_t *d_umem, const struct xcsum_desc *d_desc, uint32_t n,
				     uint32_t family, uint64_t seed, uint64_t first_index,
				     void *stream)
{
	if ((family != 4 && family != 6) || (n && (!d_umem || !d_desc)))
		return -XCSUM_ERR_INVAL;
	int dev = 0, cus = 256;
	HIPCHK(hipGetDevice(&dev));
	(void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
	HIPCHK(launch_gen(d_umem, d_desc, n, family, seed, first_index, cus * 8,
			  (hipStream_t)stream));
	return 0;
}

extern "C" int xcsum_shard_by_bytes(const struct xcsum_desc *h_desc, uint32_t n, uint32_t nshards,
				    uint32_t idx, uint32_t *first, uint32_t *count)
{
	if (!first || !count || nshards == 0 || idx >= nshards || (n && !h_desc))
		return -XCSUM_ERR_INVAL;
	uint64_t total = 0;
	for (uint32_t i = 0; i < n; i++)
		total += h_desc[i].len;
	/* shard k = frames whose starting cumulative byte lies in
	 * [k*total/nshards, (k+1)*total/nshards) */
	uint64_t lo_b = total * idx / nshards, hi_b = total * (idx + 1) / nshards;
	uint64_t cum = 0;
	uint32_t f = n, e = n;
	for (uint32_t i = 0; i < n; i++) {
		if (f == n && cum >= lo_b)
			f = i;
		if (cum >= hi_b) {
			e = i;
			break;
		}
		cum += h_desc[i].len;
	}
	if (f > e)
		f = e;
	if (idx + 1 == nshards)
		e = n;
	*first = f;
	*count = e - f;
	return 0;
}
