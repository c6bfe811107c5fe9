/* xcsum_internal.h -- shared between the kernel TU and the host API TU. */
#ifndef XCSUM_INTERNAL_H
#define XCSUM_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include "xcsum.h"
#include "xcsum_resident.h"

namespace xcsum {

/* Visiting order of a batch.  A kernel walks logical indices [0, nlog);
 * logical tile t (2^tshift frames) is frame tile (t % R) * q + t / R with
 * R = 2^rshift, so the frames in flight at any moment come from R regions
 * spread over the batch instead of one contiguous window (DESIGN.md,
 * "Visiting order").  rshift == 0: identity, nlog == n.  sparse_only: the
 * checksum kernel keeps the region order only if it finds the batch sparse
 * in the UMEM (resolve_order), else falls back to the identity. */
struct Order {
	uint32_t nlog, rshift, tshift, q;
	uint32_t sparse_only;
};

static __host__ __device__ inline Order order_identity(uint32_t n)
{
	return Order{n, 0u, 0u, 0u, 0u};
}

/* R = 2^rlog regions of 2^tlog-frame tiles; the identity when the batch is
 * too small to give every region a tile or too large for u32 indices */
static __host__ __device__ inline Order order_regions(uint32_t n, int rlog, int tlog)
{
	if (rlog <= 0 || tlog < 0 || rlog + tlog > 30 || n > (1u << 31) || n < (1u << (rlog + tlog)))
		return order_identity(n);
	const uint32_t ntiles = (n + (1u << tlog) - 1) >> tlog;
	const uint32_t q = (ntiles + (1u << rlog) - 1) >> rlog;
	return Order{(q << rlog) << tlog, (uint32_t)rlog, (uint32_t)tlog, q, 0u};
}

/* logical index -> frame index (>= n: no frame) */
static __device__ __forceinline__ uint32_t frame_of(const Order &o, uint32_t p)
{
	if (o.rshift == 0)
		return p;
	const uint32_t t = p >> o.tshift;
	const uint32_t r = t & ((1u << o.rshift) - 1u);
	return ((r * o.q + (t >> o.rshift)) << o.tshift) | (p & ((1u << o.tshift) - 1u));
}

/* ---- XCSUM_DEBUG_BOUNDS (make -C libxudp_amd debug): device-side bounds
 * checks.  Every frame load and store of every kernel is tested against the
 * bytes it may touch (its frame's extent from the descriptor, the stream
 * region of its 64-frame group, the result arrays' n entries); a violation is
 * recorded in a per-translation-unit device log (first BOUNDS_RECS kept) and
 * the access is skipped or redirected to zeros, so the run goes on without
 * faulting.  xcsum_debug_bounds() collects and clears the logs.  Not in
 * libxcsum.so: the macros compile to nothing there. */
enum BoundsSite : uint32_t {
	XB_CSUM_CHUNK = 1,      /* frame-group kernel: chunk load */
	XB_CSUM_WALK,           /* jumbo / re-cut walk load */
	XB_CSUM_HDR,            /* h_proto, udp len/check, IPv4 header loads */
	XB_CSUM_OUT,            /* out[p] / out_ip[p]: p < n */
	XB_CSUM_INPLACE,        /* in-place udp->check / iph->check store */
	XB_STREAM_REGION,       /* stream kernel: region load vs its frames' extent */
	XB_STREAM_STAGE,        /* stream kernel: LDS stage index */
	XB_BUILD_SRC,           /* build: payload block load */
	XB_BUILD_DATA,          /* build: payload / header store vs the frame slot */
	XB_BUILD_OUT,           /* build: desc_out[p] / out[p]: p < n */
	XB_RX_CHUNK,            /* receive: frame chunk load */
	XB_RX_REC,              /* receive: record store, p < n */
	XB_RX_PART,             /* receive: per-block count slot */
	XB_RX_STREAM,           /* receive stream kernel: region load */
	XB_GEN_STORE,           /* synthetic fill: store vs the frame */
	XB_SCATTER,             /* two-pass in-place: h_proto load / field store */
	XB_CSUM_REGION,         /* zero-copy: frame vs the registered region's extent */
	XB_RES_REQ,             /* resident request: umem / desc / out pointers vs
				   the context's stage, doorbell and result slot */
	XB_SITE_COUNT
};

#ifdef XCSUM_DEBUG_BOUNDS
struct BoundsRec {
	uint32_t site, index;
	uint64_t addr, lo, hi;  /* the access [addr, ...) and the allowed [lo, hi) */
};
constexpr int BOUNDS_RECS = 16;
struct BoundsLog {
	unsigned long long count;
	unsigned long long pad;
	BoundsRec rec[BOUNDS_RECS];
};
/* one reader per translation unit with kernels (xcsum_device.h) */
struct BoundsReader {
	int (*take)(BoundsLog *out);
	BoundsReader *next;
};
BoundsReader *&bounds_readers();
#endif

/* Kernel arguments (passed by value). */
struct CsumArgs {
	uint8_t *umem;                 /* frame i starts at umem + desc[i].addr - bias */
	const struct xcsum_desc *desc;
	uint32_t n;
	uint16_t *out;                 /* may be null (INPLACE only) */
	uint16_t *out_ip;              /* IPHDR: iph->check per frame (may be null) */
	uint32_t mode;
	uint32_t flags;
	uint64_t bias;
	unsigned long long *err;       /* device counter of malformed frames */
	Order ord;
	Order dense;                   /* ord.sparse_only: the order a dense batch
					  gets instead (resolve_order) */
	/* the launched kernels trust their descriptors (the host bounded the
	 * batch); an argument type with kChecked (xcsum_resident.hip) checks
	 * each one before any load of its frame (desc_ok / desc_bad) */
	static constexpr bool kChecked = false;
#ifdef XCSUM_DEBUG_BOUNDS
	/* zero-copy launches: the registered region's device extent, every
	 * frame checked against it before any load (0, 0: unchecked) */
	uint64_t reg_lo = 0, reg_hi = 0;
#endif
};

/* Second pass of the two-pass in-place schedule (xcsum_scatter.hip): store
 * res[p] (and res_ip[p]) into the check fields of every well-formed frame. */
struct ScatterArgs {
	uint8_t *umem;
	const struct xcsum_desc *desc;
	uint32_t n;
	uint32_t mode;
	const uint16_t *res;
	const uint16_t *res_ip;        /* IPHDR: iph->check values, else null */
	uint64_t bias;
	uint32_t block;                /* 0: 2-byte stores; 32 / 64: the whole
					  sector / line holding a field, read and
					  patched, when it lies inside the frame */
};

hipError_t launch_scatter(const ScatterArgs &a, int cus, hipStream_t s);

/* Frame-build kernel arguments (xcsum_build.hip). */
struct BuildArgs {
	uint8_t *umem;
	const uint8_t *src;
	const struct xcsum_msg *msgs;
	uint32_t n, frame_size, data_off, flags;
	struct xcsum_desc *desc_out;
	uint16_t *out;
	unsigned long long *err;
	uint32_t family;
	uint32_t tmpl[16];             /* 64-byte header template, memory order */
	Order ord;                     /* over messages */
};

/* Per-context tuning (xcsum_ctx_set_tuning, include/xcsum.h): which kernel
 * variant or geometry a launch takes, never its results.  Set at context
 * creation to the defaults (and, in the variant and debug builds only, from
 * the A/B environment variables: read_env_tuning), read by the launches from
 * the context -- no launch or batch reads the environment. */
struct Tuning {
	int iphdr_fpt;                 /* IPv4 header kernel: frames per thread, 1|2|4|8 */
	bool build_hdr;                /* IPv4 in-place build: header kernel (true) or
					  the payload-summing build kernel (A/B) */
	int build_G, build_K;          /* build kernel geometry, G == 0: automatic */
	int rx_G, rx_K, rx_U, rx_B;    /* receive kernel geometry, G == 0: automatic */
	int rx_rlog, rx_tlog;          /* receive visiting order: rlog -1 automatic,
					  0 descriptor order, else 2^R regions of 2^T tiles */
	uint32_t gather_ratio;         /* host path: gather when the span > ratio x bytes */
	uint32_t claim_static_64;      /* claimed tail: static share in 64ths (0: off) */
	uint32_t claim_steps;          /* claimed tail: wave steps per claim */
};

hipError_t launch_build(const BuildArgs &a, uint32_t len_hint, int cus, const Tuning &t,
			hipStream_t s);

/* Receive-path kernel arguments (xcsum_rx.hip). */
struct RxArgs {
	const uint8_t *umem;
	const struct xcsum_desc *desc;
	uint32_t n, flags;
	struct xcsum_rx_msg *msgs;
	uint32_t *count;               /* may be null */
	uint32_t *part;                /* per-block counts (ctx scratch, RX_PART_MAX) */
	Order ord;                     /* visiting order (set by launch_rx) */
	Order dense;                   /* ord.sparse_only: a dense batch's order */
};

constexpr uint32_t CLAIM_SLOTS = 256;

/* per-block delivered counts of one receive launch: >= CUs x blocks per CU */
constexpr uint32_t RX_PART_MAX = 4096;

hipError_t launch_rx(const RxArgs &a, uint32_t len_hint, int cus, const Tuning &t, hipStream_t s);
/* the build and receive kernel geometries compiled in (xcsum_ctx_set_tuning) */
bool build_geometry_supported(int G, int K);
bool rx_geometry_supported(int G, int K, int U);

/* Kernel geometry: G lanes cooperate on one frame, each segment keeps U frames
 * in flight, and each lane preloads K 16-byte chunks per frame. */
struct Geometry {
	int G, U, K;
	int B; /* 256-thread blocks per CU (0: occupancy limit) */
};

/* A/B kernels that lost their measurements live outside the product library
 * (csrc/variants/: the LDS-DMA staged kernel and the segmented stream; built
 * only by `make variant`).  Weak: null in libxcsum.so, so its
 * geometry table and dispatch hold the product kernels only. */
#define XCSUM_VARIANT_HOOK __attribute__((weak, visibility("hidden")))
XCSUM_VARIANT_HOOK bool variant_supported(Geometry g);
XCSUM_VARIANT_HOOK hipError_t launch_variant(const CsumArgs &a, Geometry g, int cus, hipStream_t s);
Geometry pick_geometry(uint32_t len_hint);
/* gather: stage each frame on its own (pinned host copy, frames packed)
 * instead of copying the UMEM range the chunk's frames span -- for frames
 * that are not known to lie in one mapped buffer (the packet.c mirror's
 * absolute pointers) and to move only the bytes the kernel reads */
int batch_host_impl(struct xcsum_ctx *c, uint8_t *h_umem, const struct xcsum_desc *h_desc,
		    uint32_t n, uint16_t *h_out, uint16_t *h_out_ip, uint32_t mode, uint32_t flags,
		    bool gather = false);
bool geometry_supported(Geometry g);
/* the claimed-tail schedule of csum_kernel (XCSUM_TUNE_CLAIM, xcsum_csum.h):
 * a counter pair of the context's ring, the static share in 64ths, wave
 * steps per claim */
struct ClaimParams {
	uint32_t *claim;
	uint32_t static_64, chunk_steps;
};
hipError_t launch_csum(const CsumArgs &a, Geometry g, int cus, hipStream_t s,
		       const ClaimParams *cp = nullptr);
/* A/B only (csrc/variants/xcsum_claim.hip, `make variant`; null in
 * libxcsum.so): -> hipErrorNotSupported for a geometry without a
 * claimed-tail kernel */
XCSUM_VARIANT_HOOK hipError_t launch_csum_claim_f0(const CsumArgs &a, Geometry g, int cus,
						   const ClaimParams &cp, hipStream_t s);
XCSUM_VARIANT_HOOK hipError_t launch_csum_claim_f1(const CsumArgs &a, Geometry g, int cus,
						   const ClaimParams &cp, hipStream_t s);
XCSUM_VARIANT_HOOK hipError_t launch_csum_claim_f2(const CsumArgs &a, Geometry g, int cus,
						   const ClaimParams &cp, hipStream_t s);
/* csum_kernel per feature set (xcsum_csum_f{0,1,2}.hip): plain, + VERIFY, + IPHDR */
hipError_t launch_csum_f0(const CsumArgs &a, Geometry g, int cus, hipStream_t s);
hipError_t launch_csum_f1(const CsumArgs &a, Geometry g, int cus, hipStream_t s);
hipError_t launch_csum_f2(const CsumArgs &a, Geometry g, int cus, hipStream_t s);
/* XCSUM_F_INPLACE without IPHDR at (16,2,6): the kernel with each frame's
 * first 4 chunks loaded temporally (xcsum_csum_tl.hip) */
hipError_t launch_csum_inplace_tl(const CsumArgs &a, Geometry g, int cus, hipStream_t s);
/* XCSUM_F_IPHDR_ONLY: iph->check from the header alone (xcsum_iphdr.hip) */
hipError_t launch_iphdr(const CsumArgs &a, int fpt, hipStream_t s);
hipError_t launch_gen(uint8_t *d_umem, const struct xcsum_desc *d_desc, uint32_t n,
		      uint32_t family, uint64_t seed, uint64_t first_index, int max_blocks,
		      hipStream_t s);

struct Region {
	uint8_t *host;
	size_t size;
	uint8_t *dev;  /* device alias of the page-locked mapping (null: staged) */
	uint8_t *reg;  /* the address handed to hipHostRegister */
	bool mapped;   /* false: registered for bookkeeping only -- its pages may
			  be moved by transparent huge pages, so
			  the GPU never touches it; batches in it are staged */
};

struct StagePool;   /* xcsum_stage.h: the context's host copy threads */

/* Per-thread context.  Owns only scratch: the error counter and the staging
 * ring of the host-resident path. */
struct Ctx {
	int device;
	Tuning tune;                   /* xcsum_ctx_set_tuning */
	uint32_t *d_claim;             /* claimed tail: CLAIM_SLOTS counter pairs (lazy) */
	uint32_t claim_seq;            /* next slot */
	StagePool *stage_pool;         /* host copies split over threads (lazy threads) */
	int cus;
	int max_blocks;
	Geometry geom;                 /* forced geometry, G == 0: automatic */
	int blocks_per_cu;             /* forced grid cap, 0: automatic */
	int order_rlog, order_tlog;    /* visiting order, rlog < 0: automatic */
	unsigned long long *d_err;
	uint32_t *d_rx_part;           /* RX_PART_MAX per-block receive counts */
	/* two-pass in-place schedule (xcsum_ctx_set_inplace): the result arrays
	 * the first pass writes, 2 x u16 per frame, grown on demand */
	int inplace_sched;
	uint32_t inplace_block;        /* second-pass store width (ScatterArgs) */
	int inplace_tl;                /* in place without IPHDR at MTU: the
					  temporal-first-chunks kernel (1, default)
					  or the plain one (XCSUM_INPLACE_TL=0, A/B) */
	uint16_t *d_inplace;
	uint32_t inplace_cap;          /* frames */
	hipEvent_t inplace_done;       /* after the last two-pass call's scatter */
	void *inplace_stream;          /* the stream of that call */
	bool inplace_recorded;         /* inplace_done was recorded */
	std::vector<Region> regions;
	/* caller streams the device entry points launched on: take_errors,
	 * unregister_umem and destroy wait for these, the host-path slots and
	 * the resident workgroups -- never for the whole device */
	std::vector<void *> streams_used;

	/* host path staging: NSLOT slots of frames + descriptors + results */
	static const int NSLOT = 2;
	hipStream_t streams[NSLOT];
	hipEvent_t done[NSLOT];
	uint8_t *d_frames[NSLOT];
	struct xcsum_desc *d_desc[NSLOT];
	uint16_t *d_out[NSLOT];
	uint16_t *h_out[NSLOT];        /* pinned */
	struct xcsum_rx_msg *d_rx_msgs[NSLOT];  /* receive records (lazy) */
	struct xcsum_rx_msg *h_rx_msgs[NSLOT];  /* pinned */
	struct xcsum_rx_msg *v_rx_msgs[NSLOT];  /* their device address */
	uint8_t *h_stage[NSLOT];       /* gathered frames (pinned, lazy) */
	struct xcsum_desc *h_dstage[NSLOT];     /* their descriptors (pinned, lazy) */
	/* device addresses of the pinned stage, its descriptors and the result
	 * slot: small gathered batches are read and answered in place by the
	 * kernel, no copies (batch_host_impl) */
	uint8_t *v_stage[NSLOT];
	struct xcsum_desc *v_dstage[NSLOT];
	uint16_t *v_out[NSLOT];
	size_t frame_cap;              /* bytes per slot */
	uint32_t desc_cap;             /* frames per slot */

	/* resident server for small host batches (xcsum_ctx_set_resident,
	 * xcsum_resident.hip): res_wg workgroups, 0 = off */
	int res_wg;
	uint32_t res_idle_us;
	uint32_t res_life_us;          /* workgroups leave after this long alive */
	uint32_t res_max_frames;       /* larger batches take the launched path */
	ResidentBell *res_bell;        /* the doorbell, pinned host memory (lazy) */
	ResidentBell *res_vbell;       /* its device alias */
	ResidentDone *res_done;        /* pinned, coherent */
	ResidentDone *res_vdone;       /* its device alias */
	hipStream_t res_stream;
	bool res_live;                 /* launched, not yet seen gone */
	uint32_t res_seq;              /* last sequence number issued (0: none) */
	uint32_t res_gen;              /* generation of the last launch (skips 0) */
	/* XCSUM_RESIDENT_TRACE=1: per-call timing, printed by xcsum_ctx_destroy */
	bool res_trace;
	uint64_t res_limit_cut;        /* test hook: XCSUM_RESIDENT_LIMIT_CUT */
	bool res_inline;               /* XCSUM_RESIDENT_INLINE=0 turns it off */
	uint64_t res_calls;
	double res_spin_us, res_call_us;
};

} /* namespace xcsum */

struct xcsum_ctx : xcsum::Ctx {};

#endif
