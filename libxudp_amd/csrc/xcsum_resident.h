/* xcsum_resident.h -- the doorbell of a resident checksum server
 * (xcsum_resident.hip), shared by the kernel and the host API. */
#ifndef XCSUM_RESIDENT_H
#define XCSUM_RESIDENT_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "xcsum.h"

namespace xcsum {

constexpr int RB_MAX_WG = 64;          /* workgroups (one bit each in a skip mask) */
constexpr int RB_DONE_STRIDE = 16;     /* one 64-byte line per workgroup's done word */
constexpr uint32_t RB_DESC_CAP = 4096; /* descriptors the doorbell holds */

/* request words: device addresses as (lo, hi) pairs */
enum {
	RB_UMEM = 0, RB_DESC = 2, RB_OUT = 4, RB_OUT_IP = 6, RB_BIAS = 8,
	RB_N = 10, RB_MODE = 11, RB_FLAGS = 12,
	RB_SEQ = 13,                   /* the request's own sequence number: a
					  request whose echo differs from seq is
					  not (yet) the one announced */
	RB_LIMIT = 14,                 /* (lo, hi): bytes readable from umem + 0
					  (desc.addr - bias + len must not pass it) */
	RB_REQ_WORDS = 16
};

/* A batch of at most RB_INLINE frames also carries its descriptors in the
 * two 64-byte lines after the request, three per line, each line with the
 * request's sequence number in word RB_INL_ECHO: the poll that reads the
 * request reads them too, which saves the workgroups the round trip for the
 * descriptors. */
constexpr uint32_t RB_INLINE = 6;
constexpr int RB_INL_ECHO = 12;

/* The doorbell, in pinned coherent host memory the workgroups read over
 * PCIe.  The host writes desc[] (always), the inline lines and req[], then
 * seq; `stop` asks the workgroups to leave.  Sequence numbers skip 0. */
/* words 2..13 of the doorbell: the context's stage, doorbell descriptor
 * array and result slot as (lo, hi) device-address pairs, which the
 * bounds-checked build checks every request's pointers against (RB_ALLOW_*
 * are u64 indices into allow[]) */
enum { RB_ALLOW_STAGE = 0, RB_ALLOW_DESC = 2, RB_ALLOW_OUT = 4, RB_ALLOW_N = 6 };

struct alignas(64) ResidentBell {
	uint32_t seq;                  /* words 0-63 are read by one load per poll */
	uint32_t stop;
	uint64_t allow[RB_ALLOW_N];    /* words 2-13 (written by the host, read with
					  every poll; only the debug build uses them) */
	uint32_t pad0[2];
	uint32_t req[16];              /* word 16 on */
	uint32_t inl[2][16];           /* word 32 on: descriptors 0-2, 3-5 */
	struct xcsum_desc desc[RB_DESC_CAP];
};

/* The answers, in pinned host memory (the host spins on them locally):
 * workgroup w stores done[RB_DONE_STRIDE * w] = seq when its part of request
 * seq is done, and done[RB_DONE_STRIDE * w + 1] = gen (its launch's
 * generation) as it leaves -- so the host learns that the workgroups are gone
 * without asking the HIP runtime on every call. */
constexpr int RB_LEFT = 1;
/* a workgroup that finds descriptors of its frames outside the request's
 * limit reads none of those frames and reports the first: [2] = seq,
 * [3] = frame index, [4..5] = desc.addr, [6] = desc.len (a bad request never
 * faults the GPU) */
constexpr int RB_BAD = 2;
/* the bounds-checked build's breadcrumb: before serving request seq a
 * workgroup stores [8] = seq, [9..10] = umem, [11] = n, [12..13] = desc, so
 * a fault names what the workgroups were reading (pinned host memory
 * survives the fault) */
constexpr int RB_CRUMB = 8;
struct alignas(64) ResidentDone {
	uint32_t done[RB_MAX_WG * RB_DONE_STRIDE];
};

hipError_t launch_resident(ResidentBell *v_bell, ResidentDone *v_done, unsigned long long *err,
			   int wg, uint32_t gen, uint32_t served0, uint32_t skip_seq,
			   uint64_t skip_mask, uint32_t idle_us, uint32_t life_us, hipStream_t s);

} /* namespace xcsum */

#endif
