/* xcsum_resident.h -- the doorbell of a resident checksum server
 * (xcsum_resident.hip), shared by the kernel and the host API. */
#ifndef XCSUM_RESIDENT_H
#define XCSUM_RESIDENT_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xcsum {

constexpr int RB_MAX_WG = 64;          /* workgroups (one bit each in a skip mask) */
constexpr int RB_DONE_STRIDE = 16;     /* one 64-byte line per workgroup's done word */

/* request words: device addresses as (lo, hi) pairs */
enum {
	RB_UMEM = 0, RB_DESC = 2, RB_OUT = 4, RB_OUT_IP = 6, RB_BIAS = 8,
	RB_N = 10, RB_MODE = 11, RB_FLAGS = 12,
	RB_REQ_WORDS = 13
};

/* In pinned, coherent host memory; the kernel sees it through its device
 * alias.  The host writes req[] and then seq (release); a workgroup answers
 * with done[RB_DONE_STRIDE * w] = seq.  Sequence numbers skip 0. */
struct ResidentBell {
	uint32_t seq;
	uint32_t stop;
	uint32_t pad0[14];
	uint32_t req[16];
	uint32_t done[RB_MAX_WG * RB_DONE_STRIDE];
};

hipError_t launch_resident(ResidentBell *v_bell, unsigned long long *err, int wg, uint32_t served0,
			   uint32_t skip_seq, uint64_t skip_mask, uint32_t idle_us, hipStream_t s);

} /* namespace xcsum */

#endif
