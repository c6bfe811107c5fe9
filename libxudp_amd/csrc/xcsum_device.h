/* xcsum_device.h -- device helpers shared by the checksum, build and receive
 * kernels (one copy, so a fix reaches all three), and the per-device
 * occupancy cache their launchers use. */
#ifndef XCSUM_DEVICE_H
#define XCSUM_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include "xcsum_internal.h"

namespace xcsum {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

/* v_dot4_u32_u8: the bytes at even / odd addresses of a little-endian dword
 * (bytes 0 and 2 / 1 and 3) added to acc -- exact u32 sums */
static __device__ __forceinline__ uint32_t dot_even(uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot4(w, 0x00010001u, acc, false);
}
static __device__ __forceinline__ uint32_t dot_odd(uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot4(w, 0x01000100u, acc, false);
}

/* whole 16-byte chunk into E (bytes at even addresses) and O (odd) */
static __device__ __forceinline__ void accum(u32x4 v, uint32_t &E, uint32_t &O)
{
	E = dot_even(v.x, E); O = dot_odd(v.x, O);
	E = dot_even(v.y, E); O = dot_odd(v.y, O);
	E = dot_even(v.z, E); O = dot_odd(v.z, O);
	E = dot_even(v.w, E); O = dot_odd(v.w, O);
}

/* Sum over each aligned group of G lanes, result in every lane of the group.
 * DPP adds within a 16-lane row (quad_perm xor 1, xor 2, row_half_mirror,
 * row_mirror), then gfx950's v_permlane16_swap / v_permlane32_swap across
 * rows: ~8 VALU instructions for 64 lanes, no LDS round trip.  Must run with
 * every lane of the wave active. */
template <int G>
static __device__ __forceinline__ uint32_t seg_sum(uint32_t v)
{
	if (G >= 2)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false); /* ^1 */
	if (G >= 4)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false); /* ^2 */
	if (G >= 8)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
	if (G >= 16)
		v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
	if (G >= 32) {
		auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
		v = p[0] + p[1];
	}
	if (G >= 64) {
		auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
		v = q[0] + q[1];
	}
	return v;
}

/* ---- bounds checks (XCSUM_DEBUG_BOUNDS only; see xcsum_internal.h) ----
 * XB_IN(p, n, lo, hi, site, index): is [p, p + n) inside [lo, hi)?  Records
 * a violation when not.  XB_LOAD(...) yields p, or `safe` (a zero block) for
 * an access outside; XB_STORE(...) says whether to store; XB_IDX(i, n, site)
 * checks an array index.  Without the debug build: p / true, no code. */
#ifdef XCSUM_DEBUG_BOUNDS
static __device__ BoundsLog g_bounds;

static __device__ __noinline__ void bounds_fail(uint32_t site, uint32_t index, uint64_t addr,
						 uint64_t lo, uint64_t hi)
{
	const unsigned long long k = atomicAdd(&g_bounds.count, 1ull);
	if (k < (unsigned long long)BOUNDS_RECS) {
		BoundsRec r;
		r.site = site;
		r.index = index;
		r.addr = addr;
		r.lo = lo;
		r.hi = hi;
		g_bounds.rec[k] = r;
	}
}

static __device__ __forceinline__ bool xb_in(uint64_t a, uint64_t n, uint64_t lo, uint64_t hi,
					     uint32_t site, uint32_t index)
{
	if (a >= lo && a + n <= hi)
		return true;
	bounds_fail(site, index, a, lo, hi);
	return false;
}

#define XB_IN(p, n, lo, hi, site, index)                                                   \
	xb_in((uint64_t)(uintptr_t)(p), (uint64_t)(n), (uint64_t)(uintptr_t)(lo),          \
	      (uint64_t)(uintptr_t)(hi), (site), (uint32_t)(index))
#define XB_LOAD(p, n, lo, hi, site, index, safe)                                           \
	(XB_IN((p), (n), (lo), (hi), (site), (index)) ? (const uint8_t *)(p)               \
						      : (const uint8_t *)(safe))
#define XB_STORE(p, n, lo, hi, site, index) XB_IN((p), (n), (lo), (hi), (site), (index))
#define XB_IDX(i, n, site) xb_in((uint64_t)(i), 1, 0, (uint64_t)(n), (site), (uint32_t)(i))

/* this translation unit's log, read and cleared by xcsum_debug_bounds() */
static int bounds_take_tu(BoundsLog *out)
{
	BoundsLog z = {};
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bounds), sizeof(*out), 0,
				hipMemcpyDeviceToHost) != hipSuccess)
		return -1;
	return hipMemcpyToSymbol(HIP_SYMBOL(g_bounds), &z, sizeof(z), 0, hipMemcpyHostToDevice) ==
			       hipSuccess ? 0 : -1;
}
static BoundsReader g_bounds_reader = {bounds_take_tu, nullptr};
__attribute__((unused)) static const int g_bounds_registered =
	(g_bounds_reader.next = bounds_readers(), bounds_readers() = &g_bounds_reader, 0);
#else
#define XB_IN(p, n, lo, hi, site, index) true
#define XB_LOAD(p, n, lo, hi, site, index, safe) (p)
#define XB_STORE(p, n, lo, hi, site, index) true
#define XB_IDX(i, n, site) true
#endif

/* low 16 bits byte-swapped (host <-> network order of a 16-bit field) */
static __device__ __forceinline__ uint32_t bswap16(uint32_t x)
{
	return ((x >> 8) & 0xffu) | ((x & 0xffu) << 8);
}

/* Blocks per CU a kernel keeps resident on the current device, computed
 * once per (kernel, device) -- `cache` is the caller's per-kernel array.
 * Lock-free: concurrent first calls may both compute the same value. */
constexpr int OCC_MAX_DEVICES = 64;

template <typename F>
static inline int occupancy_cached(std::atomic<int> (&cache)[OCC_MAX_DEVICES], F compute)
{
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= OCC_MAX_DEVICES)
		return compute();
	int v = cache[dev].load(std::memory_order_relaxed);
	if (v <= 0) {
		v = compute();
		cache[dev].store(v, std::memory_order_relaxed);
	}
	return v;
}

} /* namespace xcsum */

#endif
