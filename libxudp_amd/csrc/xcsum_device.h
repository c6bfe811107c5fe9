/* xcsum_device.h -- device helpers shared by the checksum, build and receive
 * kernels (one copy, so a fix reaches all three), and the per-device
 * occupancy cache their launchers use. */
#ifndef XCSUM_DEVICE_H
#define XCSUM_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>

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
