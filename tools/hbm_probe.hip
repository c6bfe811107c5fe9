/*
 * hbm_probe.hip -- measuring stick, not product code: the best plain
 * streaming READ rate this MI355X sustains (global_load_dwordx4, grid-stride,
 * per-thread u32 sum written once), to put the checksum kernel's HBM rate in
 * context next to the 8 TB/s spec.  Built by tools/Makefile into
 * tools/libhbmprobe.so; driven by tools/hbm_probe.py.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

template <bool NT, int UNROLL>
__global__ void __launch_bounds__(256) stream_read(const u32x4 *p, uint64_t n16, uint32_t *out)
{
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
		u32x4 v[UNROLL];
#pragma unroll
		for (int u = 0; u < UNROLL; u++)
			v[u] = NT ? __builtin_nontemporal_load((gu32x4 *)(p + i + u * stride))
				  : *((gu32x4 *)(p + i + u * stride));
#pragma unroll
		for (int u = 0; u < UNROLL; u++)
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	for (; i < n16; i += stride) {
		u32x4 v = *((gu32x4 *)(p + i));
		acc += v.x ^ v.y ^ v.z ^ v.w;
	}
	out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" int probe_stream_read(const void *p, uint64_t nbytes, uint32_t *out, int blocks,
				 int nt, int unroll, void *stream)
{
	uint64_t n16 = nbytes / 16;
	hipStream_t s = (hipStream_t)stream;
	const u32x4 *q = (const u32x4 *)p;
#define L(NT_, U_) hipLaunchKernelGGL((stream_read<NT_, U_>), dim3(blocks), dim3(256), 0, s, q, n16, out)
	if (nt) {
		if (unroll == 1) L(true, 1); else if (unroll == 2) L(true, 2); else if (unroll == 4) L(true, 4); else L(true, 8);
	} else {
		if (unroll == 1) L(false, 1); else if (unroll == 2) L(false, 2); else if (unroll == 4) L(false, 4); else L(false, 8);
	}
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Read+write ceiling (the build kernel's copy modes move every byte twice):
 * grid-stride dwordx4 copy, UNROLL loads in flight before the stores;
 * NTS = nontemporal stores (the build kernel's destination is not re-read). */
template <bool NTS, int UNROLL>
__global__ void __launch_bounds__(256) stream_copy(const u32x4 *p, u32x4 *q, uint64_t n16)
{
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	typedef __attribute__((address_space(1))) u32x4 gw32x4;
	for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
		u32x4 v[UNROLL];
#pragma unroll
		for (int u = 0; u < UNROLL; u++)
			v[u] = __builtin_nontemporal_load((gu32x4 *)(p + i + u * stride));
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			if (NTS)
				__builtin_nontemporal_store(v[u], (gw32x4 *)(q + i + u * stride));
			else
				*((gw32x4 *)(q + i + u * stride)) = v[u];
		}
	}
	for (; i < n16; i += stride)
		q[i] = p[i];
}

extern "C" int probe_stream_copy(const void *p, void *q, uint64_t nbytes, int blocks, int nts,
				 int unroll, void *stream)
{
	uint64_t n16 = nbytes / 16;
	hipStream_t s = (hipStream_t)stream;
	const u32x4 *a = (const u32x4 *)p;
	u32x4 *b = (u32x4 *)q;
#define L(N_, U_) hipLaunchKernelGGL((stream_copy<N_, U_>), dim3(blocks), dim3(256), 0, s, a, b, n16)
	if (nts) {
		if (unroll == 1) L(true, 1); else if (unroll == 2) L(true, 2); else if (unroll == 4) L(true, 4); else L(true, 8);
	} else {
		if (unroll == 1) L(false, 1); else if (unroll == 2) L(false, 2); else if (unroll == 4) L(false, 4); else L(false, 8);
	}
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Slot-layout probe: read span16*16 bytes at a 16-aligned offset inside each
 * slot_bytes slot (xudp's UMEM: one frame per 4096-B chunk), nothing else.
 * off(slot) = off0 + (slot * rot16 % nrot) * 16: rot16 = 0 is xudp's fixed
 * offset; rot16 != 0 spreads the spans over the slot to see whether the
 * fixed in-slot offset (and so a fixed subset of HBM channels) costs rate. */
__global__ void __launch_bounds__(256) slot_read(const uint8_t *p, uint64_t nslots,
						 uint32_t slot_bytes, uint32_t span16, uint32_t off0,
						 uint32_t rot16, uint32_t nrot, uint32_t perm_mul,
						 uint32_t perm_shift, uint32_t *out)
{
	const uint64_t total = nslots * span16;
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (; i < total; i += stride) {
		uint64_t slot = i / span16;
		uint32_t w = (uint32_t)(i - slot * span16);
		if (perm_mul) {	/* visit slot groups of 2^perm_shift in a scattered order */
			uint64_t grp = slot >> perm_shift, ng = nslots >> perm_shift;
			slot = (((grp * perm_mul) & (ng - 1)) << perm_shift) |
			       (slot & ((1ull << perm_shift) - 1));
		}
		uint32_t off = off0 + (nrot ? (uint32_t)((slot * rot16) % nrot) * 16 : 0);
		u32x4 v = __builtin_nontemporal_load(
			(gu32x4 *)(p + slot * slot_bytes + off + (uint64_t)w * 16));
		acc += v.x ^ v.y ^ v.z ^ v.w;
	}
	out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" int probe_slot_read(const void *p, uint64_t nslots, uint32_t slot_bytes,
			       uint32_t span16, uint32_t off0, uint32_t rot16, uint32_t nrot,
			       uint32_t perm_mul, uint32_t perm_shift,
			       uint32_t *out, int blocks, void *stream)
{
	hipLaunchKernelGGL(slot_read, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
			   (const uint8_t *)p, nslots, slot_bytes, span16, off0, rot16, nrot,
			   perm_mul, perm_shift, out);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* In-place ceiling (the TX drop-in's mode, XCSUM_F_INPLACE | XCSUM_F_IPHDR):
 * the stream read of stream_read<true, 1> over the same buffer, plus one
 * 2-byte store per frame at eth + f1 and one at eth + f2 (udp->check at +40,
 * iph->check at +24), each issued by the thread that read the chunk holding
 * it, with a value taken from that chunk -- the write pattern of the
 * checksum kernel's in-place pass (one dirtied line per field per frame,
 * interleaved with the read stream) with none of its arithmetic.  Frames
 * are regular: frame j at j * fstride + off (packed layout, or xudp's
 * 4096-byte slots).  The candidate frame of a chunk comes from a double
 * product (exact to far below one frame at these sizes), corrected by one. */
__device__ __forceinline__ void probe_field_store(uint8_t *p, uint64_t i, u32x4 v, uint64_t fstride,
						  uint64_t off, uint64_t nframes, uint32_t f,
						  double inv)
{
	const int64_t x = (int64_t)(16 * i) - (int64_t)(off + f);   /* want j*fstride in [x, x+16) */
	if (x + 16 <= 0)
		return;
	int64_t j = x <= 0 ? 0 : (int64_t)((double)x * inv);
	if ((int64_t)(j * fstride) < x)
		j++;
	if (j >= 0 && (uint64_t)j < nframes && (int64_t)(j * fstride) < x + 16)
		*reinterpret_cast<uint16_t *>(p + j * fstride + off + f) = (uint16_t)(v.x ^ v.w);
}

template <int UNROLL>
__global__ void __launch_bounds__(256) stream_read_inplace(uint8_t *p, uint64_t n16, uint64_t fstride,
							    uint64_t off, uint64_t nframes,
							    uint32_t f1, uint32_t f2, double inv,
							    uint32_t *out)
{
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint32_t acc = 0;
	/* UNROLL chunks in flight per thread, then their stores */
	for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
		u32x4 v[UNROLL];
#pragma unroll
		for (int u = 0; u < UNROLL; u++)
			v[u] = __builtin_nontemporal_load((gu32x4 *)(p + 16 * (i + u * stride)));
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
			probe_field_store(p, i + u * stride, v[u], fstride, off, nframes, f1, inv);
			if (f2 != f1)
				probe_field_store(p, i + u * stride, v[u], fstride, off, nframes, f2, inv);
		}
	}
	for (; i < n16; i += stride) {
		const u32x4 v = __builtin_nontemporal_load((gu32x4 *)(p + 16 * i));
		acc += v.x ^ v.y ^ v.z ^ v.w;
		probe_field_store(p, i, v, fstride, off, nframes, f1, inv);
		if (f2 != f1)
			probe_field_store(p, i, v, fstride, off, nframes, f2, inv);
	}
	out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" int probe_stream_read_inplace(void *p, uint64_t nbytes, uint64_t fstride, uint64_t off,
					 uint64_t nframes, uint32_t f1, uint32_t f2, uint32_t *out,
					 int blocks, int unroll, void *stream)
{
	if (fstride < 16 || !nframes)
		return -1;
	/* no store past the buffer: the last frame's fields lie below nbytes */
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 2 > nbytes)
		return -1;
#define L(U_) hipLaunchKernelGGL((stream_read_inplace<U_>), dim3(blocks), dim3(256), 0,           \
				    (hipStream_t)stream, (uint8_t *)p, nbytes / 16, fstride, off, nframes, \
				    f1, f2, 1.0 / (double)fstride, out)
	if (unroll >= 4)
		L(4);
	else if (unroll >= 2)
		L(2);
	else
		L(1);
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Two-pass schedule of the in-place probe: the plain stream read (no
 * stores), then a second launch that stores the 2-byte field(s) of every
 * frame, one thread per frame, in frame order -- the write pattern of the
 * library's two-pass in-place schedule (xcsum_scatter.hip) with none of its
 * arithmetic.  Both launches go on `stream`; time them together. */
__global__ void __launch_bounds__(256) scatter_fields(uint8_t *p, uint64_t fstride, uint64_t off,
						      uint64_t nframes, uint32_t f1, uint32_t f2)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < nframes; j += stride) {
		uint8_t *e = p + j * fstride + off;
		*reinterpret_cast<uint16_t *>(e + f1) = (uint16_t)j;
		if (f2 != f1)
			*reinterpret_cast<uint16_t *>(e + f2) = (uint16_t)(j >> 16);
	}
}

extern "C" int probe_stream_read_twopass(void *p, uint64_t nbytes, uint64_t fstride, uint64_t off,
					 uint64_t nframes, uint32_t f1, uint32_t f2, uint32_t *out,
					 int blocks, void *stream)
{
	if (fstride < 16 || !nframes || (f1 & 1) || (f2 & 1) || (off & 1))
		return -1;
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 2 > nbytes)
		return -1;
	hipLaunchKernelGGL((stream_read<true, 4>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
			   (const u32x4 *)p, nbytes / 16, out);
	uint64_t sb = (nframes + 255) / 256;
	if (sb > (uint64_t)blocks)
		sb = (uint64_t)blocks;
	hipLaunchKernelGGL(scatter_fields, dim3((unsigned)sb), dim3(256), 0, (hipStream_t)stream,
			   (uint8_t *)p, fstride, off, nframes, f1, f2);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* The second pass with whole-block writes: for each field, the W-byte block
 * (W = 32: a sector, 64: a line) holding it is read, patched and written
 * back in full (W/16 dwordx4 loads, then as many stores), so the memory
 * side sees complete blocks rather than 2-byte partial writes.  Blocks that
 * hold both fields are written once. */
template <int W>
__global__ void __launch_bounds__(256) scatter_blocks(uint8_t *p, uint64_t fstride, uint64_t off,
						      uint64_t nframes, uint32_t f1, uint32_t f2)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < nframes; j += stride) {
		uint8_t *e = p + j * fstride + off;
		uint8_t *b1 = (uint8_t *)((uintptr_t)(e + f1) & ~(uintptr_t)(W - 1));
		uint8_t *b2 = (uint8_t *)((uintptr_t)(e + f2) & ~(uintptr_t)(W - 1));
		const int nb = b1 == b2 ? 1 : 2;
		for (int k = 0; k < nb; k++) {
			uint8_t *b = k ? b2 : b1;
			u32x4 v[W / 16];
#pragma unroll
			for (int q = 0; q < W / 16; q++)
				v[q] = *((gu32x4 *)(b + 16 * q));
			v[0].x ^= (uint32_t)j;   /* "patch" */
#pragma unroll
			for (int q = 0; q < W / 16; q++)
				*((u32x4 *)(b + 16 * q)) = v[q];
		}
	}
}

/* stream read, then the block-write second pass (W = 32 or 64) */
extern "C" int probe_stream_read_twopass_blocks(void *p, uint64_t nbytes, uint64_t fstride,
						uint64_t off, uint64_t nframes, uint32_t f1,
						uint32_t f2, uint32_t *out, int blocks, int W,
						int read_first, void *stream)
{
	if (fstride < 64 || !nframes || ((uintptr_t)p & 63))
		return -1;
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 64 > nbytes)
		return -1;
	if (read_first)
		hipLaunchKernelGGL((stream_read<true, 4>), dim3(blocks), dim3(256), 0,
				   (hipStream_t)stream, (const u32x4 *)p, nbytes / 16, out);
	uint64_t sb = (nframes + 255) / 256;
	if (sb > (uint64_t)blocks)
		sb = (uint64_t)blocks;
	if (W == 64)
		hipLaunchKernelGGL((scatter_blocks<64>), dim3((unsigned)sb), dim3(256), 0,
				   (hipStream_t)stream, (uint8_t *)p, fstride, off, nframes, f1, f2);
	else
		hipLaunchKernelGGL((scatter_blocks<32>), dim3((unsigned)sb), dim3(256), 0,
				   (hipStream_t)stream, (uint8_t *)p, fstride, off, nframes, f1, f2);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* the 2-byte second pass alone (no read pass), to time the stores by themselves */
extern "C" int probe_scatter_fields(void *p, uint64_t nbytes, uint64_t fstride, uint64_t off,
				    uint64_t nframes, uint32_t f1, uint32_t f2, int blocks,
				    void *stream)
{
	if (fstride < 16 || !nframes || (f1 & 1) || (f2 & 1) || (off & 1))
		return -1;
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 2 > nbytes)
		return -1;
	uint64_t sb = (nframes + 255) / 256;
	if (sb > (uint64_t)blocks)
		sb = (uint64_t)blocks;
	hipLaunchKernelGGL(scatter_fields, dim3((unsigned)sb), dim3(256), 0, (hipStream_t)stream,
			   (uint8_t *)p, fstride, off, nframes, f1, f2);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* frame j whose field at eth + f lies in chunk i, or -1 (as probe_field_store) */
__device__ __forceinline__ int64_t probe_field_frame(uint64_t i, uint64_t fstride, uint64_t off,
						     uint64_t nframes, uint32_t f, double inv)
{
	const int64_t x = (int64_t)(16 * i) - (int64_t)(off + f);
	if (x + 16 <= 0)
		return -1;
	int64_t j = x <= 0 ? 0 : (int64_t)((double)x * inv);
	if ((int64_t)(j * fstride) < x)
		j++;
	return j >= 0 && (uint64_t)j < nframes && (int64_t)(j * fstride) < x + 16 ? j : -1;
}

/* The in-place probe with the chunks that hold a field loaded temporally
 * (allocated in L2 / the Infinity Cache, so the store that follows finds the
 * line cached) and every other chunk nontemporal. */
__global__ void __launch_bounds__(256) stream_read_inplace_tl(uint8_t *p, uint64_t n16,
							    uint64_t fstride, uint64_t off,
							    uint64_t nframes, uint32_t f1,
							    uint32_t f2, double inv, uint32_t *out)
{
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (; i < n16; i += stride) {
		const int64_t j1 = probe_field_frame(i, fstride, off, nframes, f1, inv);
		const int64_t j2 = f2 != f1 ? probe_field_frame(i, fstride, off, nframes, f2, inv) : -1;
		u32x4 v;
		if (j1 >= 0 || j2 >= 0)
			v = *((gu32x4 *)(p + 16 * i));
		else
			v = __builtin_nontemporal_load((gu32x4 *)(p + 16 * i));
		acc += v.x ^ v.y ^ v.z ^ v.w;
		if (j1 >= 0)
			*reinterpret_cast<uint16_t *>(p + j1 * fstride + off + f1) = (uint16_t)(v.x ^ v.w);
		if (j2 >= 0)
			*reinterpret_cast<uint16_t *>(p + j2 * fstride + off + f2) = (uint16_t)(v.y ^ v.w);
	}
	out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" int probe_stream_read_inplace_tl(void *p, uint64_t nbytes, uint64_t fstride,
					    uint64_t off, uint64_t nframes, uint32_t f1,
					    uint32_t f2, uint32_t *out, int blocks, void *stream)
{
	if (fstride < 16 || !nframes || (f1 & 1) || (f2 & 1) || (off & 1))
		return -1;
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 2 > nbytes)
		return -1;
	hipLaunchKernelGGL(stream_read_inplace_tl, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
			   (uint8_t *)p, nbytes / 16, fstride, off, nframes, f1, f2,
			   1.0 / (double)fstride, out);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* The in-place probe with whole-block stores from the reading wave: every
 * thread reads its 16-B chunk (grid-stride, consecutive threads hold
 * consecutive chunks); when the W-byte block holding the chunk contains a
 * field of some frame, every thread of that block stores its chunk back (the
 * field's bytes patched), so the block reaches L2 as one complete W-byte
 * write from one wave instruction (W = 16: only the field's chunk).  Frame
 * ownership is ignored (garbage in the fields, as in the other probes). */
template <int W>
__global__ void __launch_bounds__(256) stream_read_inplace_blk(uint8_t *p, uint64_t n16,
							     uint64_t fstride, uint64_t off,
							     uint64_t nframes, uint32_t f1,
							     uint32_t f2, double inv, uint32_t *out)
{
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (; i < n16; i += stride) {
		u32x4 v = __builtin_nontemporal_load((gu32x4 *)(p + 16 * i));
		acc += v.x ^ v.y ^ v.z ^ v.w;
		/* does this chunk's W-block hold a field? look at each chunk of it */
		const uint64_t b0 = (16 * i) / W * (W / 16);
		bool hit = false;
#pragma unroll
		for (int q = 0; q < W / 16; q++) {
			hit |= probe_field_frame(b0 + q, fstride, off, nframes, f1, inv) >= 0;
			if (f2 != f1)
				hit |= probe_field_frame(b0 + q, fstride, off, nframes, f2, inv) >= 0;
		}
		if (hit) {
			v.x ^= 1u;
			*((u32x4 *)(p + 16 * i)) = v;
		}
	}
	out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" int probe_stream_read_inplace_blk(void *p, uint64_t nbytes, uint64_t fstride,
					     uint64_t off, uint64_t nframes, uint32_t f1,
					     uint32_t f2, uint32_t *out, int blocks, int W,
					     void *stream)
{
	if (fstride < 16 || !nframes || ((uintptr_t)p & 127))
		return -1;
#define L(W_) hipLaunchKernelGGL((stream_read_inplace_blk<W_>), dim3(blocks), dim3(256), 0,        \
				 (hipStream_t)stream, (uint8_t *)p, nbytes / 16, fstride, off, nframes, \
				 f1, f2, 1.0 / (double)fstride, out)
	if (W == 16) L(16);
	else if (W == 32) L(32);
	else if (W == 64) L(64);
	else L(128);
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* The second pass as blind whole-block writes: for each field, the W-byte
 * block holding it is written in full with junk, no load of it first -- what
 * full-block stores cost when the data comes from elsewhere (registers, a
 * side buffer) rather than from a read of the line. */
template <int W>
__global__ void __launch_bounds__(256) scatter_blind(uint8_t *p, uint64_t fstride, uint64_t off,
						     uint64_t nframes, uint32_t f1, uint32_t f2)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < nframes; j += stride) {
		uint8_t *e = p + j * fstride + off;
		uint8_t *b1 = (uint8_t *)((uintptr_t)(e + f1) & ~(uintptr_t)(W - 1));
		uint8_t *b2 = (uint8_t *)((uintptr_t)(e + f2) & ~(uintptr_t)(W - 1));
		const u32x4 v = {(uint32_t)j, (uint32_t)j * 3u, (uint32_t)j * 5u, (uint32_t)j * 7u};
#pragma unroll
		for (int q = 0; q < W / 16; q++)
			*((u32x4 *)(b1 + 16 * q)) = v;
		if (b2 != b1)
#pragma unroll
			for (int q = 0; q < W / 16; q++)
				*((u32x4 *)(b2 + 16 * q)) = v;
	}
}

extern "C" int probe_stream_read_blind(void *p, uint64_t nbytes, uint64_t fstride, uint64_t off,
				       uint64_t nframes, uint32_t f1, uint32_t f2, uint32_t *out,
				       int blocks, int W, int read_first, void *stream)
{
	if (fstride < 64 || !nframes || ((uintptr_t)p & 127))
		return -1;
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 128 > nbytes)
		return -1;
	if (read_first)
		hipLaunchKernelGGL((stream_read<true, 4>), dim3(blocks), dim3(256), 0,
				   (hipStream_t)stream, (const u32x4 *)p, nbytes / 16, out);
	uint64_t sb = (nframes + 255) / 256;
	if (sb > (uint64_t)blocks)
		sb = (uint64_t)blocks;
#define L(W_) hipLaunchKernelGGL((scatter_blind<W_>), dim3((unsigned)sb), dim3(256), 0,             \
				 (hipStream_t)stream, (uint8_t *)p, fstride, off, nframes, f1, f2)
	if (W == 16) L(16);
	else if (W == 32) L(32);
	else if (W == 64) L(64);
	else L(128);
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* The second pass as a copy of saved blocks: the 64-byte block holding each
 * field was saved by the first pass into a compact side array (64 B per
 * block, in frame order); this pass streams that array and writes every
 * block back whole -- four lanes per block, one 16-byte store each, so the
 * memory side sees complete 64-byte writes and reads only the side array. */
__global__ void __launch_bounds__(256) copy_blocks(uint8_t *p, const uint8_t *side,
						   uint64_t fstride, uint64_t off, uint64_t nframes,
						   uint32_t f1, uint32_t f2)
{
	const uint32_t nb = ((off + f1) & ~63ull) == ((off + f2) & ~63ull) ? 1u : 2u;
	const uint64_t total = nframes * nb * 4;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += stride) {
		const uint64_t j = g / (4 * nb);
		const uint32_t k = (uint32_t)(g / 4 % nb), q = (uint32_t)(g & 3);
		uint8_t *e = p + j * fstride + off;
		uint8_t *b = (uint8_t *)((uintptr_t)(e + (k ? f2 : f1)) & ~(uintptr_t)63);
		const u32x4 v = __builtin_nontemporal_load((gu32x4 *)(side + 16 * g));
		*((u32x4 *)(b + 16 * q)) = v;
	}
}

extern "C" int probe_stream_read_copy(void *p, uint64_t nbytes, uint64_t fstride, uint64_t off,
				      uint64_t nframes, uint32_t f1, uint32_t f2, void *side,
				      uint64_t side_bytes, uint32_t *out, int blocks, int read_first,
				      void *stream)
{
	if (fstride < 64 || !nframes || ((uintptr_t)p & 127))
		return -1;
	if ((nframes - 1) * fstride + off + (f1 > f2 ? f1 : f2) + 128 > nbytes)
		return -1;
	if (side_bytes < nframes * 128)
		return -1;
	if (read_first)
		hipLaunchKernelGGL((stream_read<true, 4>), dim3(blocks), dim3(256), 0,
				   (hipStream_t)stream, (const u32x4 *)p, nbytes / 16, out);
	hipLaunchKernelGGL(copy_blocks, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (uint8_t *)p,
			   (const uint8_t *)side, fstride, off, nframes, f1, f2);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Header-only probe (round 5): the memory accesses of the library's
 * XCSUM_F_IPHDR_ONLY kernel (csrc/xcsum_iphdr.hip) with none of its
 * arithmetic -- per frame the 16-byte descriptor (coalesced), the seven dwords
 * at (eth + 12) & ~3 (one dwordx4 + one dwordx3, the header line), and with
 * `write` a 2-byte store at eth + 24 that depends on them -- FPT = 4 frames per
 * thread, all loads issued first, one launch per batch.  write 2/3/4 store the
 * whole 32-byte sector / 64-byte block / 128-byte line holding eth + 24
 * instead (blind, data not kept): whether a full-sector write-back is
 * cheaper than a partial one at the memory side; write 5/6/7 the 2-byte
 * store nontemporal / with sc0 sc1 / with nt (its cache policy).  The same-run ceiling
 * of an access pattern that is one scattered line read (and one scattered
 * partial write) per frame, not a stream. */
struct probe_desc { uint64_t addr; uint32_t len, options; };
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

/* LD: how the header dwords are loaded -- 0 plain (the library's kernel),
 * 1 nontemporal, 2..4 inline global loads with cache-policy bits "nt",
 * "sc1", "sc0 sc1" (whether the L2 then requests less than a 128-byte line
 * per scattered access is what the variants measure) */
template <int LD>
static __device__ __forceinline__ void load_hdr(const uint8_t *w, u32x4 &a, u32x3 &b)
{
	typedef const __attribute__((address_space(1))) u32x4 g4;
	typedef const __attribute__((address_space(1))) u32x3 g3;
	if (LD == 0) {
		a = *((g4 *)w);
		b = *((g3 *)(w + 16));
	} else if (LD == 1) {
		a = __builtin_nontemporal_load((g4 *)w);
		b = __builtin_nontemporal_load((g3 *)(w + 16));
	} else if (LD == 2) {
		asm volatile("global_load_dwordx4 %0, %2, off nt\n\t"
			     "global_load_dwordx3 %1, %2, off offset:16 nt"
			     : "=&v"(a), "=&v"(b) : "v"(w) : "memory");
	} else if (LD == 3) {
		asm volatile("global_load_dwordx4 %0, %2, off sc1\n\t"
			     "global_load_dwordx3 %1, %2, off offset:16 sc1"
			     : "=&v"(a), "=&v"(b) : "v"(w) : "memory");
	} else {
		asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
			     "global_load_dwordx3 %1, %2, off offset:16 sc0 sc1"
			     : "=&v"(a), "=&v"(b) : "v"(w) : "memory");
	}
}

template <int LD>
__global__ void __launch_bounds__(256) header_touch(uint8_t *umem, const probe_desc *desc,
						    uint32_t n, int write, uint32_t *out)
{
	constexpr int F = 4;
	const uint32_t q0 = blockIdx.x * (256u * F) + threadIdx.x;
	u32x4 d[F];
#pragma unroll
	for (int j = 0; j < F; j++) {
		const uint32_t q = q0 + 256u * j;
		d[j] = *((gu32x4 *)(desc + (q < n ? q : n - 1)));
	}
	__builtin_amdgcn_sched_barrier(0);
	u32x4 a[F];
	u32x3 b[F];
#pragma unroll
	for (int j = 0; j < F; j++) {
		const uint8_t *h = umem + ((((uint64_t)d[j].y << 32) | d[j].x) + 12);
		load_hdr<LD>((const uint8_t *)((uintptr_t)h & ~(uintptr_t)3), a[j], b[j]);
	}
	if (LD >= 2)   /* the inline loads are invisible to the waitcnt pass */
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	uint32_t acc = 0;
#pragma unroll
	for (int j = 0; j < F; j++) {
		const uint32_t v = a[j].x ^ a[j].y ^ a[j].z ^ a[j].w ^ b[j].x ^ b[j].y ^ b[j].z;
		acc ^= v;
		if (write && q0 + 256u * j < n) {
			uint8_t *e = umem + (((uint64_t)d[j].y << 32) | d[j].x);
			typedef __attribute__((address_space(1))) uint16_t w2;
			if (write == 1) {
				e[24] = (uint8_t)v;
				e[25] = (uint8_t)(v >> 8);
			} else if (write == 5) {
				__builtin_nontemporal_store((uint16_t)v, (w2 *)(e + 24));
			} else if (write == 6) {
				asm volatile("global_store_short %0, %1, off sc0 sc1"
					     :: "v"(e + 24), "v"(v) : "memory");
			} else if (write == 7) {
				asm volatile("global_store_short %0, %1, off nt"
					     :: "v"(e + 24), "v"(v) : "memory");
			} else {
				/* 2: the whole 32-byte sector holding eth + 24, 3: its
				 * 64-byte block, 4: its 128-byte line -- blind stores
				 * (the data is not kept; a timing probe) */
				const int sz = write == 2 ? 32 : write == 3 ? 64 : 128;
				typedef __attribute__((address_space(1))) u32x4 w4;
				w4 *s = (w4 *)((uintptr_t)(e + 24) & ~(uintptr_t)(sz - 1));
				const u32x4 x = {v, v ^ 1u, v ^ 2u, v ^ 3u};
				for (int k = 0; k < sz / 16; k++)
					s[k] = x;
			}
		}
	}
	if (acc == 0x9e3779b9u)
		out[blockIdx.x] = acc;
}

/* load_mode: LD above (0 = the library kernel's loads) */
extern "C" int probe_header_touch_mode(void *umem, const void *desc, uint32_t n, int write,
				       int load_mode, uint32_t *out, void *stream)
{
	if (!n || load_mode < 0 || load_mode > 4)
		return -1;
	const uint32_t blocks = (n + 1023) / 1024;
	auto *u = (uint8_t *)umem;
	auto *d = (const probe_desc *)desc;
	switch (load_mode) {
	case 0: hipLaunchKernelGGL(header_touch<0>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, u, d, n, write, out); break;
	case 1: hipLaunchKernelGGL(header_touch<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, u, d, n, write, out); break;
	case 2: hipLaunchKernelGGL(header_touch<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, u, d, n, write, out); break;
	case 3: hipLaunchKernelGGL(header_touch<3>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, u, d, n, write, out); break;
	default: hipLaunchKernelGGL(header_touch<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, u, d, n, write, out); break;
	}
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int probe_header_touch(void *umem, const void *desc, uint32_t n, int write,
				  uint32_t *out, void *stream)
{
	return probe_header_touch_mode(umem, desc, n, write, 0, out, stream);
}

/* Request-size calibration (round 5, MI355X_MICROARCH.md: "other access
 * widths are uncalibrated"): one thread per line of a strided set, reading
 * one dword from each 64-byte half of the 128-byte line named by `halves`
 * (bit 0: +0, bit 1: +64).  The L2's memory-side request counters per line,
 * for one half vs both, say whether a scattered access fetches 64 or 128
 * bytes. */
__global__ void __launch_bounds__(256) line_halves(const uint8_t *p, uint64_t nlines,
						   uint64_t stride, int halves, uint32_t *out)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	if (i >= nlines)
		return;
	const uint8_t *l = p + i * stride;
	uint32_t acc = 0;
	if (halves & 1)
		acc ^= *(const __attribute__((address_space(1))) uint32_t *)l;
	if (halves & 2)
		acc ^= *(const __attribute__((address_space(1))) uint32_t *)(l + 64);
	if (acc == 0x9e3779b9u)
		out[blockIdx.x] = acc;
}

extern "C" int probe_line_halves(const void *p, uint64_t nlines, uint64_t stride, int halves,
				 uint32_t *out, void *stream)
{
	if (!nlines || (stride & 127) || halves < 1 || halves > 3)
		return -1;
	const uint64_t blocks = (nlines + 255) / 256;
	hipLaunchKernelGGL(line_halves, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
			   (const uint8_t *)p, nlines, stride, halves, out);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Scattered-write probe (round 5): the stores of the IPv4 in-place build
 * (build_hdr_kernel, csrc/xcsum_build.hip) with nothing else -- per xudp
 * slot the 42 header bytes at F + 342 (2 + 8 + 16 + 16 bytes: one 64-byte
 * block, F + 320 .. F + 384) and, with `desc`, the frame's 16-byte
 * descriptor (coalesced), one thread per frame.  `msgs` adds the coalesced
 * 16-byte message load the build kernel makes per frame.  The same-run
 * bound of one scattered partial-block write per frame. */
__global__ void __launch_bounds__(256) slot_write(uint8_t *umem, uint32_t n, int desc, int msgs,
						  const u32x4 *m, u32x4 *d)
{
	typedef __attribute__((address_space(1))) u32x4 w4;
	typedef __attribute__((address_space(1))) uint64_t w8;
	typedef __attribute__((address_space(1))) uint16_t w2;
	const uint32_t q = blockIdx.x * 256u + threadIdx.x;
	if (q >= n)
		return;
	u32x4 v = {q, q ^ 0x55u, q + 7u, 0x0800u};
	if (msgs)
		v = *((gu32x4 *)(m + q));
	uint8_t *e = umem + (uint64_t)q * 4096u + 342u;
	*(w2 *)e = (uint16_t)v.x;
	*(w8 *)(e + 2) = ((uint64_t)v.y << 32) | v.z;
	*(w4 *)(e + 10) = v;
	*(w4 *)(e + 26) = v;
	if (desc) {
		const u32x4 o = {(uint32_t)(q * 4096u + 342u), 0u, 1514u, 0u};
		*(w4 *)(d + q) = o;
	}
}

extern "C" int probe_slot_write(void *umem, uint32_t n, int desc, int msgs, const void *m,
				void *d, void *stream)
{
	if (!n)
		return -1;
	hipLaunchKernelGGL(slot_write, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
			   (uint8_t *)umem, n, desc, msgs, (const u32x4 *)m, (u32x4 *)d);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Frame-line probe (round 6): the bytes the checksum kernel
 * must fetch on a sparse batch -- per frame its 16-byte descriptor and the
 * `line`-aligned span around [addr, addr + len) (line = 128: the request
 * size of a scattered read, profiles/r05/iphdr/r05j_line_probe.txt; 16: the
 * kernel's own chunks) -- read as a stream, with no arithmetic: one wave per
 * frame at a time (64 x 16 B = 1 KiB per load instruction, coalesced), F
 * frames per wave in flight, the frames taken in the kernel's visiting order
 * for sparse batches (2^rlog regions of 2^tlog-frame tiles,
 * csrc/xcsum_internal.h order_regions / frame_of).  The same-run ceiling of
 * xudp's slot layout (one ~1.5 KB frame per 4096-byte chunk): the contiguous
 * stream read of the whole buffer moves the gaps too. */
struct probe_order {
	uint32_t nlog, rshift, tshift, q;
};

static __device__ __forceinline__ uint32_t probe_frame_of(const probe_order &o, uint32_t p)
{
	if (o.rshift == 0)
		return p;
	const uint32_t t = p >> o.tshift;
	const uint32_t r = t & ((1u << o.rshift) - 1u);
	return ((r * o.q + (t >> o.rshift)) << o.tshift) | (p & ((1u << o.tshift) - 1u));
}

/* MAXI: load instructions per frame (64 lanes x 16 B each) */
template <bool NT, int F, int MAXI>
__global__ void __launch_bounds__(256) frame_lines(const uint8_t *umem, const probe_desc *desc,
						   uint32_t n, probe_order o, uint32_t line,
						   uint32_t *out)
{
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * 256u + threadIdx.x) >> 6);
	const uint32_t nwaves = gridDim.x * 4u;
	uint32_t acc = 0;
	for (uint32_t k0 = wave * F; k0 < o.nlog; k0 += nwaves * F) {
		u32x4 d[F];
#pragma unroll
		for (int f = 0; f < F; f++) {
			const uint32_t fr = probe_frame_of(o, k0 + f);
			d[f] = *((gu32x4 *)(desc + (k0 + f < o.nlog && fr < n ? fr : 0u)));
		}
		u32x4 v[F][MAXI];
#pragma unroll
		for (int f = 0; f < F; f++) {
			const uint32_t fr = probe_frame_of(o, k0 + f);
			const bool ok = k0 + f < o.nlog && fr < n;
			const uint64_t addr = ((uint64_t)d[f].y << 32) | d[f].x;
			const uint64_t lo = addr & ~(uint64_t)(line - 1);
			const uint64_t hi = (addr + d[f].z + line - 1) & ~(uint64_t)(line - 1);
#pragma unroll
			for (int j = 0; j < MAXI; j++) {
				const uint64_t at = lo + 16ull * (lane + 64u * j);
				const bool in = ok && at < hi;
				const gu32x4 *c = (gu32x4 *)(umem + (in ? at : lo));
				v[f][j] = in ? (NT ? __builtin_nontemporal_load(c) : *c) : u32x4{0u, 0u, 0u, 0u};
			}
		}
#pragma unroll
		for (int f = 0; f < F; f++)
#pragma unroll
			for (int j = 0; j < MAXI; j++)
				acc += v[f][j].x ^ v[f][j].y ^ v[f][j].z ^ v[f][j].w;
	}
	if (acc == 0x9e3779b9u)
		out[blockIdx.x] = acc;
}

/* line 16 or 128; every frame's span must fit 2 KiB (MTU frames, 4 frames
 * per wave in flight) or 10 KiB (jumbo frames, 2 in flight) */
extern "C" int probe_frame_spans2(const void *umem, const void *desc, uint32_t n, int rlog,
				  int tlog, uint32_t line, int nt, uint32_t max_span,
				  uint32_t *out, int blocks, void *stream)
{
	if (!n || (line != 16 && line != 128) || blocks <= 0 || rlog < 0 || tlog < 0 ||
	    rlog + tlog > 30 || max_span > 10240)
		return -1;
	probe_order o{n, 0u, 0u, 0u};
	if (rlog > 0 && n >= (1u << (rlog + tlog))) {   /* order_regions */
		const uint32_t ntiles = (n + (1u << tlog) - 1) >> tlog;
		const uint32_t q = (ntiles + (1u << rlog) - 1) >> rlog;
		o = probe_order{(q << rlog) << tlog, (uint32_t)rlog, (uint32_t)tlog, q};
	}
	auto *u = (const uint8_t *)umem;
	auto *d = (const probe_desc *)desc;
	hipStream_t st = (hipStream_t)stream;
#define L(NT_, F_, M_) hipLaunchKernelGGL((frame_lines<NT_, F_, M_>), dim3(blocks), dim3(256), 0, \
					   st, u, d, n, o, line, out)
	if (max_span <= 2048) {
		if (nt) L(true, 4, 2); else L(false, 4, 2);
	} else {
		if (nt) L(true, 2, 10); else L(false, 2, 10);
	}
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Wave-contiguous read (round 6): each wave streams its own contiguous
 * region of `region` bytes, 1 KiB per load instruction (64 lanes x 16 B),
 * UNROLL instructions in flight -- the other way to cut a stream read than
 * stream_read's grid stride, to see whether the same-run ceiling is the
 * read rate of the chip or of that one pattern. */
template <bool NT, int UNROLL>
__global__ void __launch_bounds__(256) wave_region_read(const u32x4 *p, uint64_t n16,
							uint64_t region16, uint32_t *out)
{
	const uint64_t lane = threadIdx.x & 63u;
	const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
	const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
	uint32_t acc = 0;
	for (uint64_t r0 = wave * region16; r0 < n16; r0 += nwaves * region16) {
		const uint64_t r1 = r0 + region16 < n16 ? r0 + region16 : n16;
		uint64_t i = r0 + lane;
		for (; i + 64u * (UNROLL - 1) < r1; i += 64u * UNROLL) {
			u32x4 v[UNROLL];
#pragma unroll
			for (int u = 0; u < UNROLL; u++)
				v[u] = NT ? __builtin_nontemporal_load((gu32x4 *)(p + i + 64u * u))
					  : *((gu32x4 *)(p + i + 64u * u));
#pragma unroll
			for (int u = 0; u < UNROLL; u++)
				acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
		}
		for (; i < r1; i += 64u) {
			const u32x4 v = *((gu32x4 *)(p + i));
			acc += v.x ^ v.y ^ v.z ^ v.w;
		}
	}
	if (acc == 0x9e3779b9u)
		out[blockIdx.x] = acc;
}

extern "C" int probe_wave_region_read(const void *p, uint64_t nbytes, uint64_t region,
				      int blocks, int nt, int unroll, uint32_t *out, void *stream)
{
	if (blocks <= 0 || region < 1024 || (region & 1023))
		return -1;
	const uint64_t n16 = nbytes / 16, r16 = region / 16;
	hipStream_t s = (hipStream_t)stream;
	const u32x4 *q = (const u32x4 *)p;
#define L(NT_, U_) hipLaunchKernelGGL((wave_region_read<NT_, U_>), dim3(blocks), dim3(256), 0, s, \
				      q, n16, r16, out)
	if (nt) {
		if (unroll == 2) L(true, 2); else if (unroll == 4) L(true, 4); else if (unroll == 8) L(true, 8); else L(true, 16);
	} else {
		if (unroll == 2) L(false, 2); else if (unroll == 4) L(false, 4); else if (unroll == 8) L(false, 8); else L(false, 16);
	}
#undef L
	return hipGetLastError() == hipSuccess ? 0 : -1;
}
