/*
 * xcsum_scatter.hip -- second pass of the two-pass in-place schedule.
 *
 * libxudp's TX path stores udp->check (and, for IPv4, iph->check) into every
 * frame before it publishes the frame (xudp/packet.c:156-194, driven from
 * tx.c:696-726).  Done inside the checksum pass, those 2-byte stores leave a
 * dirty partial line per field among the pass's reads, and their write-backs
 * interleave with the read stream on every HBM channel: the fused in-place
 * pass ran at 0.34 ms where the plain pass takes 0.23 ms with 2.8 % more
 * bytes.  The two-pass schedule (xcsum_batch_device with
 * XCSUM_F_INPLACE, schedule XCSUM_INPLACE_TWO_PASS) runs the plain pass into
 * a result array, then this kernel writes the fields: the writes come after
 * every read has been issued, as one short burst in frame order.
 *
 * It writes exactly the fields the fused pass writes: resolve() of
 * xcsum_csum.h decides the family and the frame's validity from the
 * descriptor length and, in AUTO mode, h_proto; a frame it calls malformed
 * is left untouched (the first pass counted it), the others get
 *   IPv4: res[p] at eth+40, with IPHDR res_ip[p] at eth+24;
 *   IPv6: res[p] at eth+60.
 * One thread per frame, grid-stride; the descriptor (16 B) and the result(s)
 * are coalesced loads, the field stores one per frame.
 */
#include "xcsum_frame.h"

namespace xcsum {

/* the two bytes of v (memory order) into byte offset o of the W-byte block
 * held as dwords w[] (static indices only: selects, no scratch) */
template <int N>
static __device__ __forceinline__ void patch_u16(uint32_t (&w)[N], uint32_t o, uint16_t v)
{
#pragma unroll
	for (int d = 0; d < N; d++)
#pragma unroll
		for (int k = 0; k < 2; k++) {
			const uint32_t pos = o + (uint32_t)k;
			const uint32_t sh = (pos & 3u) * 8u;
			const uint32_t nw = (w[d] & ~(0xffu << sh)) | ((uint32_t)((v >> (8 * k)) & 0xffu) << sh);
			w[d] = (pos >> 2) == (uint32_t)d ? nw : w[d];
		}
}

/* Store the field(s) of one W-byte block: the whole block, read and patched,
 * when it lies inside the frame (a complete block reaches the memory side
 * instead of a 2-byte partial write); else the 2-byte stores alone (the block
 * would reach into another frame, whose bytes are not this thread's). */
template <int W>
static __device__ __forceinline__ void store_block(uint8_t *eth, uint32_t len, uint8_t *blk,
						   uint32_t o1, uint16_t v1, bool two, uint32_t o2,
						   uint16_t v2, uint32_t p)
{
	/* a field at the block's last byte reaches into the next block: such a
	 * frame takes the 2-byte stores */
	if (blk >= eth && blk + W <= eth + len && o1 + 2 <= W && (!two || o2 + 2 <= W)) {
		uint32_t w[W / 4];
#pragma unroll
		for (int q = 0; q < W / 16; q++) {
			const u32x4 c = *((gu32x4 *)XB_LOAD(blk + 16 * q, 16, eth, eth + len, XB_SCATTER, p,
							   g_zero_chunk));
			w[4 * q] = c.x;
			w[4 * q + 1] = c.y;
			w[4 * q + 2] = c.z;
			w[4 * q + 3] = c.w;
		}
		patch_u16(w, o1, v1);
		if (two)
			patch_u16(w, o2, v2);
#pragma unroll
		for (int q = 0; q < W / 16; q++)
			if (XB_STORE(blk + 16 * q, 16, eth, eth + len, XB_SCATTER, p))
				*((u32x4 *)(blk + 16 * q)) = u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2],
								   w[4 * q + 3]};
		return;
	}
	if (XB_STORE(blk + o1, 2, eth, eth + len, XB_SCATTER, p))
		store_u16(blk + o1, v1);
	if (two && XB_STORE(blk + o2, 2, eth, eth + len, XB_SCATTER, p))
		store_u16(blk + o2, v2);
}

template <int W>
__global__ void __launch_bounds__(256) scatter_kernel(ScatterArgs a)
{
	const uint32_t stride = gridDim.x * 256u;
	for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < a.n; p += stride) {
		const u32x4 d = *((gu32x4 *)(a.desc + p));
		const uint16_t wire = a.res[p];
		const uint16_t ipc = a.res_ip ? a.res_ip[p] : (uint16_t)0;
		const uint64_t addr = (((uint64_t)d.y << 32) | d.x) - a.bias;
		const uint32_t len = d.z;
		uint8_t *eth = a.umem + addr;
		int mode = (int)a.mode;
		if (mode == XCSUM_MODE_AUTO) {
			/* as resolve(): h_proto only inside the frame */
			uint32_t proto = 0;
			if (len >= 14 && XB_IN(eth + 12, 2, eth, eth + len, XB_SCATTER, p))
				proto = ((uint32_t)eth[12] << 8) | eth[13];
			mode = proto == 0x0800u ? 0 : proto == 0x86DDu ? 2 : -1;
		}
		const uint32_t hdr = mode == 2 ? 54u : 34u;
		if (mode < 0 || len < hdr + 8u || len - hdr > 65535u)
			continue;
		const uint32_t fo = mode == 2 ? 60u : 40u;
		const bool ip = a.res_ip && mode != 2;
		if (W == 0) {
			if (XB_STORE(eth + fo, 2, eth, eth + len, XB_SCATTER, p))
				store_u16(eth + fo, wire);
			if (ip && XB_STORE(eth + 24, 2, eth, eth + len, XB_SCATTER, p))
				store_u16(eth + 24, ipc);
			continue;
		}
		constexpr uintptr_t M = W ? (uintptr_t)W - 1 : 0;
		uint8_t *b1 = (uint8_t *)((uintptr_t)(eth + fo) & ~M);
		uint8_t *b2 = (uint8_t *)((uintptr_t)(eth + 24) & ~M);
		if (!ip || b1 == b2) {
			store_block<W ? W : 16>(eth, len, b1, (uint32_t)(eth + fo - b1), wire, ip,
						(uint32_t)(eth + 24 - b1), ipc, p);
		} else {
			store_block<W ? W : 16>(eth, len, b2, (uint32_t)(eth + 24 - b2), ipc, false, 0, 0,
						p);
			store_block<W ? W : 16>(eth, len, b1, (uint32_t)(eth + fo - b1), wire, false, 0, 0,
						p);
		}
	}
}

hipError_t launch_scatter(const ScatterArgs &a, int cus, hipStream_t s)
{
	if (a.n == 0)
		return hipSuccess;
	uint64_t blocks = ((uint64_t)a.n + 255) / 256;
	const uint64_t cap = (uint64_t)cus * 8;
	if (blocks > cap)
		blocks = cap;
	(void)hipGetLastError();
	if (a.block == 64)
		hipLaunchKernelGGL(scatter_kernel<64>, dim3((unsigned)blocks), dim3(256), 0, s, a);
	else if (a.block == 32)
		hipLaunchKernelGGL(scatter_kernel<32>, dim3((unsigned)blocks), dim3(256), 0, s, a);
	else
		hipLaunchKernelGGL(scatter_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, s, a);
	return hipGetLastError();
}

} /* namespace xcsum */
