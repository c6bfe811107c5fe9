/*
 * xcsum_iphdr.hip -- libxudp's IPv4 TX checksum work on the device:
 * iph->check only (xcsum_batch_device with XCSUM_F_IPHDR_ONLY).
 *
 * For IPv4, xudp_packet_udp() computes one checksum per frame: the 20-byte
 * IP header's (xudp_checksum_half, cclinuxer/libxudp xudp/packet.c:43-66,
 * called from iph_build :83).  udp->check stays 0 (udp_build, packet.c:125).
 * That is the call xudp_frame_send makes for every IPv4 frame
 * (tx.c:654 inside the tx.c:696-726 loop).  It needs no payload byte: per
 * frame the 16-byte descriptor, the header (20 bytes at eth+14) and a 2-byte
 * store.  The UDP kernels (xcsum_kernels.hip) stream every payload byte, so
 * this is its own kernel: one thread per frame, FPT frames per thread with
 * all their loads issued before any is used.
 *
 * Per frame: seven dwords from (eth+12) & ~3 -- h_proto (AUTO mode) and the
 * header in one round of loads.  They stay inside [eth+9, eth+40), i.e.
 * inside every frame this path accepts (>= 42 bytes, as resolve() in
 * xcsum_csum.h).  The header sum is RFC 1071 over the 20 bytes with the
 * check field as 0, which equals xudp_checksum_half() on every header
 * iph_build() writes (its constant half, packet.c:45-47, is the version /
 * TTL / protocol / DF words iph_build stores, :73-79); with XCSUM_F_VERIFY
 * the check field is summed too and 0 means valid.
 */
#include "xcsum_frame.h"

namespace xcsum {

/* one frame's header, resolved from its descriptor */
struct HdrFrame {
	uint8_t *eth;
	const uint8_t *w;       /* dword base: (eth + 12) & ~3, or the zero block */
	uint32_t sh;            /* byte phase of eth + 12 in that dword */
	uint32_t len;
	bool load;              /* a candidate: its header is loaded */
};

/* the 20-byte IPv4 header at eth+14 from the seven dwords at (eth+12) & ~3
 * (phase sh): returns the memory-order value iph->check gets (VERIFY: 0 if
 * the header verifies); *proto = h_proto (big-endian value) */
static __device__ __forceinline__ uint16_t hdr_csum(const uint32_t (&w)[7], uint32_t sh,
						    bool verify, uint32_t *proto)
{
	uint32_t d[6];
#pragma unroll
	for (int j = 0; j < 6; j++)
		d[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);   /* bytes eth+12+4j.. */
	*proto = ((d[0] & 0xffu) << 8) | ((d[0] >> 8) & 0xffu);
	/* big-endian words: a dword's two are 256 * (bytes 0 + 2) + (bytes 1 + 3) */
	uint32_t sum = (((d[0] >> 16) & 0xffu) << 8) | (d[0] >> 24);          /* eth+14 */
#pragma unroll
	for (int j = 1; j < 5; j++)
		sum += (dot_even(d[j], 0u) << 8) + dot_odd(d[j], 0u);          /* eth+16..31 */
	sum += ((d[5] & 0xffu) << 8) | ((d[5] >> 8) & 0xffu);                 /* eth+32 */
	if (!verify)                                                          /* the check, eth+24 */
		sum -= ((d[3] & 0xffu) << 8) | ((d[3] >> 8) & 0xffu);
	sum = (sum & 0xffffu) + (sum >> 16);
	sum = (sum & 0xffffu) + (sum >> 16);
	return (uint16_t)bswap16(~sum & 0xffffu);
}

template <int FPT>
__global__ void __launch_bounds__(256) iphdr_kernel(CsumArgs a)
{
	const bool verify = (a.flags & XCSUM_F_VERIFY) != 0;
	const bool inplace = (a.flags & XCSUM_F_INPLACE) != 0 && !verify;
	const uint8_t *zero = (const uint8_t *)g_zero_chunk;
	const uint32_t q0 = blockIdx.x * (256u * FPT) + threadIdx.x;
	uint32_t p[FPT];
	u32x4 dsc[FPT];
#pragma unroll
	for (int j = 0; j < FPT; j++) {
		const uint32_t q = q0 + 256u * j;
		p[j] = q < a.ord.nlog ? frame_of(a.ord, q) : a.n;
	}
	/* the descriptor loads back to back, then the header loads */
	__builtin_amdgcn_sched_barrier(0);
#pragma unroll
	for (int j = 0; j < FPT; j++)
		dsc[j] = *((gu32x4 *)(a.desc + (p[j] < a.n ? p[j] : a.n - 1)));
	__builtin_amdgcn_sched_barrier(0);
	HdrFrame f[FPT];
#pragma unroll
	for (int j = 0; j < FPT; j++) {
		const uint64_t addr = (((uint64_t)dsc[j].y << 32) | dsc[j].x) - a.bias;
		f[j].eth = a.umem + addr;
		f[j].len = dsc[j].z;
		/* at least eth + IPv4 + UDP headers (the UDP-length rule of
		 * resolve() is applied per family below) */
		f[j].load = p[j] < a.n && f[j].len >= 42u;
		const uint8_t *h = f[j].load ? f[j].eth + 12 : zero;
		f[j].sh = (uint32_t)(uintptr_t)h & 3u;
		f[j].w = (const uint8_t *)((uintptr_t)h & ~(uintptr_t)3);
		if (f[j].load && !XB_IN(f[j].w, 28, f[j].eth, f[j].eth + f[j].len, XB_CSUM_HDR, 12))
			f[j].w = zero;
	}
	/* every frame's seven dwords in flight before the first is used; plain
	 * (temporal) loads: the iph->check store goes to the line they bring in */
	uint32_t w[FPT][7];
#pragma unroll
	for (int j = 0; j < FPT; j++)
#pragma unroll
		for (int k = 0; k < 7; k++)
			w[j][k] = ld_g<uint32_t>(f[j].w + 4 * k);
#pragma unroll
	for (int j = 0; j < FPT; j++) {
		if (p[j] >= a.n)
			continue;
		uint32_t proto = 0;
		uint16_t r = hdr_csum(w[j], f[j].sh, verify, &proto);
		/* 0 IPv4, 1 IPv6 (AUTO: untouched), -1 malformed; resolve()'s
		 * rules: the UDP length (len - 34 / len - 54) fits 16 bits */
		int kind = f[j].load && f[j].len - 34u <= 65535u ? 0 : -1;
		if (f[j].load && a.mode == XCSUM_MODE_AUTO && proto != 0x0800u)
			kind = proto == 0x86DDu && f[j].len >= 62u && f[j].len - 54u <= 65535u ? 1 : -1;
		if (kind != 0) {
			r = kind < 0 && verify ? (uint16_t)0xffffu : (uint16_t)0;
			if (kind < 0)
				atomicAdd(a.err, 1ull);
		} else if (inplace && XB_STORE(f[j].eth + 24, 2, f[j].eth, f[j].eth + f[j].len,
					      XB_CSUM_INPLACE, p[j])) {
			store_u16(f[j].eth + 24, r);
		}
		if (a.out && XB_IDX(p[j], a.n, XB_CSUM_OUT))
			st_res(a.out + p[j], r);
	}
}

template <int FPT>
static hipError_t launch_iphdr_t(const CsumArgs &a, hipStream_t s)
{
	const uint64_t per = 256u * FPT;
	const uint64_t blocks = ((uint64_t)a.ord.nlog + per - 1) / per;
	(void)hipGetLastError();
	hipLaunchKernelGGL(iphdr_kernel<FPT>, dim3((unsigned)(blocks ? blocks : 1)), dim3(256), 0, s,
			   a);
	return hipGetLastError();
}

/* fpt: frames per thread, the context's Tuning::iphdr_fpt (default 4) */
hipError_t launch_iphdr(const CsumArgs &a, int fpt, hipStream_t s)
{
	if (a.n == 0)
		return hipSuccess;
	switch (fpt) {
	case 1: return launch_iphdr_t<1>(a, s);
	case 2: return launch_iphdr_t<2>(a, s);
	case 8: return launch_iphdr_t<8>(a, s);
	default: return launch_iphdr_t<4>(a, s);
	}
}

} /* namespace xcsum */
