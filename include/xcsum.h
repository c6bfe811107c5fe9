/*
 * xcsum.h -- C ABI of the MI355X-native UDP checksum engine (libxcsum.so).
 *
 * Drop-in boundary for libxudp's per-packet UDP checksum path
 * (cclinuxer/libxudp xudp/checksum.h, driven from xudp/packet.c and
 * xudp/tx.c).  Plain pointers and sizes only; every call returns 0 or a
 * negative XCSUM_ERR_* code (the reference's convention of negative
 * XUDP_ERR_* codes, include/xudp.h:67-140), never aborts.
 *
 * Each entry point names the reference interface it replaces.  The
 * packet_info-level mirror (xudp_packet_udp & co.) is in xudp_packet.h.
 *
 * Threading: one xcsum_ctx per host thread (or per stream); the library keeps
 * no global mutable state besides the lazily created default context used by
 * the void-returning packet.c mirrors.  HIP is initialised lazily by
 * xcsum_ctx_create(), so a process may fork (libxudp's master/worker model,
 * test/case/lib.c:169) before its first call.
 */
#ifndef XCSUM_H
#define XCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XCSUM_ABI_VERSION 1

/* Layout-identical to struct xdp_desc (linux/if_xdp.h), the descriptor xudp
 * publishes on the AF_XDP TX ring (xudp/tx.c:450-452, include/queue.h:183-184).
 * addr = offset of the Ethernet frame inside the UMEM buffer, len = frame
 * length (xudp_packet_udp sets it to payload+42 / payload+62, packet.c:168/190). */
struct xcsum_desc {
	uint64_t addr;
	uint32_t len;
	uint32_t options;
};

/* What out[i] is.  In every mode out[i] is the 16-bit value to store into
 * udp->check (i.e. already in wire byte order). */
enum xcsum_mode {
	/* IPv4, xudp/checksum.h:107-140 udp_checksum() bit for bit, including
	 * its single-fold quirk (checksum.h:100-104); no 0 -> 0xffff mapping. */
	XCSUM_MODE_V4_LEGACY = 0,
	/* IPv4, RFC 768/1071 (full fold, 0 -> 0xffff). */
	XCSUM_MODE_V4_RFC = 1,
	/* IPv6, xudp/packet.c:105-117 udp_csum6() bit for bit. */
	XCSUM_MODE_V6 = 2,
	/* Per frame from eth->h_proto: 0x0800 -> V4_LEGACY (or V4_RFC with
	 * XCSUM_F_V4_RFC), 0x86DD -> V6, anything else -> out 0 + error. */
	XCSUM_MODE_AUTO = 3,
};

/* Flags (bitwise OR). */
#define XCSUM_F_INPLACE  0x1u /* also store out[i] into udp->check in the frame */
#define XCSUM_F_IPHDR    0x2u /* IPv4 frames: also compute and store iph->check
				 (== xudp_checksum_half, packet.c:43-66) */
#define XCSUM_F_V4_RFC   0x4u /* AUTO mode: IPv4 frames use V4_RFC */
#define XCSUM_F_ZEROCOPY 0x8u /* host batches: kernel reads the registered UMEM
				 through its device mapping instead of copying */
#define XCSUM_F_VERIFY   0x10u /* receive side (group/channel.c:231-255 parses but
				 never verifies): check the checksum already in each
				 frame, RFC 768/2460 rules in every mode: out[i] = 0
				 if it verifies (IPv4 check 0 = "no checksum" = valid;
				 IPv6 check 0 = invalid), nonzero otherwise (malformed
				 frames: 0xffff).  With XCSUM_F_IPHDR the IPv4 header
				 must verify too for out[i] to be 0.  Never writes. */
#define XCSUM_F_IPHDR_ONLY 0x80u /* xcsum_batch_device / _host: libxudp's IPv4 TX
				 checksum work and nothing else -- iph->check
				 (xudp_checksum_half, packet.c:43-66) computed from
				 the 20-byte header, udp->check left as it is (0,
				 packet.c:125), no payload byte read.  out[i] (if
				 d_out) = iph->check in wire order; with
				 XCSUM_F_INPLACE it is stored at eth+24; with
				 XCSUM_F_VERIFY out[i] = 0 iff the header verifies.
				 Modes V4_LEGACY / V4_RFC (the same here) and AUTO,
				 where IPv6 frames are left untouched with out[i] 0
				 (their checksum is udp_csum6: send them with
				 XCSUM_MODE_V6).  A frame is malformed under the
				 rule of the other modes (shorter than 42 bytes, UDP
				 length > 65535; AUTO: another h_proto): out[i] 0
				 (0xffff under VERIFY), counted.  XCSUM_MODE_V6:
				 -XCSUM_ERR_INVAL.  On host frames only the first 42
				 bytes of each cross PCIe (gathered, or read in place
				 from a mapped UMEM), and a context's resident
				 workgroups do not take such batches (launched). */

/* Error codes (returned negated). */
enum {
	XCSUM_ERR_INVAL = 9000,  /* bad argument */
	XCSUM_ERR_HIP,           /* a HIP runtime call failed */
	XCSUM_ERR_NODEV,         /* no such device / no GPU */
	XCSUM_ERR_NOMEM,         /* device or pinned allocation failed */
	XCSUM_ERR_NOT_REGISTERED,/* zero-copy asked for an unregistered UMEM */
	XCSUM_ERR_FRAME,         /* >=1 frame was malformed (too short, jumbo > 65535
				    UDP bytes, unknown h_proto): its out[i] is 0 */
};

/* Frame layout facts the kernel relies on (those of every frame xudp builds,
 * packet.c:19-21, :99): IPv4 has ihl == 5, IPv6 has nexthdr == UDP (no
 * extension headers); udp_len = len - 34 (IPv4) / len - 54 (IPv6); the check
 * field is 0 on entry (udp_build, packet.c:125) -- a nonzero field is summed
 * like any other byte, which is exactly a receive-side verify. */

typedef struct xcsum_ctx xcsum_ctx;

/* ---- device placement: libxudp's groups over the node's GPUs --------------
 * libxudp runs group_num groups (include/xudp.h:196-199, xudp_group_get(x,
 * gid) at :310-311), each a worker thread or a forked process
 * (test/case/lib.c:196-221), and checksums are per frame, so a group's
 * batches can go to any GPU with no exchange between GPUs.  The `device`
 * argument of xcsum_ctx_create picks one:
 *   >= 0                that device;
 *   XCSUM_DEVICE_ENV    $XCSUM_DEVICE (read when the context is created), else
 *                       device 0 -- the behaviour of rounds 1-5;
 *   XCSUM_DEVICE_AUTO   round robin over the visible devices, in the order
 *                       this process creates AUTO contexts (8 group threads
 *                       creating one context each land on 8 GPUs);
 *   XCSUM_DEVICE_GROUP(gid)  device gid mod the visible count: the same group
 *                       on the same GPU whatever the thread timing, and the
 *                       placement for forked workers (each process's AUTO
 *                       counter starts at 0).
 * The thread's default context (xudp_packet_udp_batch with ctx NULL and the
 * libxcsum_packet.so mirrors) is placed by xcsum_thread_init(gid), or, when
 * the thread never called it, by $XCSUM_DEVICE if set, else AUTO. */
#define XCSUM_DEVICE_ENV   (-1)
#define XCSUM_DEVICE_AUTO  (-2)
#define XCSUM_DEVICE_GROUP(gid) (-1000 - (int)(gid))   /* gid 0 .. 1000000 */
/* Devices this process sees (>= 1), or -XCSUM_ERR_NODEV. */
int xcsum_device_count(void);
/* The device xcsum_ctx_create(device, ...) takes when `ndev` devices are
 * visible (ndev <= 0: count them).  An AUTO answer takes a turn of the round
 * robin.  -XCSUM_ERR_NODEV for a device >= ndev or no device,
 * -XCSUM_ERR_INVAL for an unknown negative value. */
int xcsum_device_resolve(int device, int ndev);

/* Create a context bound to HIP device `device` (see above; -1 =
 * XCSUM_DEVICE_ENV: $XCSUM_DEVICE or 0). */
int xcsum_ctx_create(int device, xcsum_ctx **out);
/* xcsum_ctx_create(XCSUM_DEVICE_GROUP(gid), out): libxudp group gid's
 * context, on device gid mod the visible count. */
int xcsum_ctx_create_for_group(int gid, xcsum_ctx **out);
/* Create the calling thread's default context now, on group gid's device
 * (gid < 0: the default placement above), replacing one made earlier on
 * another device.  A libxudp worker calls it once when it starts (after any
 * fork): a missing or unusable device is then an error code at start-up
 * rather than a failure of the first xudp_packet_udp() call on the send
 * path, which cannot return one (libxcsum_packet.so aborts there).  Returns
 * 0 or -XCSUM_ERR_*. */
int xcsum_thread_init(int gid);
/* The calling thread's default context (created on first use; NULL if it
 * cannot be created). */
xcsum_ctx *xcsum_thread_ctx(void);
void xcsum_ctx_destroy(xcsum_ctx *ctx);
int xcsum_ctx_device(const xcsum_ctx *ctx);
/* Number of malformed frames seen by this context since the last call
 * (device-side counter; synchronises the context's device). */
int xcsum_ctx_take_errors(xcsum_ctx *ctx, uint64_t *count);

/* Force the kernel geometry used by this context's launches (tuning and
 * tests): G lanes per frame (8/16/32/64), U frames in flight per segment,
 * K chunks preloaded per lane.  G = 0 restores the automatic choice (from
 * len_hint).  Results never depend on the geometry.  -XCSUM_ERR_INVAL if the
 * combination is not compiled in. */
int xcsum_ctx_set_geometry(xcsum_ctx *ctx, int G, int U, int K);
/* Cap the persistent grid at `blocks_per_cu` 256-thread blocks per CU
 * (tuning; 0 = the per-geometry default, the occupancy limit at most). */
int xcsum_ctx_set_launch(xcsum_ctx *ctx, int blocks_per_cu);

/* Order in which xcsum_batch_device visits the frames (tuning knob; results
 * never depend on it).  The batch is cut into 2^tile_log2-frame tiles dealt
 * round-robin from 2^region_log2 equal regions, so the frames in flight come
 * from regions spread over the whole UMEM rather than one window.
 * region_log2 = 0: descriptor order; -1: automatic (default: per geometry
 * for dense batches, descriptor order with XCSUM_F_VERIFY at MTU; for
 * batches sparse in the UMEM 32 regions of 16-frame tiles, in place at MTU
 * 16 of 32 with XCSUM_F_IPHDR, else 8 of 16).  Env
 * XCSUM_ORDER="R,T" sets it at context creation. */
int xcsum_ctx_set_order(xcsum_ctx *ctx, int region_log2, int tile_log2);
/* Pick the visiting order for this context by timing it on the caller's own
 * batch (the arguments of xcsum_batch_device; it runs ordinary calls of it on
 * `stream` -- ~60 ms to bring the clocks up, then three rounds of the
 * automatic order and six forced ones, each order ~6-7 ms per round: ~0.2 s
 * in all -- and waits for them); a forced order is kept only if >= 1 %
 * faster than the automatic one in every round, else the order is left
 * automatic.  *region_log2 / *tile_log2 (may be NULL) receive the choice
 * (-1: automatic).  The calls write what any call writes (results, in-place
 * fields), but their malformed frames are counted apart: the count
 * xcsum_ctx_take_errors returns is unchanged by a calibration.  For a
 * caller that sends batches of one layout (libxudp's TX UMEM): once, after
 * the UMEM is set up.  Not while the stream is being captured
 * (-XCSUM_ERR_INVAL). */
int xcsum_ctx_calibrate_order(xcsum_ctx *ctx, uint8_t *d_umem, const struct xcsum_desc *d_desc,
			      uint32_t n, uint16_t *d_out, uint32_t mode, uint32_t flags,
			      uint32_t len_hint, void *stream, int *region_log2, int *tile_log2);

/* How xcsum_batch_device writes the check fields with XCSUM_F_INPLACE
 * (results and frame bytes are identical either way):
 *   FUSED: each field is stored by the pass that sums its frame;
 *   TWO_PASS: the checksum pass writes a result array (d_out, or a scratch
 *     array of the context), then a second launch stores the fields in frame
 *     order -- the stores no longer interleave with the read stream
 *     (DESIGN.md 5.3).  Its scratch (a result array of the context, used
 *     when d_out is NULL or with XCSUM_F_IPHDR) is allocated on the first
 *     such call and grown by later ones; eager calls of one context on
 *     different streams are ordered through an event.  A graph never
 *     references that scratch: a call made while its stream is captured and
 *     that would need it runs FUSED (the same bytes), so replays of a graph
 *     stay valid whatever eager calls do to the scratch.
 *   AUTO (default): FUSED.  Measured on config 2, the
 *     second pass costs more than the interleaving it removes: the lines it
 *     writes have left the caches by then and come back from HBM.
 * Env XCSUM_INPLACE=fused|two_pass sets it at context creation. */
#define XCSUM_INPLACE_AUTO     0
#define XCSUM_INPLACE_FUSED    1
#define XCSUM_INPLACE_TWO_PASS 2
int xcsum_ctx_set_inplace(xcsum_ctx *ctx, int schedule);

/* Tuning knobs of one context (sweeps, A/B and the parity tests that run
 * every kernel variant): which kernel or geometry a launch takes, never its
 * results.  The library reads no tuning from the environment on any batch
 * path; these setters are the only way in (the `make variant` A/B build also
 * takes them from XCSUM_<KNOB> at context creation).  Values (a, b, c, d):
 *   IPHDR_FPT        a = frames per thread of the IPv4 header kernel, 1|2|4|8
 *                    (default 4);
 *   BUILD_HDR        a = 0: IPv4 in-place builds take the payload-summing
 *                    build kernel (superseded in round 5; A/B and tests),
 *                    1: the header kernel (default);
 *   BUILD_GEOMETRY   a, b = G, K of the build kernel (a = 0: automatic);
 *   RX_GEOMETRY      a, b, c, d = G, K, U, blocks per CU of the receive
 *                    kernel (a = 0: automatic);
 *   RX_ORDER         a = -1 automatic (sparse batches: 32 regions of 64-frame
 *                    tiles), 0 descriptor order, else 2^a regions of 2^b
 *                    frames;
 *   GATHER_RATIO     a = host path: frames spread over more than a x their
 *                    bytes are gathered frame by frame (default 2);
 *   INPLACE_BLOCK    a = 0|32|64: store width of the two-pass scatter;
 *   INPLACE_TL       a = 0: in place without IPHDR at MTU takes the plain
 *                    kernel instead of the temporal-first-chunks one;
 *   RESIDENT_INLINE  a = 0: resident requests carry their descriptors only
 *                    in the array (A/B of the inline lines);
 *   RESIDENT_LIMIT_CUT a = bytes: resident requests carry a limit this much
 *                    short (test hook for the workgroups' descriptor check);
 *   CLAIM            a = the share of a batch's frames the checksum kernel
 *                    schedules statically, in 64ths (64: all, the default),
 *                    b = frames per claim in steps of a wave (0: 16): the
 *                    rest is claimed from a device counter by the waves that
 *                    are ahead (the claimed tail, geometries (64,1,9),
 *                    (64,1,2), (16,2,6); A/B build only -- -XCSUM_ERR_INVAL
 *                    from libxcsum.so for a < 64).
 * -XCSUM_ERR_INVAL for an unknown knob or a value not compiled in. */
enum xcsum_tuning {
	XCSUM_TUNE_IPHDR_FPT = 1,
	XCSUM_TUNE_BUILD_HDR = 2,
	XCSUM_TUNE_BUILD_GEOMETRY = 3,
	XCSUM_TUNE_RX_GEOMETRY = 4,
	XCSUM_TUNE_RX_ORDER = 5,
	XCSUM_TUNE_GATHER_RATIO = 6,
	XCSUM_TUNE_INPLACE_BLOCK = 7,
	XCSUM_TUNE_INPLACE_TL = 8,
	XCSUM_TUNE_RESIDENT_INLINE = 9,
	XCSUM_TUNE_RESIDENT_LIMIT_CUT = 10,
	XCSUM_TUNE_CLAIM = 11,
};
int xcsum_ctx_set_tuning(xcsum_ctx *ctx, int knob, int a, int b, int c, int d);

/* ---- device-resident batch ------------------------------------------------
 * Replaces the per-frame checksum work of the xudp_frame_send loop
 * (xudp/tx.c:696-726 -> __xudp_frame_send -> xudp_packet_udp, packet.c:156)
 * for a whole batch: one launch, asynchronous on `stream` (a hipStream_t;
 * NULL = the default stream).  d_umem, d_desc and d_out are device pointers
 * (d_out may be NULL with XCSUM_F_INPLACE).  len_hint = typical frame length
 * in bytes (0 = unknown); it only picks the kernel geometry, never results. */
int xcsum_batch_device(xcsum_ctx *ctx, uint8_t *d_umem, const struct xcsum_desc *d_desc,
		       uint32_t n, uint16_t *d_out, uint32_t mode, uint32_t flags,
		       uint32_t len_hint, void *stream);

/* ---- device-side frame build: xudp_frame_send on the GPU -------------------
 * Replaces the whole per-frame loop of xudp_frame_send (tx.c:696-726): for
 * every message, build eth + IPv4/IPv6 + UDP headers in front of the payload
 * in its UMEM frame slot exactly as xudp_packet_udp() does (packet.c:156-194),
 * copying the payload there first when it lives elsewhere (the memcpy of
 * xudp_packet_udp_payload, packet.c:196-203, fused with the checksum pass),
 * compute iph->check (packet.c:43-66) / udp->check (IPv6: packet.c:105-117;
 * IPv4: 0 as packet.c:125, or RFC with XCSUM_F_V4_RFC), and write the
 * xdp_desc each frame is published with (tx.c:450-452).
 * One route per batch, like xudp_tx_info_prepare() (tx.c:690). */
struct xcsum_route {
	uint8_t family;         /* 4 or 6 */
	uint8_t pad[3];
	uint8_t dmac[6];
	uint8_t smac[6];
	uint16_t sport_be;      /* network byte order, as sin_port */
	uint16_t dport_be;
	uint8_t saddr[16];      /* IPv4: first 4 bytes */
	uint8_t daddr[16];
};

struct xcsum_msg {
	uint64_t src;           /* payload offset from d_src (ignored in place) */
	uint32_t len;           /* payload bytes */
	uint32_t slot;          /* UMEM frame slot: data = d_umem + slot*frame_size + data_off */
};

#define XCSUM_F_BUILD_INPLACE 0x20u /* payloads already sit at their frame's data
				       offset (the zero-copy xudp_frame_alloc path,
				       tx.c:760): no copy, d_src unused */
#define XCSUM_F_SRC_ALIGNED   0x40u /* the caller guarantees every payload source
				       (d_src + src) is 16-byte aligned: cheaper
				       copy kernel; results are undefined if not */

/* d_desc_out[i] = {slot*frame_size + data_off - (42|62), payload + 42|62, 0};
 * d_out (may be NULL) = the udp->check written.  frame_size and data_off must
 * be multiples of 16 (xudp: 4096 and 384), d_umem 16-aligned.
 * Messages that do not fit their slot or exceed 65527 payload bytes get
 * desc len 0, no frame, and count as malformed.  len_hint = typical payload
 * bytes (kernel geometry only).  Asynchronous on `stream`. */
int xcsum_build_device(xcsum_ctx *ctx, const struct xcsum_route *route,
		       const uint8_t *d_src, const struct xcsum_msg *d_msgs, uint32_t n,
		       uint8_t *d_umem, uint32_t frame_size, uint32_t data_off,
		       struct xcsum_desc *d_desc_out, uint16_t *d_out, uint32_t flags,
		       uint32_t len_hint, void *stream);

/* ---- receive path: xudp_nic_recv_channel's per-frame work on the GPU ------
 * Replaces the loop of xudp_nic_recv_channel (group/channel.c:211-267) for a
 * batch of received frames (the xdp_desc array dequeued from the RX ring):
 * packet_parse() (include/packet_parse.h:101-165, with its quirks: h_proto
 * first byte 0x08 OR second byte 0x00 parses as IPv4; IPv6 UDP is taken at
 * iph6 + 1 even after extension headers), the stats-request test
 * (channel.c:182-190) and the fields of xudp_fill_msg() (channel.c:69-128),
 * one record per descriptor.  With XCSUM_F_VERIFY the UDP checksum is also
 * verified under RFC 768/2460 with the length from the UDP header (received
 * frames may carry Ethernet padding); with XCSUM_F_IPHDR also the IPv4 header
 * checksum over 4*ihl bytes.  The reference verifies nothing. */
enum xcsum_rx_status {
	XCSUM_RX_OK = 0,        /* deliver (xudp_fill_msg) */
	XCSUM_RX_PARSE = 1,     /* packet_parse() returned 0: not UDP over IPv4/IPv6,
				   or truncated (the reference does not skip these,
				   channel.c:241 tests ret < 0; it is never true) */
	XCSUM_RX_STATS = 2,     /* iph->saddr == iph->daddr: a stats request the host
				   answers (channel.c:189); recycle the frame */
	XCSUM_RX_CSUM = 3,      /* XCSUM_F_VERIFY: checksum invalid, or the UDP length
				   does not fit the frame */
};

struct xcsum_rx_msg {
	uint64_t frame;         /* desc.addr (m->recycle1 / m->frame, channel.c:113-123) */
	uint64_t body;          /* UMEM offset of the UDP payload, udp + 1 (m->p) */
	uint32_t size;          /* ntohs(udp->len) - 8 (m->size; wraps below 8 as the
				   reference's int does) */
	uint8_t status;         /* enum xcsum_rx_status */
	uint8_t family;         /* 4 or 6; 0 when the parse failed */
	uint16_t l4_off;        /* UDP header offset in the frame */
	uint16_t sport_be;      /* peer port, udp->source (network order) */
	uint16_t dport_be;      /* local port, udp->dest */
	uint32_t reserved;
	uint8_t saddr[16];      /* peer address (IPv4: first 4 bytes) */
	uint8_t daddr[16];      /* local address */
};

/* d_msgs[i] describes d_desc[i] (64 bytes each; fields past `status` are 0
 * when the parse failed).  d_count (may be NULL) receives the number of
 * XCSUM_RX_OK records (uint32, device memory).  flags: XCSUM_F_VERIFY,
 * XCSUM_F_IPHDR.  len_hint = typical frame length (kernel geometry only).
 * d_umem must be 4-byte aligned (-XCSUM_ERR_INVAL otherwise); frames may sit
 * at any byte offset in it.  Asynchronous on `stream`; with d_count the
 * launches use per-context scratch, so keep one context's receive batches on
 * one stream (one context per stream, as everywhere in this ABI). */
int xcsum_rx_device(xcsum_ctx *ctx, const uint8_t *d_umem, const struct xcsum_desc *d_desc,
		    uint32_t n, struct xcsum_rx_msg *d_msgs, uint32_t *d_count, uint32_t flags,
		    uint32_t len_hint, void *stream);

/* Same for received frames in the host UMEM (the AF_XDP RX ring's frames):
 * frames are staged to the device with chunked, double-buffered
 * hipMemcpyAsync, or with XCSUM_F_ZEROCOPY read in place over PCIe from a
 * registered UMEM; the 64-byte records come back into h_msgs.  A sparse
 * batch (one frame per UMEM chunk, as the RX ring hands them over) is read
 * in place from a registered UMEM, and its small frames are gathered frame
 * by frame from a pageable one, instead of copying the range with its gaps.
 * Records hold UMEM offsets either way.  *h_count (may be NULL)
 * = number of XCSUM_RX_OK records.  flags: XCSUM_F_VERIFY, XCSUM_F_IPHDR,
 * XCSUM_F_ZEROCOPY.  Synchronous. */
int xcsum_rx_host(xcsum_ctx *ctx, const uint8_t *h_umem, const struct xcsum_desc *h_desc,
		  uint32_t n, struct xcsum_rx_msg *h_msgs, uint32_t *h_count, uint32_t flags);

/* ---- host-resident batch (frames in the AF_XDP UMEM) ----------------------
 * Same semantics with host pointers.  Synchronous.  Frames are moved with
 * chunked, double-buffered hipMemcpyAsync -> kernel -> the 2-byte results
 * back: DMA'd in place from a registered UMEM, copied into the context's
 * pinned stages first from pageable memory (never handed to the runtime's
 * own pinning: DESIGN.md 6); with XCSUM_F_INPLACE the
 * results are also written into the host frames' udp->check (and iph->check
 * with XCSUM_F_IPHDR).  With XCSUM_F_ZEROCOPY and a registered UMEM the
 * kernel reads the frames in place over PCIe instead.  Frames spread over
 * the UMEM (one per 4096-byte chunk, as xudp lays them out) are read in
 * place from a registered UMEM even without XCSUM_F_ZEROCOPY, and small ones
 * are gathered frame by frame from a pageable UMEM; the results do not
 * depend on the transport. */
int xcsum_batch_host(xcsum_ctx *ctx, uint8_t *h_umem, const struct xcsum_desc *h_desc,
		     uint32_t n, uint16_t *h_out, uint32_t mode, uint32_t flags);

/* Page-lock and map a host region (xudp's UMEM, xudp/xsk.c:222-341) for DMA
 * and zero-copy access.  Ownership stays with the caller.  Unregistering
 * waits for this context's work first (its host-path streams, its resident
 * workgroups, the streams its device entry points ran on), so the caller may
 * unmap the region as soon as it returns.
 *
 * Only memory whose pages stay put is mapped for the GPU: a region that is
 * eligible for transparent huge pages (a VMA flagged MADV_HUGEPAGE -- numpy
 * does that to arrays of 4 MiB and up -- or THP "always" without
 * MADV_NOHUGEPAGE) is registered for bookkeeping only and its batches are
 * staged through the context's pinned buffers (same results; DESIGN.md 6:
 * every registered-memory GPU fault of rounds 2-4 was on such memory).
 * libxudp's UMEM (anon_map: MAP_SHARED | MAP_ANONYMOUS | MAP_POPULATE |
 * MAP_LOCKED, include/common.h:37-41) is mapped.  xcsum_umem_mapped() says
 * which: 1 mapped, 0 staged, -XCSUM_ERR_NOT_REGISTERED if base is unknown.
 *
 * Contract: eligibility is read ONCE, at registration (the VMA flags in
 * /proc/self/smaps and the THP sysfs modes; the parser is
 * libxudp_amd/csrc/xcsum_thp.h).  Until the range is unregistered the caller
 * must not make it THP-eligible -- madvise(MADV_HUGEPAGE) on it,
 * prctl(PR_SET_THP_DISABLE, 0) after registering with THP disabled, or a
 * change of the THP modes -- nor mremap(), munmap() or remap it: the GPU
 * keeps its mapping of the pages found at registration.  To change any of
 * that, unregister, change it, register again. */
int xcsum_register_umem(xcsum_ctx *ctx, void *base, size_t size);
int xcsum_unregister_umem(xcsum_ctx *ctx, void *base);
int xcsum_umem_mapped(xcsum_ctx *ctx, const void *base);

/* Resident workgroups for small host batches (libxudp sends in batches of
 * tx_batch_num = 100 frames, xudp/xudp.c:74; tx.c:673-734 is one batch).
 * `workgroups` (1-64; 16 is a good start) checksum workgroups stay on the
 * device and poll a doorbell in pinned host memory: a host batch of at most
 * 4096 frames and 256 KiB of frame bytes is gathered into the context's
 * pinned stage and then costs a doorbell store and a spin on the answer
 * instead of a kernel launch and its completion (TX loop: 1 frame 9-11 us
 * instead of 17-24 us, 100 MTU frames 18-21 us instead of ~25 us).
 * Results are the same bytes.  The workgroups leave after `idle_us` (0:
 * 20000) without a batch and come back with the next one.  0 workgroups: off
 * (the default; env XCSUM_RESIDENT="W[,idle_us[,max_frames]]" sets it at
 * context creation, e.g. for the packet.c mirrors' default contexts).  While they are resident, a device-wide
 * synchronisation by others (hipDeviceSynchronize, torch.cuda.synchronize)
 * waits until they leave, i.e. up to idle_us after this context's last
 * batch; the library's own device-wide waits (xcsum_ctx_take_errors,
 * xcsum_unregister_umem, xcsum_ctx_destroy) stop them first.
 *
 * Cost to other GPU work: a live resident grid holds its hardware queue, and
 * streams beyond GPU_MAX_HW_QUEUES (4) share queues, so a kernel of another
 * stream on the same GPU may wait behind it.  Every workgroup therefore
 * leaves after `life_us` alive even while busy (default 2000; the next batch
 * relaunches them, ~10 us once per life): that wait is at most life_us plus
 * one batch -- measured 1.9 ms at the default, 200 ms at life_us = 200000
 * (tests/test_gpu_resident.py::test_resident_queue_sharing). */
int xcsum_ctx_set_resident(xcsum_ctx *ctx, int workgroups, uint32_t idle_us);
/* The resident workgroups' life bound in microseconds (0: the default 2000);
 * running workgroups leave and the next batch launches them with it. */
int xcsum_ctx_set_resident_life(xcsum_ctx *ctx, uint32_t life_us);

/* Number of the context's host-path slots with copies or kernels still in
 * flight.  Always 0 after xcsum_batch_host / xcsum_rx_host return, on error
 * returns too: no work of a finished call touches the caller's memory. */
int xcsum_ctx_pending(xcsum_ctx *ctx);

/* Diagnostics (no reference counterpart): the hipError_t of the last HIP call
 * that made an entry point of this thread return -XCSUM_ERR_HIP (0: none),
 * with the library source line and the error's name. */
int xcsum_last_hip_error(int *line, const char **name);

/* Wait for all work the context issued on `stream`. */
int xcsum_sync(xcsum_ctx *ctx, void *stream);

/* ---- synthetic frames (bench + tests; same bytes on host and device) ------
 * Frames exactly as xudp_packet_udp() lays them out (packet.c:156-194) with
 * both check fields 0, random MACs/addresses/ports/payload from a SplitMix64
 * stream keyed by (seed, first_index + i).  family: 4 or 6.
 * gen_layout fills descriptors: payload size uniform in [pmin, pmax], frames
 * packed back to back at `align`-byte boundaries (stride == 0), or one frame
 * every `stride` bytes at offset `offset` (UMEM-mirror layout). */
int xcsum_gen_layout(uint32_t n, uint32_t family, uint32_t pmin, uint32_t pmax,
		     uint64_t seed, uint64_t first_index, uint32_t align,
		     uint32_t stride, uint32_t offset,
		     struct xcsum_desc *h_desc, uint64_t *umem_bytes);
int xcsum_gen_fill_host(uint8_t *h_umem, const struct xcsum_desc *h_desc, uint32_t n,
			uint32_t family, uint64_t seed, uint64_t first_index);
int xcsum_gen_fill_device(uint8_t *d_umem, const struct xcsum_desc *d_desc, uint32_t n,
			  uint32_t family, uint64_t seed, uint64_t first_index, void *stream);

/* Split [0, n) into `nshards` contiguous ranges of near-equal frame bytes
 * (multi-GPU sharding, one range per GPU); returns shard `idx`'s range. */
int xcsum_shard_by_bytes(const struct xcsum_desc *h_desc, uint32_t n, uint32_t nshards,
			 uint32_t idx, uint32_t *first, uint32_t *count);

#ifdef __cplusplus
}
#endif
#endif /* XCSUM_H */
