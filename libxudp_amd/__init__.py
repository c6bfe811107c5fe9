"""libxudp_amd -- MI355X-native UDP checksum engine for cclinuxer/libxudp.

The product is ``libxcsum.so`` (gfx950 HIP kernels + the C ABI declared in
``include/xcsum.h`` and ``include/xudp_packet.h``).  This module is a thin
ctypes binding used by the tests, ``bench.py`` and ``__graft_entry__``; C
callers (libxudp's tx.c) link the shared library directly, see INTEGRATION.md.

Importing never falls back to anything: if the library is missing the import
raises, and every compute call goes to the GPU kernel or returns an error.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# XCSUM_LIB selects an A/B build variant of the library (tuning only)
_PRODUCT_LIB = os.path.join(HERE, "libxcsum.so")
LIB_PATH = os.environ.get("XCSUM_LIB") or _PRODUCT_LIB
# the void packet.c mirrors (xudp_packet_udp, xudp_packet_udp_payload): the
# same symbols as libxudp's packet.o, so a library of their own, linked
# instead of packet.o (include/xudp_packet.h); it binds to
# whichever libxcsum.so (SONAME) the process loaded first
PACKET_LIB_PATH = os.path.join(HERE, "libxcsum_packet.so")

# include/xcsum.h
MODE_V4_LEGACY = 0
MODE_V4_RFC = 1
MODE_V6 = 2
MODE_AUTO = 3

F_INPLACE = 0x1
F_IPHDR = 0x2
F_V4_RFC = 0x4
F_ZEROCOPY = 0x8
F_VERIFY = 0x10
F_IPHDR_ONLY = 0x80   # libxudp's IPv4 TX call: iph->check alone (batch_device / batch_host)

ERR_INVAL = 9000
ERR_HIP = 9001
ERR_NODEV = 9002
ERR_NOMEM = 9003
ERR_NOT_REGISTERED = 9004
ERR_FRAME = 9005

ERR_NAMES = {ERR_INVAL: "XCSUM_ERR_INVAL", ERR_HIP: "XCSUM_ERR_HIP",
             ERR_NODEV: "XCSUM_ERR_NODEV", ERR_NOMEM: "XCSUM_ERR_NOMEM",
             ERR_NOT_REGISTERED: "XCSUM_ERR_NOT_REGISTERED",
             ERR_FRAME: "XCSUM_ERR_FRAME"}

# kernel geometries compiled into libxcsum.so (XCSUM_GEOMETRIES in
# csrc/xcsum_kernels.hip): (G lanes per frame, U frames per iteration, K chunks)
REG_GEOMETRIES = [(64, 1, 2), (64, 1, 9), (32, 1, 3), (32, 1, 6), (16, 1, 2), (16, 1, 3),
                  (16, 1, 6), (16, 2, 6), (16, 1, 12), (8, 1, 2), (8, 2, 1), (8, 1, 12),
                  (4, 2, 2), (4, 4, 2), (4, 1, 2), (2, 1, 4), (2, 2, 4), (1, 1, 6), (1, 1, 8),
                  (1, 2, 6)]
# stream kernel (csum_stream_kernel<KC>): a wave per 64 packed frames, the
# region they occupy streamed through a KC-KiB LDS stage: G = 64, U = 0, K = KC
STREAM_GEOMETRIES = [(64, 0, 4), (64, 0, 8), (64, 0, 16)]
# every geometry libxcsum.so runs (the parity tests sweep them all)
GEOMETRIES = REG_GEOMETRIES + STREAM_GEOMETRIES
# A/B kernels outside libxcsum.so (csrc/variants/, `make -C libxudp_amd variant
# NAME=ab`, loaded with XCSUM_LIB): LDS-DMA staged csum_lds_kernel<K, D>
# (G = 16, U = 10 + ring depth D) and the segmented stream (64, frames per
# unit, rows in flight)
LDS_GEOMETRIES = [(16, 12, 6), (16, 13, 6), (16, 12, 3), (16, 14, 3)]
SEG_GEOMETRIES = [(64, 64, 4), (64, 64, 8), (64, 16, 4)]
# round 6: the same with the finished spans added into LDS words (K = 100 + D)
SEG_ATOM_GEOMETRIES = [(g, f, 100 + d) for g, f, d in SEG_GEOMETRIES]


# bounds-checked debug build (make -C libxudp_amd debug; BoundsSite in
# csrc/xcsum_internal.h, in order from 1)
BOUNDS_SITES = ["csum_chunk", "csum_walk", "csum_hdr", "csum_out", "csum_inplace",
                "stream_region", "stream_stage", "build_src", "build_data", "build_out",
                "rx_chunk", "rx_rec", "rx_part", "rx_stream", "gen_store", "scatter", "csum_region", "res_req"]


def debug_build():
    """True when the loaded library is the bounds-checked debug build."""
    return hasattr(lib(), "xcsum_debug_bounds")


def take_bounds(max_recs=16):
    """(violations since the last call, [(site, index, addr, lo, hi), ...]);
    synchronises the device.  Debug build only."""
    L = lib()
    fn = L.xcsum_debug_bounds
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_int]
    count = ctypes.c_uint64(0)
    recs = np.zeros(4 * max_recs, dtype=np.uint64)
    _check(fn(ctypes.byref(count), recs.ctypes.data, max_recs), "xcsum_debug_bounds")
    out = []
    for k in range(min(int(count.value), max_recs)):
        sid, addr, lo, hi = (int(x) for x in recs[4 * k:4 * k + 4])
        site = sid >> 32
        name = BOUNDS_SITES[site - 1] if 1 <= site <= len(BOUNDS_SITES) else str(site)
        out.append((name, sid & 0xffffffff, addr, lo, hi))
    return int(count.value), out


def variants_built():
    """True when the loaded library is a variants build (A/B kernels in)."""
    return hasattr(lib(), "xcsum_variants_built")


def variant_geometries():
    """The A/B geometries the loaded library runs ([] for libxcsum.so)."""
    return LDS_GEOMETRIES + SEG_GEOMETRIES + SEG_ATOM_GEOMETRIES if variants_built() else []


# xcsum_ctx_set_inplace schedules
INPLACE_AUTO, INPLACE_FUSED, INPLACE_TWO_PASS = 0, 1, 2

# xcsum_ctx_set_tuning knobs (enum xcsum_tuning)
TUNE_IPHDR_FPT, TUNE_BUILD_HDR, TUNE_BUILD_GEOMETRY, TUNE_RX_GEOMETRY, TUNE_RX_ORDER = 1, 2, 3, 4, 5
TUNE_GATHER_RATIO, TUNE_INPLACE_BLOCK, TUNE_INPLACE_TL = 6, 7, 8
TUNE_RESIDENT_INLINE, TUNE_RESIDENT_LIMIT_CUT, TUNE_CLAIM = 9, 10, 11

# device placement (include/xcsum.h)
DEVICE_ENV, DEVICE_AUTO = -1, -2


def DEVICE_GROUP(gid):
    """xcsum_ctx_create device argument for libxudp group gid"""
    return -1000 - int(gid)


def device_resolve(device, ndev=0):
    """The device xcsum_ctx_create(device) takes with ndev visible devices
    (ndev <= 0: count them); negative = -XCSUM_ERR_*"""
    return lib().xcsum_device_resolve(int(device), int(ndev))

F_BUILD_INPLACE = 0x20
F_SRC_ALIGNED = 0x40

# struct xcsum_desc == struct xdp_desc
DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
# struct xcsum_msg (device frame build)
MSG_DTYPE = np.dtype([("src", "<u8"), ("len", "<u4"), ("slot", "<u4")])

# struct xcsum_rx_msg (64 bytes) and enum xcsum_rx_status
RX_MSG_DTYPE = np.dtype([("frame", "<u8"), ("body", "<u8"), ("size", "<u4"), ("status", "u1"),
                         ("family", "u1"), ("l4_off", "<u2"), ("sport_be", "<u2"),
                         ("dport_be", "<u2"), ("reserved", "<u4"), ("saddr", "u1", 16),
                         ("daddr", "u1", 16)])
RX_OK, RX_PARSE, RX_STATS, RX_CSUM = 0, 1, 2, 3

HDR4 = 42  # eth 14 + ip 20 + udp 8
HDR6 = 62  # eth 14 + ip6 40 + udp 8


class XcsumError(RuntimeError):
    def __init__(self, rc, what):
        self.rc = rc
        super().__init__(f"{what} failed: -{ERR_NAMES.get(-rc, rc)}")


_lib = None

_SIGS = {
    "xcsum_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "xcsum_ctx_destroy": (None, [ctypes.c_void_p]),
    "xcsum_ctx_device": (ctypes.c_int, [ctypes.c_void_p]),
    "xcsum_ctx_take_errors": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "xcsum_ctx_set_geometry": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int]),
    "xcsum_ctx_set_launch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "xcsum_ctx_set_order": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "xcsum_ctx_calibrate_order": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_void_p,
                                                 ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_int)]),
    "xcsum_ctx_set_resident": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]),
    "xcsum_ctx_set_inplace": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "xcsum_ctx_set_tuning": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "xcsum_ctx_set_resident_life": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "xcsum_device_count": (ctypes.c_int, []),
    "xcsum_device_resolve": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "xcsum_ctx_create_for_group": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "xcsum_thread_init": (ctypes.c_int, [ctypes.c_int]),
    "xcsum_thread_ctx": (ctypes.c_void_p, []),
    "xcsum_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    "xcsum_build_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p]),
    "xcsum_rx_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    "xcsum_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_uint32]),
    "xcsum_rx_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]),
    "xcsum_register_umem": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "xcsum_unregister_umem": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "xcsum_umem_mapped": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "xcsum_sync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "xcsum_ctx_pending": (ctypes.c_int, [ctypes.c_void_p]),
    "xcsum_last_hip_error": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_char_p)]),
    "xcsum_gen_layout": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "xcsum_gen_fill_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]),
    "xcsum_gen_fill_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_void_p]),
    "xcsum_shard_by_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_uint32)]),
    "xudp_packet_build_headers": (None, [ctypes.c_void_p]),
    "xudp_packet_udp_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint32]),
}


def lib():
    """Load libxcsum.so (raises ImportError if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C libxudp_amd` "
                "or `python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process: torch ships its own libamdhip64.so
        # (same SONAME as /opt/rocm's).  Loaded first, it also serves
        # libxcsum.so's DT_NEEDED; loaded after ours, it would be a second
        # runtime in the process and torch.cuda would see no device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name, None)
            if fn is None:
                # only an older A/B build (XCSUM_LIB) may lack a symbol: the
                # product library exports them all (tests/test_abi.py)
                if LIB_PATH == _PRODUCT_LIB:
                    raise ImportError(f"{LIB_PATH} does not export {name}")
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# libxcsum_packet.so
_PACKET_SIGS = {
    "xudp_packet_udp": (None, [ctypes.c_void_p]),
    "xudp_packet_udp_payload": (None, [ctypes.c_void_p]),
}
_packet_lib = None


def packet_lib():
    """Load libxcsum_packet.so (after libxcsum.so, which it needs)."""
    global _packet_lib
    if _packet_lib is None:
        lib()
        if not os.path.exists(PACKET_LIB_PATH):
            raise ImportError(f"{PACKET_LIB_PATH} is missing: build it with `make -C libxudp_amd`")
        L = ctypes.CDLL(PACKET_LIB_PATH)
        for name, (res, args) in _PACKET_SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _packet_lib = L
    return _packet_lib


def _check(rc, what):
    if rc != 0:
        if ERR_NAMES.get(-rc) == "XCSUM_ERR_HIP":
            line, name = ctypes.c_int(0), ctypes.c_char_p()
            code = lib().xcsum_last_hip_error(ctypes.byref(line), ctypes.byref(name))
            what = f"{what} ({(name.value or b'?').decode()} = {code} at xcsum_api.hip:{line.value})"
        raise XcsumError(rc, what)
    return rc


def _check_nonneg(rc, what):
    if rc < 0:
        _check(rc, what)
    return rc


def _ptr(a):
    """Raw address of a numpy array, torch tensor, int or None."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError(type(a))


# ---- synthetic frames (host side, no GPU needed) -------------------------

def gen_layout(n, family, pmin, pmax=None, seed=0, first_index=0, align=8, stride=0, offset=0):
    """Descriptors for n synthetic frames -> (desc ndarray, umem_bytes)."""
    if pmax is None:
        pmax = pmin
    desc = np.zeros(n, dtype=DESC_DTYPE)
    nbytes = ctypes.c_uint64(0)
    _check(lib().xcsum_gen_layout(n, family, pmin, pmax, seed, first_index, align, stride,
                                  offset, _ptr(desc), ctypes.byref(nbytes)), "xcsum_gen_layout")
    return desc, int(nbytes.value)


def umem_buffer(nbytes):
    """A host UMEM mapped the way libxudp maps one (anon_map: MAP_SHARED |
    MAP_ANONYMOUS, populated and locked, include/common.h:37-41), never backed
    by transparent huge pages (MADV_NOHUGEPAGE before the pages exist), as a
    zeroed uint8 ndarray.  xcsum_register_umem GPU-maps such memory (numpy's
    own heap arrays may be THP-eligible and are then staged).
    The mapping lives as long as the array; locking is best effort."""
    import mmap
    size = max(4096, (int(nbytes) + 4095) & ~4095)
    m = mmap.mmap(-1, size, flags=mmap.MAP_SHARED | mmap.MAP_ANONYMOUS)
    if hasattr(mmap, "MADV_NOHUGEPAGE"):
        m.madvise(mmap.MADV_NOHUGEPAGE)
    arr = np.frombuffer(m, dtype=np.uint8, count=int(nbytes))
    arr[:] = 0                                  # populate
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.mlock(ctypes.c_void_p(arr.ctypes.data), ctypes.c_size_t(size))
    except (OSError, AttributeError):
        pass
    return arr


def as_umem(arr):
    """A copy of `arr` (uint8) in a umem_buffer()."""
    u = umem_buffer(len(arr))
    u[:] = arr
    return u


def gen_fill_host(umem, desc, family, seed=0, first_index=0):
    _check(lib().xcsum_gen_fill_host(_ptr(umem), _ptr(desc), len(desc), family, seed,
                                     first_index), "xcsum_gen_fill_host")


def gen_frames_host(n, family, pmin, pmax=None, seed=0, first_index=0, align=8, stride=0,
                    offset=0, pad=64):
    """Convenience: (umem uint8 ndarray, desc) generated on the host."""
    desc, nbytes = gen_layout(n, family, pmin, pmax, seed, first_index, align, stride, offset)
    umem = np.zeros(nbytes + pad, dtype=np.uint8)
    gen_fill_host(umem, desc, family, seed, first_index)
    return umem, desc


def shard_by_bytes(desc, nshards, idx):
    first = ctypes.c_uint32(0)
    count = ctypes.c_uint32(0)
    _check(lib().xcsum_shard_by_bytes(_ptr(desc), len(desc), nshards, idx, ctypes.byref(first),
                                      ctypes.byref(count)), "xcsum_shard_by_bytes")
    return int(first.value), int(count.value)


def alg_bytes(desc, family):
    """Algorithmic bytes of a batch: span read + 2-byte write.
    span = udp_len + 8 (IPv4 addresses) or + 32 (IPv6)."""
    ln = desc["len"].astype(np.int64)
    if family == 6:
        span = ln - 54 + 32
    else:
        span = ln - 34 + 8
    return int(span.sum()) + 2 * len(desc)


# ---- device context --------------------------------------------------------

class Engine:
    """One xcsum_ctx (one device, one host thread)."""

    def __init__(self, device=-1):
        self._ctx = ctypes.c_void_p(0)
        _check(lib().xcsum_ctx_create(device, ctypes.byref(self._ctx)), "xcsum_ctx_create")
        self.device = lib().xcsum_ctx_device(self._ctx)

    @property
    def ctx(self):
        return self._ctx

    def close(self):
        if self._ctx:
            lib().xcsum_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_geometry(self, G=0, U=0, K=0):
        _check(lib().xcsum_ctx_set_geometry(self._ctx, G, U, K), "xcsum_ctx_set_geometry")

    def set_launch(self, blocks_per_cu=0):
        _check(lib().xcsum_ctx_set_launch(self._ctx, blocks_per_cu), "xcsum_ctx_set_launch")

    def set_order(self, region_log2=-1, tile_log2=0):
        _check(lib().xcsum_ctx_set_order(self._ctx, region_log2, tile_log2),
               "xcsum_ctx_set_order")

    def calibrate_order(self, d_umem, d_desc, n, d_out, mode, flags=0, len_hint=0, stream=None):
        """Time the visiting orders on this batch and keep the fastest
        (xcsum_ctx_calibrate_order); returns (region_log2, tile_log2),
        (-1, 0) = automatic.  Synchronous."""
        r, t = ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().xcsum_ctx_calibrate_order(self._ctx, _ptr(d_umem), _ptr(d_desc), n,
                                               _ptr(d_out), mode, flags, len_hint,
                                               _ptr(stream), ctypes.byref(r), ctypes.byref(t)),
               "xcsum_ctx_calibrate_order")
        return r.value, t.value

    def set_inplace(self, schedule=INPLACE_AUTO):
        """how XCSUM_F_INPLACE writes the check fields (INPLACE_*)"""
        _check(lib().xcsum_ctx_set_inplace(self._ctx, schedule), "xcsum_ctx_set_inplace")

    def set_resident(self, workgroups=0, idle_us=0):
        """Resident workgroups for small host batches (0: off), see xcsum.h."""
        _check(lib().xcsum_ctx_set_resident(self._ctx, workgroups, idle_us),
               "xcsum_ctx_set_resident")

    def set_resident_life(self, life_us=0):
        """The resident workgroups' life bound (0: default 2000 us)."""
        _check(lib().xcsum_ctx_set_resident_life(self._ctx, life_us),
               "xcsum_ctx_set_resident_life")

    def set_tuning(self, knob, a=0, b=0, c=0, d=0):
        """xcsum_ctx_set_tuning (TUNE_*): kernel variant / geometry, never results."""
        _check(lib().xcsum_ctx_set_tuning(self._ctx, knob, a, b, c, d), "xcsum_ctx_set_tuning")

    def take_errors(self):
        c = ctypes.c_uint64(0)
        _check(lib().xcsum_ctx_take_errors(self._ctx, ctypes.byref(c)), "xcsum_ctx_take_errors")
        return int(c.value)

    def batch_device(self, d_umem, d_desc, n, d_out, mode, flags=0, len_hint=0, stream=None):
        """Asynchronous device-resident batch (pointers: torch tensors or ints)."""
        _check(lib().xcsum_batch_device(self._ctx, _ptr(d_umem), _ptr(d_desc), n, _ptr(d_out),
                                        mode, flags, len_hint, _ptr(stream)),
               "xcsum_batch_device")

    def build_device(self, route, d_src, d_msgs, n, d_umem, frame_size, data_off, d_desc_out,
                     d_out=None, flags=0, len_hint=0, stream=None):
        """Device-side xudp_frame_send: headers + payload copy + checksums."""
        _check(lib().xcsum_build_device(self._ctx, ctypes.byref(route), _ptr(d_src),
                                        _ptr(d_msgs), n, _ptr(d_umem), frame_size, data_off,
                                        _ptr(d_desc_out), _ptr(d_out), flags, len_hint,
                                        _ptr(stream)), "xcsum_build_device")

    def rx_device(self, d_umem, d_desc, n, d_msgs, d_count=None, flags=0, len_hint=0,
                  stream=None):
        """Device-side receive batch: parse + fill_msg (+ verify) per frame."""
        _check(lib().xcsum_rx_device(self._ctx, _ptr(d_umem), _ptr(d_desc), n, _ptr(d_msgs),
                                     _ptr(d_count), flags, len_hint, _ptr(stream)),
               "xcsum_rx_device")

    def batch_host(self, umem, desc, out, mode, flags=0):
        _check(lib().xcsum_batch_host(self._ctx, _ptr(umem), _ptr(desc), len(desc), _ptr(out),
                                      mode, flags), "xcsum_batch_host")

    def rx_host(self, umem, desc, msgs, flags=0):
        """Receive batch on host frames; fills msgs (RX_MSG_DTYPE), returns
        the number of XCSUM_RX_OK records."""
        count = ctypes.c_uint32(0)
        _check(lib().xcsum_rx_host(self._ctx, _ptr(umem), _ptr(desc), len(desc), _ptr(msgs),
                                   ctypes.byref(count), flags), "xcsum_rx_host")
        return count.value

    def register_umem(self, buf):
        _check(lib().xcsum_register_umem(self._ctx, _ptr(buf), buf.nbytes),
               "xcsum_register_umem")

    def unregister_umem(self, buf):
        _check(lib().xcsum_unregister_umem(self._ctx, _ptr(buf)), "xcsum_unregister_umem")

    def umem_mapped(self, buf):
        """1: the registered buffer is GPU-mapped; 0: staged (xcsum_umem_mapped)"""
        return _check_nonneg(lib().xcsum_umem_mapped(self._ctx, _ptr(buf)),
                             "xcsum_umem_mapped")

    def pending(self):
        """Host-path slots with work still in flight (0 after every host call)."""
        return _check_nonneg(lib().xcsum_ctx_pending(self._ctx), "xcsum_ctx_pending")

    def sync(self, stream=None):
        _check(lib().xcsum_sync(self._ctx, _ptr(stream)), "xcsum_sync")

    def gen_fill_device(self, d_umem, d_desc, n, family, seed=0, first_index=0, stream=None):
        _check(lib().xcsum_gen_fill_device(_ptr(d_umem), _ptr(d_desc), n, family, seed,
                                           first_index, _ptr(stream)), "xcsum_gen_fill_device")


# ---- packet.c mirror (include/xudp_packet.h) ------------------------------

AF_INET = 2
AF_INET6 = 10


class SockaddrIn(ctypes.Structure):
    _fields_ = [("sin_family", ctypes.c_uint16), ("sin_port", ctypes.c_uint16),
                ("sin_addr", ctypes.c_uint8 * 4), ("sin_zero", ctypes.c_uint8 * 8)]


class SockaddrIn6(ctypes.Structure):
    _fields_ = [("sin6_family", ctypes.c_uint16), ("sin6_port", ctypes.c_uint16),
                ("sin6_flowinfo", ctypes.c_uint32), ("sin6_addr", ctypes.c_uint8 * 16),
                ("sin6_scope_id", ctypes.c_uint32)]


class Route(ctypes.Structure):
    """struct xcsum_route: one batch's addressing (xudp_tx_info_prepare)."""
    _fields_ = [("family", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 3),
                ("dmac", ctypes.c_uint8 * 6), ("smac", ctypes.c_uint8 * 6),
                ("sport_be", ctypes.c_uint16), ("dport_be", ctypes.c_uint16),
                ("saddr", ctypes.c_uint8 * 16), ("daddr", ctypes.c_uint8 * 16)]


def make_route(family, smac, dmac, saddr, sport, daddr, dport):
    """Ports in host order; addresses as bytes (4 or 16)."""
    r = Route()
    r.family = family
    r.dmac[:] = list(dmac)
    r.smac[:] = list(smac)
    r.sport_be = htons(sport)
    r.dport_be = htons(dport)
    r.saddr[:len(saddr)] = list(saddr)
    r.daddr[:len(daddr)] = list(daddr)
    return r


class _FromUnion(ctypes.Union):
    _fields_ = [("_from", SockaddrIn), ("_from6", SockaddrIn6)]


class PacketInfo(ctypes.Structure):
    """struct packet_info (xudp/packet.h:28-53, include/xudp_packet.h)."""
    _fields_ = [("family", ctypes.c_uint8), ("dmac", ctypes.c_void_p), ("smac", ctypes.c_void_p),
                ("to", ctypes.c_void_p), ("from_", ctypes.c_void_p), ("u", _FromUnion),
                ("head", ctypes.c_void_p), ("data", ctypes.c_void_p),
                ("payload", ctypes.c_void_p), ("payload_size", ctypes.c_int),
                ("packet", ctypes.c_void_p), ("len", ctypes.c_int)]


def htons(p):
    return ((p & 0xff) << 8) | (p >> 8)


class PacketArgs:
    """Keeps the buffers a PacketInfo points to alive."""

    def __init__(self, family, payload, smac, dmac, saddr, sport, daddr, dport, headroom=64,
                 tailroom=64, buf=None, offset=0):
        self.family = family
        self.smac = (ctypes.c_uint8 * 6)(*smac)
        self.dmac = (ctypes.c_uint8 * 6)(*dmac)
        if family == 6:
            self.src = SockaddrIn6(AF_INET6, htons(sport), 0, (ctypes.c_uint8 * 16)(*saddr), 0)
            self.dst = SockaddrIn6(AF_INET6, htons(dport), 0, (ctypes.c_uint8 * 16)(*daddr), 0)
        else:
            self.src = SockaddrIn(AF_INET, htons(sport), (ctypes.c_uint8 * 4)(*saddr))
            self.dst = SockaddrIn(AF_INET, htons(dport), (ctypes.c_uint8 * 4)(*daddr))
        self.payload = np.frombuffer(bytes(payload) + b"\0", dtype=np.uint8).copy()
        if buf is None:
            buf = np.zeros(headroom + len(payload) + tailroom, dtype=np.uint8)
        self.buf = buf
        self.info = PacketInfo()
        self.info.family = AF_INET6 if family == 6 else AF_INET
        self.info.dmac = ctypes.addressof(self.dmac)
        self.info.smac = ctypes.addressof(self.smac)
        self.info.to = ctypes.addressof(self.dst)
        self.info.from_ = ctypes.addressof(self.src)
        self.info.head = buf.ctypes.data + offset
        self.info.data = buf.ctypes.data + offset + HDR6 + 2  # == head + XUDP_TX_HEADROOM
        self.info.payload = self.payload.ctypes.data
        self.info.payload_size = len(payload)

    def frame(self):
        """Frame bytes [packet, packet + len) after a build."""
        off = self.info.packet - self.buf.ctypes.data
        return self.buf[off:off + self.info.len].copy()


def packet_build_headers(pa):
    lib().xudp_packet_build_headers(ctypes.byref(pa.info))


def packet_udp_payload(pa):
    packet_lib().xudp_packet_udp_payload(ctypes.byref(pa.info))


def packet_udp(pa):
    packet_lib().xudp_packet_udp(ctypes.byref(pa.info))


def packet_udp_batch(engine, pas, flags=0):
    arr = (PacketInfo * len(pas))(*[p.info for p in pas])
    _check(lib().xudp_packet_udp_batch(engine.ctx if engine else None, arr, len(pas), flags),
           "xudp_packet_udp_batch")
    for p, a in zip(pas, arr):
        p.info.packet = a.packet
        p.info.len = a.len
