"""oracle -- TEST INFRASTRUCTURE ONLY: ctypes bindings of the parity oracles.

* ``port()``: oracle/liboracle.so, the CPU restatement of xudp/checksum.h and
  xudp/packet.c (oracle/xcsum_oracle.c, every function cites file:line).
* ``ref()``: oracle/_ref/libxudpref.so, the reference's own packet.c and
  checksum.h compiled in place (oracle/Makefile, oracle/ref_shim.c); it exists
  only where it was built from /root/reference (it travels to the GPU box as
  a prebuilt binary, never as source).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this package, and only as the checker / timed CPU baseline.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libxudpref.so")

MODE_V4_LEGACY, MODE_V4_RFC, MODE_V6, MODE_AUTO = 0, 1, 2, 3

_port = None
_ref = None

u8p = ctypes.c_void_p


def port():
    global _port
    if _port is None:
        if not os.path.exists(PORT_PATH):
            raise FileNotFoundError(f"{PORT_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(PORT_PATH)
        L.orc_checksum.restype = ctypes.c_uint16
        L.orc_checksum.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_udp_checksum.restype = ctypes.c_uint16
        L.orc_udp_checksum.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16]
        L.orc_udp_csum6.restype = ctypes.c_uint16
        L.orc_udp_csum6.argtypes = [u8p, ctypes.c_uint32, u8p, u8p]
        L.orc_ip_checksum_half.restype = ctypes.c_uint16
        L.orc_ip_checksum_half.argtypes = [u8p]
        L.orc_ip_header_rfc.restype = ctypes.c_uint16
        L.orc_ip_header_rfc.argtypes = [u8p]
        L.orc_build_frame.restype = ctypes.c_uint32
        L.orc_build_frame.argtypes = [u8p, u8p, ctypes.c_uint32, ctypes.c_int, u8p, u8p, u8p,
                                      ctypes.c_uint16, u8p, ctypes.c_uint16, ctypes.c_int]
        L.orc_batch.restype = None
        L.orc_batch.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int, ctypes.c_uint32]
        L.orc_batch_timed.restype = ctypes.c_double
        L.orc_batch_timed.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int,
                                      ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
        L.orc_packet_parse.restype = ctypes.c_int
        L.orc_packet_parse.argtypes = [u8p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_uint32)]
        L.orc_rx_batch.restype = None
        L.orc_rx_batch.argtypes = [u8p, u8p, ctypes.c_uint32, ctypes.c_uint32, u8p]
        _port = L
    return _port


def have_ref():
    return os.path.exists(REF_PATH)


def ref():
    global _ref
    if _ref is None:
        if not have_ref():
            raise FileNotFoundError(f"{REF_PATH} missing (built only where /root/reference exists)")
        L = ctypes.CDLL(REF_PATH)
        L.ref_udp_checksum.restype = ctypes.c_uint16
        L.ref_udp_checksum.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16]
        L.ref_udp_csum6.restype = ctypes.c_uint16
        L.ref_udp_csum6.argtypes = [u8p, ctypes.c_uint32, u8p, u8p]
        L.ref_udp_csum4_rfc.restype = ctypes.c_uint16
        L.ref_udp_csum4_rfc.argtypes = [u8p, ctypes.c_uint32, u8p, u8p]
        L.ref_ip_checksum_half.restype = ctypes.c_uint16
        L.ref_ip_checksum_half.argtypes = [u8p]
        L.ref_packet_udp_payload.restype = ctypes.c_int
        L.ref_packet_udp_payload.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, u8p, u8p,
                                             u8p, ctypes.c_uint16, u8p, ctypes.c_uint16,
                                             ctypes.POINTER(ctypes.c_int64)]
        L.ref_packet_parse.restype = ctypes.c_int
        L.ref_packet_parse.argtypes = [u8p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_uint32)]
        L.ref_batch.restype = None
        L.ref_batch.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int]
        L.ref_batch_timed.restype = ctypes.c_double
        L.ref_batch_timed.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int]
        _ref = L
    return _ref


def _p(a):
    return a.ctypes.data if a is not None else None


def batch(umem, desc, mode, flags=0):
    """Oracle (restatement) output for a batch: uint16 array, wire order."""
    out = np.zeros(len(desc), dtype=np.uint16)
    port().orc_batch(_p(umem), _p(desc), len(desc), _p(out), mode, flags)
    return out


def ref_batch(umem, desc, mode):
    """Reference output (modes 0 = IPv4 udp_checksum, 2 = IPv6 udp_csum6)."""
    out = np.zeros(len(desc), dtype=np.uint16)
    ref().ref_batch(_p(umem), _p(desc), len(desc), _p(out), mode)
    return out


def ip_header_rfc(frame_bytes):
    buf = np.ascontiguousarray(frame_bytes[14:34], dtype=np.uint8)
    return port().orc_ip_header_rfc(_p(buf))


def build_frame_ref(payload, family, smac, dmac, saddr, sport, daddr, dport):
    """Frame exactly as the reference xudp_packet_udp_payload() writes it.
    Ports are host-order ints; returns the frame bytes (uint8 array)."""
    head = np.zeros(64 + len(payload) + 64, dtype=np.uint8)
    pl = np.frombuffer(bytes(payload), dtype=np.uint8).copy() if len(payload) else \
        np.zeros(1, dtype=np.uint8)
    off = ctypes.c_int64(0)
    b = lambda x: np.frombuffer(bytes(x), dtype=np.uint8).copy()
    sm, dm, sa, da = b(smac), b(dmac), b(saddr), b(daddr)
    be = lambda p: ((p & 0xff) << 8) | (p >> 8)  # htons as the raw u16 value
    ln = ref().ref_packet_udp_payload(_p(head), _p(pl), len(payload), family, _p(sm), _p(dm),
                                      _p(sa), be(sport), _p(da), be(dport), ctypes.byref(off))
    return head[off.value:off.value + ln].copy()


def build_frame(payload, family, smac, dmac, saddr, sport, daddr, dport, v4_rfc=False):
    """Frame bytes from the oracle's packet.c restatement (orc_build_frame)."""
    pl = np.frombuffer(bytes(payload) + b"\0", dtype=np.uint8).copy()
    buf = np.zeros(len(payload) + 64, dtype=np.uint8)
    b = lambda x: np.frombuffer(bytes(x), dtype=np.uint8).copy()
    sm, dm, sa, da = b(smac), b(dmac), b(saddr), b(daddr)
    be = lambda p: ((p & 0xff) << 8) | (p >> 8)
    n = port().orc_build_frame(_p(buf), _p(pl), len(payload), family, _p(dm), _p(sm), _p(sa),
                               be(sport), _p(da), be(dport), int(bool(v4_rfc)))
    return buf[:n].copy()


def _parse(fn, frame):
    buf = np.ascontiguousarray(np.frombuffer(bytes(frame), dtype=np.uint8))
    fam, l3, l4 = ctypes.c_int(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
    r = fn(_p(buf), len(buf), ctypes.byref(fam), ctypes.byref(l3), ctypes.byref(l4))
    return (int(r), fam.value, l3.value, l4.value) if r == 1 else (int(r), 0, 0, 0)


def packet_parse(frame):
    """The restatement of include/packet_parse.h:101-165: (ret, family, l3, l4)."""
    return _parse(port().orc_packet_parse, frame)


def ref_packet_parse(frame):
    """The reference's own packet_parse(), compiled from include/packet_parse.h."""
    return _parse(ref().ref_packet_parse, frame)


RX_MSG_DTYPE = np.dtype([("frame", "<u8"), ("body", "<u8"), ("size", "<u4"), ("status", "u1"),
                         ("family", "u1"), ("l4_off", "<u2"), ("sport_be", "<u2"),
                         ("dport_be", "<u2"), ("reserved", "<u4"), ("saddr", "u1", 16),
                         ("daddr", "u1", 16)])


def rx_batch(umem, desc, flags=0):
    """Receive records (struct xcsum_rx_msg) the oracle expects for a batch."""
    out = np.zeros(len(desc), dtype=RX_MSG_DTYPE)
    port().orc_rx_batch(_p(umem), _p(desc), len(desc), flags, _p(out))
    return out
