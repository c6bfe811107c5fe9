#!/usr/bin/env python3
"""Generate tests/golden/* from the REFERENCE (run in the build container only).

Every expected value here comes from cclinuxer/libxudp's own code compiled in
place (oracle/_ref/libxudpref.so, recipe oracle/Makefile):
  * frames are built by the reference's xudp_packet_udp_payload()
    (xudp/packet.c:196-203) -- its IPv4 iph->check (xudp_checksum_half,
    packet.c:43-66) and IPv6 udp->check (udp_csum6, packet.c:105-117) are the
    expected outputs; the stored frames have those fields zeroed, i.e. the
    state at the moment the checksum is taken;
  * IPv4 UDP checksums come from udp_checksum() (xudp/checksum.h:107-140,
    single-fold quirk included) and, for the optional RFC mode, from the
    reference's do_csum/sum32/csum_fold composed like udp_csum6.
Outputs:
  fixtures.npz  -- ~1.2k frames (<1 MB): umem bytes, descriptors, family,
                   expected legacy / rfc / v6 / iphdr values
  build_fixtures.npz -- frames built by xudp_packet_udp_payload() for two
                   fixed routes and many payload sizes (device frame build)
  rx_fixtures.npz -- received frames with the reference's packet_parse()
                   results and the expected receive records
  digests.json  -- SHA-256 of the reference's output array for BASELINE.json
                   configs 1-5 over the synthetic generator's frames
                   (libxudp_amd gen_* == reference-built frames, see
                   tests/test_generator.py), plus frame-byte digests.
Usage: python tests/golden/make_golden.py [--no-digests]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import libxudp_amd as X  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED_BASE = 0x78756470  # "xudp"

# BASELINE.json configs: (n, family, pmin, pmax)
CONFIGS = {
    1: (4096, 4, 64, 64),
    2: (1 << 20, 4, 1472, 1472),
    3: (1 << 20, 4, 64, 64),
    4: (1 << 20, 6, 1472, 1472),
    5: (8 << 20, 4, 64, 9000),
}


def be_sum(b):
    """exact integer sum of big-endian 16-bit words (odd tail padded)"""
    b = bytes(b)
    if len(b) % 2:
        b += b"\0"
    a = np.frombuffer(b, dtype=">u2").astype(np.int64)
    return int(a.sum())


class FixtureBuilder:
    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)
        self.frames = []   # (bytes, family)
        self.exp = []      # (legacy, rfc, v6, iphdr)

    def add(self, family, payload, saddr=None, daddr=None, sport=None, dport=None):
        r = self.rng
        smac = r.integers(0, 256, 6, dtype=np.uint8).tobytes()
        dmac = r.integers(0, 256, 6, dtype=np.uint8).tobytes()
        alen = 16 if family == 6 else 4
        saddr = saddr if saddr is not None else r.integers(0, 256, alen, dtype=np.uint8).tobytes()
        daddr = daddr if daddr is not None else r.integers(0, 256, alen, dtype=np.uint8).tobytes()
        sport = int(r.integers(0, 65536)) if sport is None else sport
        dport = int(r.integers(0, 65536)) if dport is None else dport
        f = oracle.build_frame_ref(payload, family, smac, dmac, saddr, sport, daddr, dport)
        R = oracle.ref()
        legacy = rfc = v6 = iph = 0
        if family == 6:
            v6 = int(f[60:62].view("<u2")[0])  # written by the reference's udp_csum6
            f[60:62] = 0
        else:
            iph = int(f[24:26].view("<u2")[0])  # written by xudp_checksum_half
            f[24:26] = 0
            udp = np.ascontiguousarray(f[34:])
            s = int(f[26:30].view("<u4")[0])
            d = int(f[30:34].view("<u4")[0])
            h = R.ref_udp_checksum(udp.ctypes.data, s, d, len(udp))
            legacy = ((h & 0xff) << 8) | (h >> 8)  # htons -> wire order
            sa = np.ascontiguousarray(f[26:30])
            da = np.ascontiguousarray(f[30:34])
            rfc = R.ref_udp_csum4_rfc(udp.ctypes.data, len(udp), sa.ctypes.data, da.ctypes.data)
        self.frames.append((f.tobytes(), family))
        self.exp.append((legacy, rfc, v6, iph))
        return len(self.frames) - 1

    def craft_v4(self, payload_len, target_legacy_host, high=True):
        """IPv4 frame whose legacy result is `target` (host order), by setting
        the last two payload bytes (payload_len even, >= 2)."""
        r = self.rng
        lo = 0xE0 if high else 0
        pl = bytearray(r.integers(lo, 256, payload_len, dtype=np.uint8).tobytes())
        saddr = r.integers(0, 256, 4, dtype=np.uint8).tobytes()
        daddr = r.integers(0, 256, 4, dtype=np.uint8).tobytes()
        sport, dport = int(r.integers(0, 65536)), int(r.integers(0, 65536))
        udp_len = 8 + payload_len
        base = be_sum(saddr + daddr) + 17 + udp_len + be_sum(
            sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + udp_len.to_bytes(2, "big")) + \
            be_sum(pl[:-2])
        want = (~target_legacy_host) & 0xffff  # need (u16)(l + h) == want
        for w in range(65536):
            S = base + w
            if ((S & 0xffff) + (S >> 16)) & 0xffff == want:
                pl[-2:] = w.to_bytes(2, "big")
                return self.add(4, bytes(pl), saddr, daddr, sport, dport)
        raise RuntimeError("no word found")

    def craft_v6_zero(self, payload_len):
        """IPv6 frame whose one's complement sum folds to 0xffff, so
        csum_fold() gives 0 and udp_csum6 maps it to CSUM_MANGLED_0."""
        r = self.rng
        pl = bytearray(r.integers(0, 256, payload_len, dtype=np.uint8).tobytes())
        saddr = r.integers(0, 256, 16, dtype=np.uint8).tobytes()
        daddr = r.integers(0, 256, 16, dtype=np.uint8).tobytes()
        sport, dport = int(r.integers(0, 65536)), int(r.integers(0, 65536))
        udp_len = 8 + payload_len
        pl[-2:] = b"\0\0"
        S = be_sum(saddr + daddr) + 17 + udp_len + be_sum(
            sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + udp_len.to_bytes(2, "big")) + \
            be_sum(pl)
        while S >> 16:
            S = (S & 0xffff) + (S >> 16)
        w = (~S) & 0xffff  # adding w makes the folded sum 0xffff
        pl[-2:] = w.to_bytes(2, "big")
        return self.add(6, bytes(pl), saddr, daddr, sport, dport)

    def pack(self, seed):
        """Place frames back to back at random 1..16-byte phases (odd span
        starts included)."""
        r = np.random.default_rng(seed)
        off = 0
        addr, lens, fam = [], [], []
        for b, f in self.frames:
            off += int(r.integers(0, 16))
            addr.append(off)
            lens.append(len(b))
            fam.append(f)
            off += len(b)
        umem = np.zeros(off + 64, dtype=np.uint8)
        for a, (b, _) in zip(addr, self.frames):
            umem[a:a + len(b)] = np.frombuffer(b, dtype=np.uint8)
        e = np.array(self.exp, dtype=np.uint16)
        return dict(umem=umem, addr=np.array(addr, dtype=np.uint64),
                    len=np.array(lens, dtype=np.uint32), family=np.array(fam, dtype=np.uint8),
                    exp_legacy=e[:, 0], exp_rfc=e[:, 1], exp_v6=e[:, 2], exp_iphdr=e[:, 3])


def build_fixtures():
    fb = FixtureBuilder(12345)
    r = fb.rng
    rnd = lambda n, lo=0: r.integers(lo, 256, n, dtype=np.uint8).tobytes()
    for L in range(0, 300):                       # every small size, random bytes
        fb.add(4, rnd(L))
    for L in range(0, 300):
        fb.add(6, rnd(L))
    for L in range(0, 100):                       # saturating bytes
        fb.add(4, b"\xff" * L, saddr=b"\xff" * 4, daddr=b"\xff" * 4, sport=0xffff, dport=0xffff)
        fb.add(6, b"\xff" * L, saddr=b"\xff" * 16, daddr=b"\xff" * 16, sport=0xffff,
               dport=0xffff)
    for L in (0, 1, 2, 3, 7, 64, 65):             # all-zero frames
        fb.add(4, b"\0" * L, saddr=b"\0" * 4, daddr=b"\0" * 4, sport=0, dport=0)
        fb.add(6, b"\0" * L, saddr=b"\0" * 16, daddr=b"\0" * 16, sport=0, dport=0)
    quirk = 0                                     # legacy != rfc, high-valued bytes
    while quirk < 120:
        L = int(r.integers(1, 1473))
        i = fb.add(4, rnd(L, 0xE0))
        leg, rfc = int(fb.exp[i][0]), int(fb.exp[i][1])
        if leg != rfc:
            quirk += 1
        else:
            fb.frames.pop()
            fb.exp.pop()
    for t in (0x0000, 0xffff, 0xfffe, 0x0001):    # crafted legacy results
        for L in (2, 64, 1472):
            fb.craft_v4(L, t)
    for L in (2, 64, 1472, 8998):                 # crafted IPv6 0 -> 0xffff
        fb.craft_v6_zero(L)
    for L in (1471, 1472):                        # MTU
        for _ in range(5):
            fb.add(4, rnd(L))
            fb.add(6, rnd(L))
    for L in (8999, 9000):                        # jumbo
        fb.add(4, rnd(L))
        fb.add(6, rnd(L))
    d = fb.pack(777)
    np.savez_compressed(os.path.join(OUT, "fixtures.npz"), **d)
    nq = int(((d["family"] == 4) & (d["exp_legacy"] != d["exp_rfc"])).sum())
    print(f"fixtures.npz: {len(d['len'])} frames, {d['umem'].nbytes} umem bytes, "
          f"{nq} IPv4 frames where legacy != rfc")


BUILD_ROUTES = {
    4: dict(smac=bytes.fromhex("020000000001"), dmac=bytes.fromhex("020000000002"),
            saddr=bytes([10, 0, 35, 2]), sport=3486, daddr=bytes([10, 0, 35, 1]), dport=40000),
    6: dict(smac=bytes.fromhex("0a1b2c3d4e5f"), dmac=bytes.fromhex("f0e1d2c3b4a5"),
            saddr=bytes.fromhex("10002000300040000000000000000002"), sport=3487,
            daddr=bytes.fromhex("fe800000000000001122334455667788"), dport=65535),
}


def build_frame_fixtures():
    """Frames built by the reference's xudp_packet_udp_payload() (packet.c:196)
    for two fixed routes and many payload sizes: pins the device frame build."""
    rng = np.random.default_rng(4242)
    out = {}
    for fam, rt in BUILD_ROUTES.items():
        lens = list(range(0, 130)) + [255, 256, 257, 1000, 1457, 1471, 1472, 4095, 8999]
        pays, frames = [], []
        for i, L in enumerate(lens):
            pl = rng.integers(0, 256, L, dtype=np.uint8).tobytes() if i % 7 else b"\xff" * L
            f = oracle.build_frame_ref(pl, fam, rt["smac"], rt["dmac"], rt["saddr"], rt["sport"],
                                       rt["daddr"], rt["dport"])
            pays.append(pl)
            frames.append(f.tobytes())
        out[f"v{fam}_lens"] = np.array(lens, dtype=np.uint32)
        out[f"v{fam}_payloads"] = np.frombuffer(b"".join(pays), dtype=np.uint8)
        out[f"v{fam}_frames"] = np.frombuffer(b"".join(frames), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "build_fixtures.npz"), **out)
    print("build_fixtures.npz:", {k: v.shape for k, v in out.items()})


def sha_u16(h, arr):
    h.update(np.ascontiguousarray(arr, dtype="<u2").tobytes())


def config_digest(cid, chunk=1 << 18, threads=8):
    n, fam, pmin, pmax = CONFIGS[cid]
    seed = SEED_BASE ^ cid
    mode = 2 if fam == 6 else 0
    h_ref = hashlib.sha256()
    h_rfc = hashlib.sha256()
    h_frames = hashlib.sha256() if n <= (1 << 20) else None
    total_alg = 0
    R = oracle.ref()
    P = oracle.port()
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        umem, desc = X.gen_frames_host(m, fam, pmin, pmax, seed=seed, first_index=first)
        out = np.zeros(m, dtype=np.uint16)
        R.ref_batch_timed(umem.ctypes.data, desc.ctypes.data, m, out.ctypes.data, mode, threads, 1)
        sha_u16(h_ref, out)
        if fam == 4:
            rfc = np.zeros(m, dtype=np.uint16)
            P.orc_batch_timed(umem.ctypes.data, desc.ctypes.data, m, rfc.ctypes.data, 1, 0,
                              threads, 1)
            sha_u16(h_rfc, rfc)
        if h_frames is not None:
            for dd in desc:
                h_frames.update(umem[dd["addr"]:dd["addr"] + dd["len"]].tobytes())
        total_alg += X.alg_bytes(desc, fam)
    rec = dict(n=n, family=fam, pmin=pmin, pmax=pmax, seed=seed,
               mode="v6" if fam == 6 else "v4_legacy",
               sha256_out=h_ref.hexdigest(), alg_bytes=total_alg)
    if fam == 4:
        rec["sha256_out_v4_rfc"] = h_rfc.hexdigest()
        rec["v4_rfc_source"] = "oracle port (restatement), cross-checked vs ref_udp_csum4_rfc"
    if h_frames is not None:
        rec["sha256_frames"] = h_frames.hexdigest()
    return rec


def iphdr_digest(cid, chunk=1 << 18):
    """SHA-256 of the reference's xudp_checksum_half() (packet.c:43-66, the one
    checksum libxudp's IPv4 TX call computes) over every frame of an IPv4
    config: the full-size pin of XCSUM_F_IPHDR_ONLY (bench.py --flags
    iphdr_only).  ref_batch mode 4 runs the reference function in place."""
    n, fam, pmin, pmax = CONFIGS[cid]
    assert fam == 4
    seed = SEED_BASE ^ cid
    h = hashlib.sha256()
    R = oracle.ref()
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        umem, desc = X.gen_frames_host(m, fam, pmin, pmax, seed=seed, first_index=first)
        out = np.zeros(m, dtype=np.uint16)
        R.ref_batch(umem.ctypes.data, desc.ctypes.data, m, out.ctypes.data, 4)
        sha_u16(h, out)
    return h.hexdigest()


def shard_digests(cid, worlds=(2, 4, 8), chunk=1 << 18, threads=8):
    """Per-shard SHA-256 of the reference's udp_checksum outputs for a sharded
    config (5): the job split by bytes into N shards (xcsum_shard_by_bytes,
    bench.rank_slice), one digest per shard, so `bench.py --shard r/N` can pin
    one rank's share timed alone.  The concatenation is checked against the
    whole-job sha256_out on the way."""
    n, fam, pmin, pmax = CONFIGS[cid]
    seed = SEED_BASE ^ cid
    mode = 2 if fam == 6 else 0
    R = oracle.ref()
    out = np.zeros(n, dtype=np.uint16)
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        umem, desc = X.gen_frames_host(m, fam, pmin, pmax, seed=seed, first_index=first)
        R.ref_batch_timed(umem.ctypes.data, desc.ctypes.data, m, out[first:].ctypes.data, mode,
                          threads, 1)
    whole = hashlib.sha256(out.astype("<u2").tobytes()).hexdigest()
    full, _ = X.gen_layout(n, fam, pmin, pmax, seed=seed)
    res = {}
    for w in worlds:
        hs, end = [], 0
        for r in range(w):
            first, count = X.shard_by_bytes(full, w, r)
            assert first == end
            end = first + count
            hs.append(hashlib.sha256(out[first:end].astype("<u2").tobytes()).hexdigest())
        assert end == n
        res[f"sha256_out_shards{w}"] = hs
    return whole, res


def rx_fixtures():
    """rx_fixtures.npz: received frames (tests/golden/rx_frames.py corpus) at
    irregular offsets, the reference's own packet_parse() result for each
    (include/packet_parse.h compiled in place), and the records the oracle
    restatement expects from xcsum_rx_device for flags 0 / VERIFY /
    VERIFY|IPHDR."""
    sys.path.insert(0, OUT)
    import rx_frames
    frames, expect = zip(*rx_frames.corpus())
    umem, offs, lens = rx_frames.layout(frames, np.random.default_rng(3))
    desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
    desc["addr"], desc["len"] = offs, lens
    refparse = np.array([oracle.ref_packet_parse(f) for f in frames], dtype=np.int64)
    recs = {f"rec_{name}": oracle.rx_batch(umem, desc, fl).view(np.uint8)
            for name, fl in (("plain", 0), ("verify", X.F_VERIFY),
                             ("iphdr", X.F_VERIFY | X.F_IPHDR))}
    np.savez_compressed(os.path.join(OUT, "rx_fixtures.npz"), umem=umem,
                        desc=desc.view(np.uint8), expect=np.array(expect),
                        refparse=refparse, **recs)
    print(f"rx_fixtures.npz: {len(frames)} frames, {umem.nbytes} bytes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-digests", action="store_true")
    ap.add_argument("--only-build", action="store_true", help="only build_fixtures.npz")
    ap.add_argument("--only-rx", action="store_true", help="only rx_fixtures.npz")
    ap.add_argument("--only-iphdr", action="store_true",
                    help="only add the IPv4 header-checksum digests (sha256_iphdr) to digests.json")
    ap.add_argument("--configs", default="1,2,3,4,5")
    ap.add_argument("--only-shards", action="store_true",
                    help="only add config 5's per-shard digests (sha256_out_shards{2,4,8})")
    args = ap.parse_args()
    if not oracle.have_ref():
        sys.exit("oracle/_ref/libxudpref.so missing: run `make -C oracle` next to /root/reference")
    if args.only_shards:
        path = os.path.join(OUT, "digests.json")
        digests = json.load(open(path))
        whole, res = shard_digests(5)
        assert whole == digests["config5"]["sha256_out"], "config 5 whole-job digest moved"
        digests["config5"].update(res)
        digests["config5"]["shards_source"] = \
            "reference checksum.h udp_checksum (oracle/_ref), split by xcsum_shard_by_bytes"
        json.dump(digests, open(path, "w"), indent=1, sort_keys=True)
        print({k: v[:1] for k, v in res.items()})
        return
    if args.only_build:
        build_frame_fixtures()
        return
    if args.only_rx:
        rx_fixtures()
        return
    if args.only_iphdr:
        path = os.path.join(OUT, "digests.json")
        digests = json.load(open(path))
        for c in [int(x) for x in args.configs.split(",")]:
            if CONFIGS[c][1] == 4:
                digests[f"config{c}"]["sha256_iphdr"] = iphdr_digest(c)
                digests[f"config{c}"]["iphdr_source"] = \
                    "reference xudp_checksum_half (packet.c:43-66), oracle/_ref ref_batch mode 4"
                print(f"config{c}: sha256_iphdr {digests[f'config{c}']['sha256_iphdr']}")
        json.dump(digests, open(path, "w"), indent=1, sort_keys=True)
        return
    build_fixtures()
    build_frame_fixtures()
    rx_fixtures()
    if not args.no_digests:
        path = os.path.join(OUT, "digests.json")
        digests = json.load(open(path)) if os.path.exists(path) else {}
        for c in [int(x) for x in args.configs.split(",")]:
            digests[f"config{c}"] = config_digest(c)
            print(f"config{c}: {digests[f'config{c}']}")
            json.dump(digests, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
