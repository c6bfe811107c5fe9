"""Device-side frame build (xcsum_build_device = xudp_frame_send on the GPU).

CPU: the oracle's packet.c restatement (orc_build_frame) reproduces the frames
the REFERENCE's xudp_packet_udp_payload() built (tests/golden/build_fixtures.npz).
GPU: the build kernel reproduces the same bytes, in copy and in-place modes."""
import os

import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import GOLDEN

ROUTES = {
    4: dict(smac=bytes.fromhex("020000000001"), dmac=bytes.fromhex("020000000002"),
            saddr=bytes([10, 0, 35, 2]), sport=3486, daddr=bytes([10, 0, 35, 1]), dport=40000),
    6: dict(smac=bytes.fromhex("0a1b2c3d4e5f"), dmac=bytes.fromhex("f0e1d2c3b4a5"),
            saddr=bytes.fromhex("10002000300040000000000000000002"), sport=3487,
            daddr=bytes.fromhex("fe800000000000001122334455667788"), dport=65535),
}


@pytest.fixture(scope="module")
def bfix():
    g = np.load(os.path.join(GOLDEN, "build_fixtures.npz"))
    return {k: g[k] for k in g.files}


def split(buf, lens):
    out, o = [], 0
    for L in lens:
        out.append(buf[o:o + L])
        o += L
    return out


def test_build_fixture_shape(bfix):
    for fam, hdr in ((4, 42), (6, 62)):
        lens = bfix[f"v{fam}_lens"]
        assert bfix[f"v{fam}_frames"].size == int(lens.sum()) + hdr * len(lens)
        assert lens.min() == 0 and lens.max() >= 8999


@pytest.mark.parametrize("fam", [4, 6])
def test_oracle_build_matches_reference_frames(bfix, fam):
    hdr = 42 if fam == 4 else 62
    lens = bfix[f"v{fam}_lens"]
    pays = split(bfix[f"v{fam}_payloads"], lens)
    frames = split(bfix[f"v{fam}_frames"], lens + hdr)
    r = ROUTES[fam]
    for p, f in zip(pays, frames):
        got = oracle.build_frame(p.tobytes(), fam, r["smac"], r["dmac"], r["saddr"], r["sport"],
                                 r["daddr"], r["dport"])
        assert np.array_equal(got, f)


def test_build_argument_validation():
    L = X.lib()
    r = X.make_route(4, b"\0" * 6, b"\0" * 6, b"\0" * 4, 1, b"\0" * 4, 2)
    import ctypes
    assert L.xcsum_build_device(None, ctypes.byref(r), None, None, 1, None, 4096, 384, None,
                                None, 0, 0, None) == -X.ERR_INVAL


# every instantiation of build_kernel (csrc/xcsum_build.hip XCSUM_BUILD_GEOMETRIES);
# tests/test_gpu_build.py runs each through XCSUM_BUILD_GEOMETRY
BUILD_GEOMETRIES = [(4, 1), (8, 2), (16, 2), (16, 3), (16, 6), (32, 3), (64, 2), (64, 9)]


def test_build_geometry_list_matches_kernel():
    import re
    src = open(os.path.join(os.path.dirname(X.__file__), "csrc", "xcsum_build.hip")).read()
    body = src.split("#define XCSUM_BUILD_GEOMETRIES(X)")[1].split("\n\n")[0]
    found = [tuple(map(int, m)) for m in re.findall(r"X\((\d+), (\d+)\)", body)]
    assert found == BUILD_GEOMETRIES
