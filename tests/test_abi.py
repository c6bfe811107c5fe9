"""CPU: the C-ABI library loads and exports exactly what include/*.h declares;
argument validation works without touching a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import libxudp_amd as X

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("xcsum.h", "xudp_packet.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[a-z][\w \*]*?\b(\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def exported_symbols(path=None):
    out = subprocess.run(["nm", "-D", "--defined-only", path or X.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_library_loads():
    assert X.lib() is not None
    assert X.packet_lib() is not None


def test_every_declared_function_is_exported():
    """libxcsum.so exports every declared function except the two packet.o
    symbols, which only libxcsum_packet.so defines (so libxcsum.so links
    beside libxudp's own packet.o, ref Makefile:41)."""
    decl = declared_functions()
    mirror = set(X._PACKET_SIGS)
    assert mirror == {"xudp_packet_udp", "xudp_packet_udp_payload"}
    assert set(decl) == set(X._SIGS) | mirror, set(decl) ^ (set(X._SIGS) | mirror)
    core = exported_symbols()
    missing = sorted(set(decl) - mirror - core)
    assert not missing, missing
    assert not (mirror & core), "libxcsum.so must not define packet.o's symbols"
    pk = exported_symbols(X.PACKET_LIB_PATH)
    assert mirror <= pk and not (pk & set(X._SIGS)), pk


def test_packet_mirror_needs_libxcsum_by_soname():
    """libxcsum_packet.so binds to whichever libxcsum.so the process loaded
    (the product, the debug or the TSan build): DT_NEEDED libxcsum.so, and
    every build of libxcsum.so carries that SONAME."""
    out = subprocess.run(["readelf", "-d", X.PACKET_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert "Shared library: [libxcsum.so]" in out
    out = subprocess.run(["readelf", "-d", X.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert "Library soname: [libxcsum.so]" in out


def test_python_binding_covers_the_abi():
    assert len(declared_functions()) >= 20


def test_struct_layouts_match_c():
    """struct xcsum_desc == struct xdp_desc (16 B); struct packet_info matches
    xudp/packet.h:28-53 as compiled by gcc from include/xudp_packet.h."""
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include <linux/if_xdp.h>
#include "xudp_packet.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(struct xcsum_desc),
         sizeof(struct xdp_desc), offsetof(struct xdp_desc, len),
         sizeof(struct packet_info), offsetof(struct packet_info, head),
         offsetof(struct packet_info, payload_size), offsetof(struct packet_info, packet),
         offsetof(struct packet_info, len));
  return 0; }'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o",
                        os.path.join(d, "l")], check=True)
        vals = [int(v) for v in subprocess.run([os.path.join(d, "l")], capture_output=True,
                                               text=True, check=True).stdout.split()]
    assert vals[0] == vals[1] == 16 and vals[2] == 8
    P = X.PacketInfo
    assert vals[3:] == [ctypes.sizeof(P), P.head.offset, P.payload_size.offset, P.packet.offset,
                        P.len.offset]


REF_PACKET_H = "/root/reference/xudp/packet.h"


@pytest.mark.skipif(not os.path.exists(REF_PACKET_H), reason="reference not present")
def test_packet_info_layout_equals_reference():
    """Compile the reference's packet.h and ours side by side (build container only)."""
    import tempfile
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include HDR
int main(void){ printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(struct packet_info),
 offsetof(struct packet_info, dmac), offsetof(struct packet_info, head),
 offsetof(struct packet_info, data), offsetof(struct packet_info, payload_size),
 offsetof(struct packet_info, packet), offsetof(struct packet_info, len)); return 0; }'''
    outs = []
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(prog)
        for hdr, inc in (('"packet.h"', ["-I", "/root/reference/xudp", "-I",
                                         "/root/reference/common"]),
                         ('"xudp_packet.h"', ["-I", os.path.join(ROOT, "include")])):
            exe = os.path.join(d, "p%d" % len(outs))
            subprocess.run(["gcc", f"-DHDR={hdr}", *inc, c, "-o", exe], check=True)
            outs.append(subprocess.run([exe], capture_output=True, text=True).stdout)
    assert outs[0] == outs[1]


def test_ctx_create_without_gpu_reports_nodev():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(X.XcsumError) as e:
        X.Engine(0)
    assert e.value.rc == -X.ERR_NODEV


def test_argument_validation_without_gpu():
    L = X.lib()
    assert L.xcsum_batch_device(None, None, None, 0, None, 0, 0, 0, None) == -X.ERR_INVAL
    assert L.xcsum_batch_host(None, None, None, 1, None, 0, 0) == -X.ERR_INVAL
    assert L.xcsum_ctx_set_geometry(None, 16, 1, 6) == -X.ERR_INVAL
    assert L.xcsum_ctx_create(0, None) == -X.ERR_INVAL
    assert L.xcsum_ctx_device(None) == -X.ERR_INVAL
    n = ctypes.c_uint64(0)
    d = np.zeros(4, dtype=X.DESC_DTYPE)
    assert L.xcsum_gen_layout(4, 5, 0, 10, 0, 0, 8, 0, 0, d.ctypes.data, ctypes.byref(n)) \
        == -X.ERR_INVAL                                   # family must be 4 or 6
    assert L.xcsum_gen_layout(4, 4, 10, 5, 0, 0, 8, 0, 0, d.ctypes.data, ctypes.byref(n)) \
        == -X.ERR_INVAL                                   # pmin > pmax
    assert L.xcsum_gen_layout(4, 4, 0, 5000, 0, 0, 8, 4096, 342, d.ctypes.data,
                              ctypes.byref(n)) == -X.ERR_INVAL  # frame exceeds stride
    f, c = ctypes.c_uint32(), ctypes.c_uint32()
    assert L.xcsum_shard_by_bytes(d.ctypes.data, 4, 2, 2, ctypes.byref(f), ctypes.byref(c)) \
        == -X.ERR_INVAL
    assert L.xcsum_unregister_umem(None, None) == -X.ERR_INVAL
    assert L.xudp_packet_udp_batch(None, None, 0, 0) == 0       # empty batch is a no-op
    r, t = ctypes.c_int(7), ctypes.c_int(7)
    assert L.xcsum_ctx_calibrate_order(None, None, None, 1, None, 0, 0, 0, None,
                                       ctypes.byref(r), ctypes.byref(t)) == -X.ERR_INVAL
    assert (r.value, t.value) == (7, 7)                         # untouched on error
    assert L.xcsum_ctx_set_tuning(None, X.TUNE_IPHDR_FPT, 4, 0, 0, 0) == -X.ERR_INVAL
    assert L.xcsum_ctx_set_resident_life(None, 100) == -X.ERR_INVAL
    assert L.xcsum_ctx_create_for_group(-1, None) == -X.ERR_INVAL


def test_geometry_list_matches_kernel_source():
    """X.GEOMETRIES (what the parity tests sweep) == the instantiations in
    the XCSUM_GEOMETRIES table (csrc/xcsum_csum.h, instantiated per feature set
    in xcsum_csum_f{0,1,2}.hip) + the stream dispatch of csrc/xcsum_kernels.hip;
    the A/B lists == the dispatch of csrc/variants/ (LDS-staged, segmented)."""
    import re
    csrc = os.path.join(ROOT, "libxudp_amd", "csrc")
    src = open(os.path.join(csrc, "xcsum_kernels.hip")).read()
    vsrc = open(os.path.join(csrc, "variants", "xcsum_lds.hip")).read()
    hdr = open(os.path.join(csrc, "xcsum_csum.h")).read()
    table = hdr[hdr.index("#define XCSUM_GEOMETRIES"):]
    table = table[:table.index("\n\n")]
    reg = [tuple(map(int, m)) for m in re.findall(r"X\((\d+), (\d+), (\d+)\)", table)]
    lds = [tuple(map(int, m)) for m in re.findall(
        r"g\.U == (\d+) && g\.K == (\d+)\) return launch_lds_t", vsrc)]
    lds = [(16, int(u), int(k)) for u, k in lds]
    stream = [(64, 0, int(k)) for k in re.findall(
        r"if \(g\.K == (\d+)\) return launch_stream_t", src)]
    internal = open(os.path.join(csrc, "variants", "xcsum_variants.h")).read()
    segt = internal[internal.index("#define XCSUM_SEG_GEOMETRIES"):]
    segt = segt[:segt.index("\n")]
    seg = [(64, int(f), int(d)) for f, d in re.findall(r"X\((\d+), (\d+)\)", segt)]
    assert sorted(seg) == sorted(X.SEG_GEOMETRIES)
    assert reg == X.REG_GEOMETRIES
    assert sorted(lds) == sorted(X.LDS_GEOMETRIES)
    assert sorted(stream) == sorted(X.STREAM_GEOMETRIES)
    assert X.GEOMETRIES == X.REG_GEOMETRIES + X.STREAM_GEOMETRIES


def test_rx_msg_layout_matches_c():
    """struct xcsum_rx_msg (64 B) == libxudp_amd.RX_MSG_DTYPE, field by field."""
    names = [n for n in X.RX_MSG_DTYPE.names]
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"xcsum.h\"\nint main(void){\n" + \
        'printf("%zu\\n", sizeof(struct xcsum_rx_msg));\n' + "".join(
            f'printf("%zu\\n", offsetof(struct xcsum_rx_msg, {n}));\n' for n in names) + \
        "return 0; }\n"
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "r.c")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o",
                        os.path.join(d, "r")], check=True)
        vals = [int(v) for v in subprocess.run([os.path.join(d, "r")], capture_output=True,
                                               text=True, check=True).stdout.split()]
    assert vals[0] == X.RX_MSG_DTYPE.itemsize == 64
    assert vals[1:] == [X.RX_MSG_DTYPE.fields[n][1] for n in names]


def test_constants_match_header():
    """Every mode, flag, error code, schedule and receive status the Python
    binding mirrors has the value include/xcsum.h gives it (compiled by gcc
    and printed, no GPU)."""
    import subprocess
    import tempfile
    names = {
        "XCSUM_MODE_V4_LEGACY": X.MODE_V4_LEGACY, "XCSUM_MODE_V4_RFC": X.MODE_V4_RFC,
        "XCSUM_MODE_V6": X.MODE_V6, "XCSUM_MODE_AUTO": X.MODE_AUTO,
        "XCSUM_F_INPLACE": X.F_INPLACE, "XCSUM_F_IPHDR": X.F_IPHDR,
        "XCSUM_F_V4_RFC": X.F_V4_RFC, "XCSUM_F_ZEROCOPY": X.F_ZEROCOPY,
        "XCSUM_F_VERIFY": X.F_VERIFY, "XCSUM_F_IPHDR_ONLY": X.F_IPHDR_ONLY,
        "XCSUM_F_BUILD_INPLACE": X.F_BUILD_INPLACE, "XCSUM_F_SRC_ALIGNED": X.F_SRC_ALIGNED,
        "XCSUM_ERR_INVAL": X.ERR_INVAL, "XCSUM_ERR_HIP": X.ERR_HIP,
        "XCSUM_ERR_NODEV": X.ERR_NODEV, "XCSUM_ERR_NOMEM": X.ERR_NOMEM,
        "XCSUM_ERR_NOT_REGISTERED": X.ERR_NOT_REGISTERED, "XCSUM_ERR_FRAME": X.ERR_FRAME,
        "XCSUM_INPLACE_AUTO": X.INPLACE_AUTO, "XCSUM_INPLACE_FUSED": X.INPLACE_FUSED,
        "XCSUM_INPLACE_TWO_PASS": X.INPLACE_TWO_PASS,
        "XCSUM_RX_OK": X.RX_OK, "XCSUM_RX_PARSE": X.RX_PARSE, "XCSUM_RX_STATS": X.RX_STATS,
        "XCSUM_RX_CSUM": X.RX_CSUM,
        "XCSUM_TUNE_IPHDR_FPT": X.TUNE_IPHDR_FPT, "XCSUM_TUNE_BUILD_HDR": X.TUNE_BUILD_HDR,
        "XCSUM_TUNE_BUILD_GEOMETRY": X.TUNE_BUILD_GEOMETRY,
        "XCSUM_TUNE_RX_GEOMETRY": X.TUNE_RX_GEOMETRY, "XCSUM_TUNE_RX_ORDER": X.TUNE_RX_ORDER,
        "XCSUM_TUNE_GATHER_RATIO": X.TUNE_GATHER_RATIO,
        "XCSUM_TUNE_INPLACE_BLOCK": X.TUNE_INPLACE_BLOCK,
        "XCSUM_TUNE_INPLACE_TL": X.TUNE_INPLACE_TL,
        "XCSUM_TUNE_RESIDENT_INLINE": X.TUNE_RESIDENT_INLINE,
        "XCSUM_TUNE_RESIDENT_LIMIT_CUT": X.TUNE_RESIDENT_LIMIT_CUT,
        "XCSUM_TUNE_CLAIM": X.TUNE_CLAIM,
        "XCSUM_DEVICE_ENV": X.DEVICE_ENV, "XCSUM_DEVICE_AUTO": X.DEVICE_AUTO,
        "XCSUM_DEVICE_GROUP(7)": X.DEVICE_GROUP(7),
    }
    src = "#include <stdio.h>\n#include \"xcsum.h\"\nint main(void) {\n" + "".join(
        f'  printf("{k} %lld\\n", (long long)({k}));\n' for k in names) + "  return 0;\n}\n"
    d = tempfile.mkdtemp()
    open(os.path.join(d, "c.c"), "w").write(src)
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", os.path.join(d, "c.c"), "-o", os.path.join(d, "c")],
                   check=True)
    out = subprocess.run([os.path.join(d, "c")], capture_output=True, text=True, check=True).stdout
    got = {k: int(v) for k, v in (line.rsplit(" ", 1) for line in out.splitlines())}
    assert got == names


def test_make_install_tree_links():
    """`make -C libxudp_amd install PREFIX=...`: both
    libraries, both headers and xcsum.pc land in the tree, and C programs
    built with the .pc file's flags link and load from it -- setup (a)
    against -lxcsum (a context without a GPU reports NODEV), setup (b) with
    -lxcsum_packet -lxcsum (the mirror library finds libxcsum.so by its
    $ORIGIN rpath).  No GPU."""
    import tempfile
    pre = tempfile.mkdtemp()
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "libxudp_amd"), "install",
                        f"PREFIX={pre}"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    for f in ("lib/libxcsum.so", "lib/libxcsum_packet.so", "include/xcsum.h",
              "include/xudp_packet.h", "lib/pkgconfig/xcsum.pc"):
        assert os.path.exists(os.path.join(pre, f)), f
    pc = dict(line.split("=", 1) for line in open(os.path.join(pre, "lib/pkgconfig/xcsum.pc"))
              .read().splitlines() if "=" in line and ":" not in line)
    fields = dict(line.split(": ", 1) for line in open(os.path.join(pre, "lib/pkgconfig/xcsum.pc"))
                  .read().splitlines() if ": " in line)

    def expand(v):
        for _ in range(3):
            for k, x in pc.items():
                v = v.replace("${" + k + "}", x)
        return v.split()
    assert pc["prefix"] == pre
    src_a = ('#include <stdio.h>\n#include <xcsum.h>\nint main(void) { xcsum_ctx *c = 0;\n'
             '  int rc = xcsum_ctx_create(-1, &c); if (!rc) xcsum_ctx_destroy(c);\n'
             '  printf("%d\\n", rc); return 0; }\n')
    src_b = ('#include <stdio.h>\n#include <xudp_packet.h>\nint main(void) {\n'
             '  printf("%d\\n", xudp_packet_udp != 0 && xudp_packet_udp_batch != 0); return 0; }\n')
    d = tempfile.mkdtemp()
    outs = []
    for name, src, extra in (("a", src_a, []), ("b", src_b, ["-lxcsum_packet"])):
        open(os.path.join(d, name + ".c"), "w").write(src)
        exe = os.path.join(d, name)
        libs = expand(fields["Libs"])
        subprocess.run(["gcc", "-std=c11", *expand(fields["Cflags"]), os.path.join(d, name + ".c"),
                        "-o", exe, *libs[:1], *extra, *libs[1:]], check=True)
        env = {k: v for k, v in os.environ.items() if k != "LD_LIBRARY_PATH"}
        outs.append(subprocess.run([exe], capture_output=True, text=True, check=True,
                                   env=env, timeout=120).stdout.strip())
    assert outs[0] in ("0", str(-X.ERR_NODEV))
    assert outs[1] == "1"
