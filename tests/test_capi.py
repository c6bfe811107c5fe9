"""The C ABI from plain C (tests/c/capi_check.c): headers compile as C11 with
-Werror, the program links against libxcsum.so like libxudp would, and on a
GPU box every check passes (batches vs the oracle, KAT3/KAT4 frames, error
codes).  Without a GPU the program must report NODEV and skip (exit 77)."""
import os
import subprocess

import pytest

import libxudp_amd as X

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c")
BIN = os.path.join(CDIR, "capi_check")


def _build():
    r = subprocess.run(["make", "-s", "-C", CDIR], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(BIN)


def _run():
    return subprocess.run([BIN], capture_output=True, text=True, timeout=600)


def test_capi_builds_and_skips_without_gpu():
    _build()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_capi_check_gpu")
    r = _run()
    assert r.returncode == 77, r.stdout + r.stderr


@pytest.mark.gpu
def test_capi_check_gpu():
    """Batches vs the oracle (C heap and xudp's anon_map UMEM; staged,
    registered, zero-copy, in place), KAT3/KAT4, error codes, two workers
    forked before any HIP call, two threads with two contexts and streams."""
    if not os.path.exists(BIN):
        _build()
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


RING = os.path.join(CDIR, "umem_ring")


def test_umem_ring_builds_and_skips_without_gpu():
    _build()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_umem_ring_gpu")
    r = subprocess.run([RING], capture_output=True, text=True, timeout=300)
    assert r.returncode == 77, r.stdout + r.stderr


@pytest.mark.gpu
def test_umem_ring_gpu():
    """libxudp's TX loop shape on its own UMEM mapping: checksum batch, then
    descriptors, then the producer index; a NIC thread checks every frame it
    dequeues and completes it; frames are reused (tests/c/umem_ring.c)."""
    if not os.path.exists(RING):
        _build()
    r = subprocess.run([RING], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


TSAN_BIN = os.path.join(CDIR, "tsan", "capi_check")
TSAN_ENV = "halt_on_error=1 exitcode=66 ignore_noninstrumented_modules=1 report_signal_unsafe=0"


@pytest.mark.gpu
def test_threads_tsan_clean():
    """Two host threads, two contexts, two streams on device 0, with the
    library's host code built under ThreadSanitizer (tests/c/Makefile tsan):
    no data race reported, results still exact."""
    if not os.path.exists(TSAN_BIN):
        pytest.fail("tests/c/tsan/capi_check missing: `make -C tests/c tsan` (built by "
                    "__graft_entry__.build())")
    env = dict(os.environ, TSAN_OPTIONS=TSAN_ENV)
    r = subprocess.run([TSAN_BIN, "--threads"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failures" in r.stdout


_NODEV_SCRIPT = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
import libxudp_amd as X
import socket
pa = X.PacketArgs(4, b"abcdef", bytes.fromhex("020000000001"), bytes.fromhex("020000000002"),
                  socket.inet_aton("10.0.35.2"), 3486, socket.inet_aton("10.0.35.1"), 40000)
# the batch call reports the failure and leaves the frame unpublishable
ctypes.memmove(pa.info.data, pa.info.payload, pa.info.payload_size)
rc = X.lib().xudp_packet_udp_batch(None, ctypes.byref(pa.info), 1, 0)
print("batch", rc, pa.frame().tobytes().hex(), flush=True)
# the void mirror cannot report it: it must end the process before returning
X.packet_udp_payload(pa)
print("returned", flush=True)
"""


def _void_mirror_failure(env_extra):
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tests"), **env_extra)
    r = subprocess.run([os.sys.executable, "-c", _NODEV_SCRIPT, ROOT], capture_output=True,
                       text=True, timeout=300, env=env)
    assert "returned" not in r.stdout, r.stdout + r.stderr
    assert r.returncode == -6, (r.returncode, r.stdout + r.stderr)      # SIGABRT
    assert "xudp_packet_udp: the GPU checksum path failed" in r.stderr, r.stderr
    _, rc, frame = r.stdout.split()[-3:]
    from test_oracle import KAT4
    want = bytearray.fromhex(KAT4)
    want[24:26] = b"\0\0"            # iph->check: not computed, never on the CPU
    assert frame == want.hex()
    return int(rc)


def test_void_mirror_failure_contract_without_device():
    """xudp_packet_udp() returns void like packet.c:156 and its caller
    publishes the frame right after (tx.c:649-671).  With no usable GPU the
    batch call returns -XCSUM_ERR_NODEV (headers built, check fields 0), and
    the void mirror aborts the process before returning, so a frame without
    its checksum is never published (include/xudp_packet.h).  A child with
    every device hidden."""
    rc = _void_mirror_failure({"HIP_VISIBLE_DEVICES": "-1", "ROCR_VISIBLE_DEVICES": "-1"})
    assert rc == -X.ERR_NODEV


@pytest.mark.gpu
def test_void_mirror_failure_contract_bad_device():
    """The same on a GPU box through a context that cannot be created:
    XCSUM_DEVICE names a device that does not exist."""
    rc = _void_mirror_failure({"XCSUM_DEVICE": "99"})
    assert rc in (-X.ERR_NODEV, -X.ERR_HIP)


COEXIST = os.path.join(CDIR, "coexist")


def test_coexist_links_beside_packet_o():
    """libxcsum.so links beside a stand-in for libxudp's packet.o (the two
    void mirrors' symbols): no duplicate definitions, the program's calls
    reach packet.o, libxcsum.so defines neither (tests/c/coexist.c).  Without
    a GPU the batch leg reports NODEV and the program exits 77 after the
    link and symbol checks."""
    _build()
    import torch
    r = subprocess.run([COEXIST], capture_output=True, text=True, timeout=300)
    if torch.cuda.is_available():
        assert r.returncode == 0, r.stdout + r.stderr
    else:
        assert r.returncode == 77, r.stdout + r.stderr
        assert "0 failures" in r.stdout


@pytest.mark.gpu
def test_coexist_batch_on_gpu():
    """The same program on a GPU: xudp_packet_udp_batch() builds KAT4 (IPv4)
    and KAT3 (IPv6) byte for byte on the GPU without calling packet.o."""
    if not os.path.exists(COEXIST):
        _build()
    r = subprocess.run([COEXIST], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
