"""The C ABI from plain C (tests/c/capi_check.c): headers compile as C11 with
-Werror, the program links against libxcsum.so like libxudp would, and on a
GPU box every check passes (batches vs the oracle, KAT3/KAT4 frames, error
codes).  Without a GPU the program must report NODEV and skip (exit 77)."""
import os
import subprocess

import pytest

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
import ctypes, errno, os, sys
sys.path.insert(0, sys.argv[1])
import libxudp_amd as X
from test_oracle import KAT4
L = ctypes.CDLL(X.LIB_PATH, use_errno=True)
import socket
pa = X.PacketArgs(4, b"abcdef", bytes.fromhex("020000000001"), bytes.fromhex("020000000002"),
                  socket.inet_aton("10.0.35.2"), 3486, socket.inet_aton("10.0.35.1"), 40000)
ctypes.set_errno(0)
L.xudp_packet_udp_payload(ctypes.byref(pa.info))
print(ctypes.get_errno() == errno.EIO, pa.frame().tobytes().hex())
"""


def test_void_mirror_failure_path_without_device():
    """xudp_packet_udp() returns void like packet.c:156.  With no usable GPU it
    cannot checksum: it must say so through errno = EIO and leave both check
    fields 0 with every other header byte built --
    never a CPU-computed value.  Run in a child with every device hidden."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1",
               PYTHONPATH=os.path.join(ROOT, "tests"))
    r = subprocess.run([os.sys.executable, "-c", _NODEV_SCRIPT, ROOT], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    eio, frame = r.stdout.split()[-2:]
    from test_oracle import KAT4
    want = bytearray.fromhex(KAT4)
    want[24:26] = b"\0\0"            # iph->check: not computed
    assert eio == "True"
    assert frame == want.hex()
