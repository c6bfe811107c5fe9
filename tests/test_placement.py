"""CPU: device placement of libxudp's groups over a node's GPUs (VERDICT r5
#2; include/xcsum.h "device placement").  libxudp runs group_num groups as
threads or forked workers (ref include/xudp.h:196-199, :310-311,
test/case/lib.c:196-221); xcsum_device_resolve is the mapping
xcsum_ctx_create applies, pinned here over faked device counts (1, 2, 8)
with 8 threads -- no GPU needed."""
import os
import subprocess
import sys
import threading
from collections import Counter

import pytest

import libxudp_amd as X

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("ndev", [1, 2, 8])
def test_auto_round_robin_over_8_threads(ndev):
    """8 group threads each creating one AUTO context: every device gets
    8/ndev of them (the round robin is process-wide and thread-safe)."""
    got, barrier = [], threading.Barrier(8)

    def worker():
        barrier.wait()
        got.append(X.device_resolve(X.DEVICE_AUTO, ndev))

    th = [threading.Thread(target=worker) for _ in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert len(got) == 8 and all(0 <= d < ndev for d in got)
    assert Counter(got) == Counter({d: 8 // ndev for d in range(ndev)})


@pytest.mark.parametrize("ndev", [1, 2, 8])
def test_group_mapping_is_gid_mod_ndev(ndev):
    """XCSUM_DEVICE_GROUP(gid): device gid mod the visible count, whatever
    the thread timing or process (forked workers)."""
    for gid in list(range(20)) + [1000, 999999, 1000000]:
        assert X.device_resolve(X.DEVICE_GROUP(gid), ndev) == gid % ndev
    # 8 groups on 8 GPUs: one each
    assert sorted(X.device_resolve(X.DEVICE_GROUP(g), 8) for g in range(8)) == list(range(8))


def test_explicit_and_invalid_devices():
    assert X.device_resolve(3, 8) == 3
    assert X.device_resolve(8, 8) == -X.ERR_NODEV
    assert X.device_resolve(0, 1) == 0
    assert X.device_resolve(-3, 8) == -X.ERR_INVAL          # no such policy
    assert X.device_resolve(X.DEVICE_GROUP(1000001), 8) == -X.ERR_INVAL


_ENV_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import libxudp_amd as X
print(X.device_resolve(X.DEVICE_ENV, 8), X.device_resolve(X.DEVICE_ENV, 2))
"""


@pytest.mark.parametrize("env,want", [({}, "0 0"), ({"XCSUM_DEVICE": "5"}, "5 -9002")])
def test_env_policy(env, want):
    """XCSUM_DEVICE_ENV (-1, the rounds 1-5 default): $XCSUM_DEVICE, else 0."""
    e = {k: v for k, v in os.environ.items() if k != "XCSUM_DEVICE"}
    e.update(env)
    r = subprocess.run([sys.executable, "-c", _ENV_SCRIPT, ROOT], capture_output=True,
                       text=True, env=e, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == want.split()


def test_thread_init_without_gpu_is_an_error_code():
    """a missing device is reported by xcsum_thread_init at a
    worker's start-up (an error code), not by an abort on the first send."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: tests/test_gpu_placement.py")
    assert X.lib().xcsum_device_count() == -X.ERR_NODEV
    assert X.lib().xcsum_thread_init(3) == -X.ERR_NODEV
    assert X.lib().xcsum_thread_init(-1) == -X.ERR_NODEV
    assert X.lib().xcsum_thread_ctx() is None
