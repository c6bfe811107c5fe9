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
    if not os.path.exists(BIN):
        _build()
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
