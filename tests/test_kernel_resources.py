"""CPU: the gfx950 code objects as compiled (make -C libxudp_amd asm, the
device ISA + the compiler's resource report): no kernel spills to scratch
memory.  Round 2 hit two ways to lose a fast kernel silently -- a struct
kept in scratch because of a conditional partial update, and register caps
that spill -- and both show up here first."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_kernel_uses_scratch():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "libxudp_amd"), "-j8", "asm"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    rep = open(os.path.join(ROOT, "libxudp_amd", "build", "asm", "resource.txt")).read()
    names = re.findall(r"Function Name: (\S+)", rep)
    scratch = [int(v) for v in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", rep)]
    assert len(names) == len(scratch) and len(names) >= 90
    bad = [n for n, v in zip(names, scratch) if v]
    assert not bad, f"{len(bad)} kernels use scratch: {bad[:5]}"
