"""CPU: the registration policy's smaps parser (libxudp_amd/csrc/xcsum_thp.h,
used by xcsum_register_umem) on synthetic /proc/self/smaps text: which VMAs
make a range THP-eligible (staged, never GPU-mapped) under each THP mode.
The header is compiled here by g++ into a small driver; no GPU."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r'''
#include "xcsum_thp.h"
#include <stdlib.h>
int main(int argc, char **argv) {
  /* smaps lo hi never always sh_always sh_advise */
  FILE *f = fopen(argv[1], "r");
  xcsum::ThpModes m;
  m.never = atoi(argv[4]); m.always = atoi(argv[5]);
  m.sh_always = atoi(argv[6]); m.sh_advise = atoi(argv[7]);
  printf("%d\n", (int)xcsum::thp_eligible_smaps(f, strtoul(argv[2], 0, 16),
                                                strtoul(argv[3], 0, 16), m));
  fclose(f);
  return 0;
}
'''

# three VMAs: private anonymous [1000,3000), shared anonymous [5000,7000),
# private [9000,a000)
def smaps(flags_a, flags_b, flags_c="rd wr mr mw me ac"):
    vma = lambda lo, hi, perms, fl: (
        f"{lo}-{hi} {perms} 00000000 00:00 0 \n"
        "Size:                  8 kB\n"
        "AnonHugePages:         0 kB\n"
        "THPeligible:    0\n"
        f"VmFlags: {fl} \n")
    return (vma("1000", "3000", "rw-p", flags_a) + vma("5000", "7000", "rw-s", flags_b)
            + vma("9000", "a000", "rw-p", flags_c))


@pytest.fixture(scope="module")
def driver():
    d = tempfile.mkdtemp()
    src = os.path.join(d, "thp.cc")
    exe = os.path.join(d, "thp")
    open(src, "w").write(DRIVER)
    subprocess.run(["g++", "-O1", "-std=c++17", "-I",
                    os.path.join(ROOT, "libxudp_amd", "csrc"), src, "-o", exe], check=True)

    def run(text, lo, hi, never=0, always=0, sh_always=0, sh_advise=0):
        p = os.path.join(d, "smaps")
        open(p, "w").write(text)
        out = subprocess.run([exe, p, lo, hi, str(never), str(always), str(sh_always),
                              str(sh_advise)], capture_output=True, text=True, check=True)
        return out.stdout.strip() == "1"
    return run


PRIV = "rd wr mr mw me ac"
SHARED = "rd wr sh mr mw me ms lo sd"        # anon_map: MAP_SHARED | MAP_LOCKED


@pytest.mark.parametrize("mode", ["madvise", "always", "never"])
def test_private_vma(driver, mode):
    m = dict(never=int(mode == "never"), always=int(mode == "always"))
    # numpy's MADV_HUGEPAGE heap ("hg"): eligible unless THP is never
    assert driver(smaps(PRIV + " hg", SHARED), "1800", "1900", **m) == (mode != "never")
    # plain private memory: eligible only under "always"
    assert driver(smaps(PRIV, SHARED), "1800", "1900", **m) == (mode == "always")
    # MADV_NOHUGEPAGE ("nh", X.umem_buffer): never eligible
    assert not driver(smaps(PRIV + " nh", SHARED), "1800", "1900", **m)


@pytest.mark.parametrize("shmem", ["never", "advise", "always", "within_size", "force"])
def test_shared_vma(driver, shmem):
    """libxudp's anon_map UMEM is shared memory: its own sysfs mode
    (shmem_enabled) decides; "nh" keeps it mapped under any mode."""
    m = dict(sh_always=int(shmem in ("always", "within_size", "force")),
             sh_advise=int(shmem == "advise"), always=1)
    assert driver(smaps(PRIV, SHARED), "5800", "5900", **m) == (m["sh_always"] == 1)
    assert driver(smaps(PRIV, SHARED + " hg"), "5800", "5900", **m) == (shmem != "never")
    assert not driver(smaps(PRIV, SHARED + " nh"), "5800", "5900", **m)


def test_only_overlapping_vmas_count(driver):
    text = smaps(PRIV + " hg", SHARED, PRIV)
    assert driver(text, "2fff", "3001")          # touches the "hg" VMA's last byte
    assert not driver(text, "3000", "5000")      # the gap
    assert not driver(text, "5000", "6000")      # the shared VMA, shmem never
    assert driver(text, "0", "ffff")             # spans all of them
    assert not driver(text, "9000", "a000")      # a private VMA, THP madvise


def test_flag_tokens_are_whole_words(driver):
    """'sh' inside another token (e.g. a future two-letter flag written next to
    it) does not make a private VMA shared, nor 'hg' a substring match."""
    assert not driver(smaps("rd wr mr xsh", SHARED), "1800", "1900")
    assert not driver(smaps("rd wr mr hgx", SHARED), "1800", "1900")
    assert driver(smaps("hg rd wr", SHARED), "1800", "1900")  # first flag after the colon
