"""CPU: the host path's copies into the pinned stages
(libxudp_amd/csrc/xcsum_stage.h, used by xcsum_batch_host / xcsum_rx_host /
xudp_packet_udp_batch): the frame-by-frame gather (each frame at its 16-byte
phase, at most `cap` bytes, staged descriptors keeping the frame's length),
split over threads from 16K frames or 4 MiB up, and the threaded range copy
-- against a serial restatement, byte for byte, on random descriptor sets.
Compiled here by g++ into a small driver (and once more under
ThreadSanitizer when the toolchain has it); no GPU."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r'''
#include "xcsum_stage.h"
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint64_t rnd() {                      /* SplitMix64 */
  uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

int main(int argc, char **argv) {
  if (argc == 2 && !strcmp(argv[1], "budget")) {
    /* threads a large copy takes under this process's CPU budget */
    printf("usable=%d threads=%d\n", xcsum::usable_cpus(),
           xcsum::stage_threads(64u << 20, 1));
    return 0;
  }
  if (argc == 2 && !strcmp(argv[1], "grow")) {
    /* the pool grows between calls (2 parts, then 4, then 3 ...): every part
     * of every call runs exactly once, on a worker or the caller */
    xcsum::StagePool pool;
    const int ks[] = {2, 4, 3, 1, 4, 2};
    for (int rep = 0; rep < 2000; rep++) {
      const int k = ks[rep % 6];
      int hits[xcsum::STAGE_THREADS] = {0};
      pool.run(k, [&](int t) { hits[t]++; });
      for (int t = 0; t < xcsum::STAGE_THREADS; t++)
        if (hits[t] != (t < k)) { printf("rep %d k %d part %d ran %d times\n", rep, k, t, hits[t]); return 1; }
      if (rep == 0 && pool.threads() != 1) { printf("threads %d after k=2\n", pool.threads()); return 1; }
    }
    printf("ok pool=%d\n", pool.threads());
    return 0;
  }
  xcsum::StagePool pool;
  const uint32_t n = (uint32_t)atoi(argv[1]);
  const uint32_t cap = (uint32_t)strtoul(argv[2], 0, 10);
  const uint32_t maxlen = (uint32_t)atoi(argv[3]);
  rng_state ^= (uint64_t)atoi(argv[4]);
  /* frames anywhere in a UMEM, random order, phases and lengths */
  const uint64_t umem_bytes = (uint64_t)n * (maxlen + 64) + 4096;
  std::vector<uint8_t> umem(umem_bytes);
  for (auto &b : umem) b = (uint8_t)rnd();
  std::vector<xcsum_desc> d(n), ds(n), ref_ds(n);
  for (uint32_t k = 0; k < n; k++) {
    d[k].len = (uint32_t)(rnd() % (maxlen + 1));
    d[k].addr = rnd() % (umem_bytes - d[k].len);
    d[k].options = 0;
  }
  /* serial restatement */
  uint64_t pos = 0, total = 0;
  for (uint32_t k = 0; k < n; k++) {
    const uint64_t len = d[k].len < cap ? d[k].len : cap;
    const uint64_t off = ((pos + 15) & ~(uint64_t)15) + (d[k].addr & 15);
    ref_ds[k] = xcsum_desc{off, d[k].len, 0};
    pos = off + len;
  }
  total = pos;
  std::vector<uint8_t> ref(total + 64, 0xa5), got(total + 64, 0xa5);
  for (uint32_t k = 0; k < n; k++)
    memcpy(ref.data() + ref_ds[k].addr, umem.data() + d[k].addr,
           d[k].len < cap ? d[k].len : cap);
  uint64_t r = 0;
  for (int rep = 0; rep < 3; rep++) {   /* the pool's threads serve every call */
    std::fill(got.begin(), got.end(), 0xa5);
    r = xcsum::gather_frames(&pool, got.data(), umem.data(), d.data(), ds.data(), n, cap);
    if (memcmp(ref.data(), got.data(), ref.size())) { printf("gathered bytes differ\n"); return 1; }
  }
  if (r != total) { printf("pos %llu != %llu\n", (unsigned long long)r, (unsigned long long)total); return 1; }
  for (uint32_t k = 0; k < n; k++)
    if (ds[k].addr != ref_ds[k].addr || ds[k].len != d[k].len || ds[k].options) {
      printf("desc %u\n", k); return 1;
    }
  if (memcmp(ref.data(), got.data(), ref.size())) { printf("gathered bytes differ\n"); return 1; }
  /* the range copy, at a size that splits (>= 4 MiB, not a page multiple) */
  const uint64_t m = umem_bytes - 4093 < (9u << 20) ? umem_bytes - 4093 : (9u << 20) + 77;
  std::vector<uint8_t> dst(m + 16, 0x3c);
  xcsum::stage_copy(&pool, dst.data(), umem.data() + 3, m);
  if (memcmp(dst.data(), umem.data() + 3, m) || dst[m] != 0x3c) { printf("range copy\n"); return 1; }
  xcsum::stage_copy(nullptr, dst.data(), umem.data() + 5, m);   /* no pool: serial */
  if (memcmp(dst.data(), umem.data() + 5, m)) { printf("serial range copy\n"); return 1; }
  printf("ok threads=%d pool=%d\n", xcsum::stage_threads(total, n), pool.threads());
  return 0;
}
'''


def build(tsan=False):
    d = tempfile.mkdtemp()
    src = os.path.join(d, "stage.cc")
    exe = os.path.join(d, "stage_tsan" if tsan else "stage")
    open(src, "w").write(DRIVER)
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "libxudp_amd", "csrc"), src, "-o", exe]
    if tsan:
        cmd.insert(1, "-fsanitize=thread")
    r = subprocess.run(cmd, capture_output=True, text=True)
    return exe if r.returncode == 0 else None


@pytest.fixture(scope="module")
def driver():
    exe = build()
    assert exe, "g++ failed on xcsum_stage.h"
    return exe


CASES = [  # frames, cap, max frame length, seed
    (1, 0xffffffff, 1514, 1), (100, 0xffffffff, 1514, 2), (100, 42, 1514, 3),
    (5000, 0xffffffff, 9000, 4), (20000, 42, 1514, 5), (20000, 0xffffffff, 200, 6),
    (70000, 42, 1514, 7), (70000, 0xffffffff, 1514, 8), (3000, 0xffffffff, 3, 9)]


@pytest.mark.parametrize("n,cap,maxlen,seed", CASES)
def test_gather_and_range_copy(driver, n, cap, maxlen, seed):
    r = subprocess.run([driver, str(n), str(cap), str(maxlen), str(seed)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    if n >= 16384 and _usable() >= 4:
        assert "threads=1 " not in r.stdout      # the split path ran
        assert "pool=0" not in r.stdout          # on the pool's threads


def _usable():
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return n


def test_budget_follows_affinity(driver):
    """the copy threads follow the caller's CPU budget, not the
    machine's CPU count: one CPU in the affinity mask (a libxudp TX worker
    pinned to a core) -> 1 thread; a wide mask -> STAGE_THREADS (4)."""
    import shutil
    if not shutil.which("taskset"):
        pytest.skip("no taskset")
    cpu = sorted(os.sched_getaffinity(0))[0]
    r = subprocess.run(["taskset", "-c", str(cpu), driver, "budget"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.split() == ["usable=1", "threads=1"], r.stdout
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) >= 3:
        r = subprocess.run(["taskset", "-c", ",".join(map(str, cpus[:3])), driver, "budget"],
                           capture_output=True, text=True, timeout=60)
        assert r.stdout.split() == ["usable=3", "threads=1"], r.stdout
    r = subprocess.run([driver, "budget"], capture_output=True, text=True, timeout=60)
    want = 4 if _usable() >= 8 else (_usable() // 2 if _usable() >= 4 else 1)
    assert r.stdout.split() == [f"usable={_usable()}", f"threads={want}"], r.stdout


def test_gather_threads_tsan_clean():
    exe = build(tsan=True)
    if exe is None:
        pytest.skip("no ThreadSanitizer runtime for g++ here")
    r = subprocess.run([exe, "70000", "42", "1514", "11"], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]


def test_pool_grows_between_calls(driver):
    """A pool started by a 2-part call grows on a 4-part one; the new workers
    take only the job posted after they start, every part runs once."""
    r = subprocess.run([driver, "grow"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.split() == ["ok", "pool=3"], r.stdout + r.stderr


def test_pool_growth_tsan_clean():
    exe = build(tsan=True)
    if exe is None:
        pytest.skip("no ThreadSanitizer runtime for g++ here")
    r = subprocess.run([exe, "grow"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
