#!/usr/bin/env python3
"""Headline benchmark: device-resident UDP checksum GiB/s (BASELINE.json metric).

A step = one xcsum_batch_device() launch over one batch of synthetic frames
already resident in HBM: by default BASELINE config 2, 1,048,576 x 1472-byte
UDP/IPv4 frames (1.6 GB), checksummed bit-exactly like xudp/checksum.h's
udp_checksum().  N>1: one process per GPU (torch.distributed.run), each rank
checksums its own batch (weak scaling, no collective on the data path; the
only collectives are the timing barrier and the max-over-ranks of the elapsed
time).

value    = algorithmic bytes of all ranks / max-over-ranks wall time, GiB/s
           (algorithmic bytes per frame = UDP length + pseudo-header address
           bytes + 2-byte result).  Timing: W eager warm-up
           launches, then >= --ramp-ms (300) of untimed back-to-back K-step
           bodies so the clocks reach their working point, then --reps (5)
           timed repetitions of exactly K steps, each bracketed by barrier +
           synchronize; the median repetition is reported (all are listed)
roofline = the checksum kernel's algorithmic bytes per launch / its average
           launch duration (HIP events on the launch stream), vs 8 TB/s HBM3E
cpu_baseline = the reference's own checksum.h (oracle/_ref, compiled from
           /root/reference in the build container) on a bounded sample of the
           same workload on this host's cores: 1, 16 and os.cpu_count()
           threads (rank 0, N=1 only)
parity   = the timed output's SHA-256 against the reference's digest of the
           same frames (config 5 at N>1: all ranks' shards concatenated), plus
           a 4096-frame spot check against the oracle

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import libxudp_amd as X  # noqa: E402

SEED_BASE = 0x78756470  # "xudp"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    2: dict(n=1 << 20, family=4, pmin=1472, pmax=1472, mode=X.MODE_V4_LEGACY, shard=False,
            name="1M x 1472B UDP/IPv4, device-resident (BASELINE config 2)"),
    3: dict(n=1 << 20, family=4, pmin=64, pmax=64, mode=X.MODE_V4_LEGACY, shard=False,
            name="1M x 64B UDP/IPv4, device-resident (BASELINE config 3)"),
    4: dict(n=1 << 20, family=6, pmin=1472, pmax=1472, mode=X.MODE_V6, shard=False,
            name="1M x 1472B UDP/IPv6, device-resident (BASELINE config 4)"),
    5: dict(n=8 << 20, family=4, pmin=64, pmax=9000, mode=X.MODE_V4_LEGACY, shard=True,
            name="8M x U[64,9000]B UDP/IPv4 sharded by bytes over the GPUs (BASELINE config 5)"),
}
MODE_NAMES = {0: "v4_legacy", 1: "v4_rfc", 2: "v6", 3: "auto"}
FLAG_NAMES = {"inplace": X.F_INPLACE, "iphdr": X.F_IPHDR, "rfc": X.F_V4_RFC, "verify": X.F_VERIFY,
              "iphdr_only": X.F_IPHDR_ONLY}


def parse_flags(text):
    """--flags inplace,iphdr -> XCSUM_F_* bits"""
    f = 0
    for w in filter(None, (t.strip() for t in text.split(","))):
        if w not in FLAG_NAMES:
            raise SystemExit(f"--flags: unknown flag {w!r} (known: {', '.join(FLAG_NAMES)})")
        f |= FLAG_NAMES[w]
    return f


def alg_bytes_flags(desc, family, flags, with_out):
    """Algorithmic bytes of one launch: the span read (UDP
    length + pseudo-header addresses), plus with XCSUM_F_IPHDR on IPv4 the 12
    header bytes before the addresses; writes: the 2-byte result when there
    is a result array, and every 2-byte check field written in place.
    XCSUM_F_IPHDR_ONLY: 20 header bytes read per frame, nothing else."""
    if flags & X.F_IPHDR_ONLY:
        # libxudp's IPv4 TX call: the 20-byte header read, iph->check written
        # (in place and/or into the result array); no payload byte
        inplace = (flags & X.F_INPLACE) and not (flags & X.F_VERIFY)
        return len(desc) * (20 + 2 * ((1 if with_out else 0) + (1 if inplace else 0)))
    span = X.alg_bytes(desc, family) - 2 * len(desc)
    v4 = family == 4
    read = span + (12 * len(desc) if (flags & X.F_IPHDR) and v4 else 0)
    inplace = (flags & X.F_INPLACE) and not (flags & X.F_VERIFY)
    fields = (1 if inplace else 0) + (1 if inplace and (flags & X.F_IPHDR) and v4 else 0)
    return read + 2 * len(desc) * ((1 if with_out else 0) + fields)


def reference_call(cfg, flags):
    """Which of the reference's computations a bench line times (VERDICT r4
    #2: a 'drop-in' number must be a call libxudp makes)."""
    v6 = cfg["family"] == 6
    inplace = flags & X.F_INPLACE and not flags & X.F_VERIFY
    if flags & X.F_VERIFY:
        return "receive-side verify (new: the reference never verifies, group/channel.c:231-255)"
    if flags & X.F_IPHDR_ONLY:
        return ("libxudp's IPv4 TX checksum: xudp_checksum_half (packet.c:43-66), udp->check "
                "left 0 (packet.c:125)" + (", stored in place" if inplace else ""))
    if v6:
        return ("libxudp's IPv6 TX checksum: udp_csum6 (packet.c:105-117)"
                + (", stored in place as packet.c:188 does" if inplace else ""))
    if cfg["mode"] == X.MODE_V4_RFC or flags & X.F_V4_RFC:
        return "IPv4 RFC 768 UDP checksum (an option; the reference leaves udp->check 0)"
    if inplace:
        return ("checksum.h udp_checksum stored into udp->check"
                + (" + iph->check" if flags & X.F_IPHDR else "")
                + ": not a call libxudp makes (it leaves the IPv4 udp->check 0, packet.c:125; "
                  "its IPv4 call is --flags inplace,iphdr_only)")
    return ("checksum.h udp_checksum (checksum.h:107-140, the BASELINE metric's function; no "
            "caller in the reference)" + (" + xudp_checksum_half" if flags & X.F_IPHDR else ""))


def elf_section(path, name):
    """Bytes of one section of an ELF64 little-endian file (None if absent)."""
    import struct
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        return None
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sect(i):
        # sh_name, sh_type, sh_flags, sh_addr, sh_offset, sh_size
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
    stroff = sect(shstrndx)[4]
    for i in range(shnum):
        nm, _, _, _, off, size = sect(i)
        end = data.index(b"\0", stroff + nm)
        if data[stroff + nm:end].decode() == name:
            return data[off:off + size]
    return None


def lib_sha16():
    """SHA-256 prefix of the loaded libxcsum.so's device code (its
    .hip_fatbin section, every gfx950 kernel).  Host-code edits (error-line
    numbers included) leave it unchanged; falls back to the whole file."""
    import hashlib
    sec = elf_section(X.LIB_PATH, ".hip_fatbin")
    if sec is None:
        with open(X.LIB_PATH, "rb") as f:
            sec = f.read()
    return hashlib.sha256(sec).hexdigest()[:16]


def _code_objects(sec):
    """The gfx950 code objects in a .hip_fatbin section: one clang offload
    bundle per translation unit ('__CLANG_OFFLOAD_BUNDLE__', entry count,
    then per entry: offset, size, triple length, triple)."""
    import struct
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    i = sec.find(magic)
    while i >= 0:
        n, = struct.unpack_from("<Q", sec, i + len(magic))
        p = i + len(magic) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", sec, p)
            triple = sec[p + 24:p + 24 + tlen]
            p += 24 + tlen
            if b"gfx950" in triple:
                yield sec[i + off:i + off + size]
        i = sec.find(magic, i + 1)


def _elf_symbol_bytes(co, want):
    """{symbol name: bytes} of the defined symbols of ELF code object `co`
    whose names satisfy want(name)."""
    import struct
    shoff, = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    sh = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + k * shentsize) for k in range(shnum)]
    out = {}
    for s_ in sh:
        if s_[1] != 2:                      # SHT_SYMTAB
            continue
        strtab = sh[s_[6]]                  # sh_link
        for e in range(s_[5] // 24):
            nm, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, s_[4] + 24 * e)
            if not shndx or shndx >= shnum or not size:
                continue
            name = co[strtab[4] + nm:co.index(b"\0", strtab[4] + nm)].decode()
            if want(name):
                sec_ = sh[shndx]
                o = sec_[4] + (value - sec_[3])
                out[name] = co[o:o + size]
    return out


def kernel_sha16(demangled):
    """SHA-256 prefix of ONE kernel's gfx950 machine code and kernel
    descriptor in the loaded libxcsum.so, named as rocprofv3 names it (e.g.
    'void xcsum::csum_kernel<16, 2, 6, 0>(xcsum::CsumArgs)').  Ties PMC
    counters to the kernel that was measured: other kernels, host code and
    new translation units leave it unchanged.  None if not found."""
    import hashlib
    import re
    m = re.search(r"xcsum::(\w+)<([^>]*)>", demangled or "")
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    mangled = (f"{len(m.group(1))}{m.group(1)}I" + "".join(f"Li{a}E" for a in args) + "E")
    sec = elf_section(X.LIB_PATH, ".hip_fatbin")
    if sec is None:
        return None
    for co in _code_objects(sec):
        syms = _elf_symbol_bytes(co, lambda n: mangled in n)
        if syms:
            h = hashlib.sha256()
            for k in sorted(syms):          # the function and its .kd
                h.update(k.encode() + b"\0" + syms[k])
            return h.hexdigest()[:16]
    return None


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def launch_plan(gpus, environ):
    """What `bench.py --gpus N` does with the environment it was started in:
    "launch" -- N > 1 and no WORLD_SIZE: this process starts the N rank
    processes itself (launch_ranks) and only relays their exit code;
    "run" -- it is one rank (WORLD_SIZE from torch.distributed.run or from
    launch_ranks, or N = 1 without one).  A WORLD_SIZE that disagrees with
    --gpus is an error: the line would otherwise report a GPU count nobody
    asked for.  Returns ("launch"|"run", message or None)."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: need at least one GPU"
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return ("launch", None) if gpus > 1 else ("run", None)
    try:
        world = int(ws)
    except ValueError:
        return "error", f"WORLD_SIZE={ws!r} is not a number"
    if world != gpus:
        return "error", (f"WORLD_SIZE={world} but --gpus {gpus}: run `bench.py --gpus {gpus}` "
                         f"bare (it starts its own ranks) or under torch.distributed.run with "
                         f"--nproc-per-node {gpus}")
    return "run", None


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(environ, rank, world, port):
    """Environment of rank `rank` of a launch_ranks job: the variables
    torch.distributed.run sets (one node, LOCAL_RANK = RANK = the GPU index)."""
    env = dict(environ)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", ROLE_RANK=str(rank),
               ROLE_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               TORCHELASTIC_RUN_ID="bench")
    # dmabuf IPC only on this pool (RCCL's peer mappings)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def launch_ranks(world, argv, grace_s=30.0, script=None):
    """Start `world` rank processes of this script (the same arguments, one
    per GPU, LOCAL_RANK = GPU) and wait for them.  The parent never imports
    torch nor touches a GPU, and it starts children rather than replacing
    itself.  Rank 0 writes the JSON line to the inherited stdout; the other
    ranks' stdout goes to stderr.  When a rank fails, the rest get `grace_s`
    to finish (they would block in the next barrier) and are then killed; a
    SIGTERM/SIGINT to the parent is passed on.  Returns the exit code: 0 if
    every rank exited 0, else the first failing rank's code (or 1)."""
    import signal
    import subprocess
    port = free_port()
    script = script or os.path.abspath(__file__)

    def die_with_parent():
        # in the child, before it runs anything: a parent killed outright
        # (SIGKILL from a time limit) takes its ranks with it
        try:
            import ctypes
            ctypes.CDLL(None).prctl(1, signal.SIGKILL)   # PR_SET_PDEATHSIG
        except (OSError, AttributeError):
            pass
    procs = []
    try:
        for r in range(world):
            procs.append(subprocess.Popen([sys.executable, "-u", script, *argv],
                                          env=rank_env(os.environ, r, world, port),
                                          stdout=None if r == 0 else sys.stderr.fileno(),
                                          preexec_fn=die_with_parent))
    except OSError as e:
        # the ranks already started would wait for the missing one at the
        # rendezvous: end them
        print(f"bench: could not start rank {len(procs)}: {e}", file=sys.stderr)
        for p in procs:
            p.kill()
            p.wait()
        return 1

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    rc, failed_at = 0, None
    try:
        live = set(range(world))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 1
                    failed_at = time.monotonic()
                    print(f"bench: rank {r} exited with {c}", file=sys.stderr)
            if live and failed_at is not None and time.monotonic() - failed_at > grace_s:
                for r in live:
                    procs[r].kill()
                    print(f"bench: rank {r} killed after rank failure", file=sys.stderr)
                for r in live:
                    procs[r].wait()
                break
            time.sleep(0.05)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def rank_slice(cfg, rank, world):
    """(first global frame index, frame count) owned by `rank`.  Config 5 is
    one 8M-frame job split by bytes over the ranks (strong scaling); the others
    give every rank its own full batch (weak scaling).  No data-path
    collective: a frame's checksum depends on that frame only."""
    n = cfg["n"]
    if cfg["shard"]:
        full, _ = X.gen_layout(n, cfg["family"], cfg["pmin"], cfg["pmax"],
                               seed=SEED_BASE ^ cfg["id"])
        return X.shard_by_bytes(full, world, rank)
    return rank * n, n


def h2d(torch, arr, dev):
    """Host array -> device tensor through torch's pinned host memory: the HIP
    runtime pins pageable buffers of >= 1 MiB in place for a copy, and numpy's
    large arrays are backed by transparent huge pages -- the combination
    DESIGN.md 6 traces the registered-memory faults to."""
    return torch.from_numpy(np.ascontiguousarray(arr)).pin_memory().to(dev)


def d2h(torch, t):
    """Device tensor -> numpy array in pinned host memory (see h2d)."""
    if t.device.type == "cpu":
        return t.numpy().copy()
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


def build_batch(cfg, rank, world, torch, dev, eng, stream, flags=0):
    """Descriptors + frames for this rank, generated on the device."""
    seed = SEED_BASE ^ cfg["id"]
    first, count = rank_slice(cfg, rank, world)
    if cfg.get("layout") == "umem":
        # xudp's own TX layout: one frame per 4096-byte chunk, eth at F+342
        # (IPv4) / F+322 (IPv6), SURVEY a14
        off = 322 if cfg["family"] == 6 else 342
        desc, nbytes = X.gen_layout(count, cfg["family"], cfg["pmin"], cfg["pmax"], seed=seed,
                                    first_index=first, stride=4096, offset=off)
    else:
        desc, nbytes = X.gen_layout(count, cfg["family"], cfg["pmin"], cfg["pmax"], seed=seed,
                                    first_index=first)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    # rotate buffers so each pass streams >= 1 GiB: nothing is served from the
    # 256 MiB Infinity Cache (SURVEY.md 7 hard part iv).  XCSUM_F_IPHDR_ONLY
    # touches only the header lines (~120-160 MB of a config-2 batch, which
    # would stay in the Infinity Cache between launches): rotate by those
    touched = real_bytes(desc, flags) if flags & X.F_IPHDR_ONLY else nbytes
    nrot = max(1, math.ceil((1 << 30) / max(touched, 1)))
    bufs = [torch.empty(nbytes + 64, dtype=torch.uint8, device=dev) for _ in range(nrot)]
    eng.gen_fill_device(bufs[0], d_desc, count, cfg["family"], seed, first, stream=stream)
    for b in bufs[1:]:
        b.copy_(bufs[0])
    out = torch.empty(max(count, 1), dtype=torch.int16, device=dev)
    torch.cuda.synchronize(dev)
    return desc, d_desc, bufs, out, first, count


def host_cpu_facts():
    """CPUs this process may use: affinity mask and cgroup v2 quota (on the GPU
    box os.cpu_count() is the whole machine, not this job's share)."""
    facts = {"host_cpus": os.cpu_count()}
    try:
        facts["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        facts["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            facts["cpu_model"] = next((ln.split(":", 1)[1].strip() for ln in f
                                       if ln.startswith("model name")), "")
    except OSError:
        pass
    return facts


def cpu_baseline(cfg, seconds=15.0, flags=0):
    """The reference checksum.h timed on this host over a bounded sample:
    1 thread, 16 threads and os.cpu_count() threads (static frame partition).
    Each leg first runs one untimed repetition (thread creation, caches), then
    one timed repetition sizes the leg to its share of `seconds`.  With
    XCSUM_F_IPHDR_ONLY: the reference's xudp_checksum_half (packet.c:43-66,
    ref_batch mode 4), 22 algorithmic bytes per frame as on the GPU."""
    import oracle  # test infrastructure, used here only as the CPU baseline
    seed = SEED_BASE ^ cfg["id"]
    m = min(cfg["n"], 1 << 16)
    umem, desc = X.gen_frames_host(m, cfg["family"], cfg["pmin"], cfg["pmax"], seed=seed)
    out = np.zeros(m, dtype=np.uint16)
    hdr_only = bool(flags & X.F_IPHDR_ONLY)
    alg = 22 * m if hdr_only else X.alg_bytes(desc, cfg["family"])
    mode = 4 if hdr_only else 2 if cfg["family"] == 6 else 0
    if oracle.have_ref():
        kind, L = "reference", oracle.ref()
        timed = lambda th, reps: L.ref_batch_timed(umem.ctypes.data, desc.ctypes.data, m,
                                                   out.ctypes.data, mode, th, reps)
    else:
        kind, L = "port", oracle.port()
        pmode, pflags = (0, X.F_IPHDR_ONLY) if hdr_only else (mode, 0)
        timed = lambda th, reps: L.orc_batch_timed(umem.ctypes.data, desc.ctypes.data, m,
                                                   out.ctypes.data, pmode, pflags, th, reps)
    facts = host_cpu_facts()
    usable = min(v for v in (facts.get("affinity_cpus"), facts.get("cgroup_cpu_quota"),
                             facts.get("host_cpus")) if v)
    facts["cores_usable"] = usable
    allc = max(1, min(256, os.cpu_count() or 1))
    legs = [(1, 0.3), (min(16, allc), 0.35)]
    if allc > 16:
        legs.append((allc, 0.35))
    res, secs = {}, {}
    t_start = time.perf_counter()
    for th, share in legs:
        # warm (threads, page faults, caches), then grow the repetition count
        # until one timed run fills the leg's share: sizing from a single short
        # run undershot by 10x on the box (thread start-up, cgroup quota)
        timed(th, 1)
        target = seconds * share
        reps, t = 1, timed(th, 1)
        while t < 0.8 * target and reps < (1 << 24):
            reps = max(reps + 1, int(reps * target / max(t, 1e-4)) if t >= 0.05 else reps * 10)
            t = timed(th, reps)
        res[th] = alg * reps / t / 2**30
        secs[th] = round(t, 3)
    total = time.perf_counter() - t_start
    if kind == "reference":
        exp = oracle.ref_batch(umem, desc, mode)
    else:
        exp = oracle.batch(umem, desc, 0 if hdr_only else mode, X.F_IPHDR_ONLY if hdr_only else 0)
    assert np.array_equal(out, exp)
    best_th = max(res, key=lambda k: res[k])
    legs_txt = ", ".join(f"{th} thread{'s' if th > 1 else ''} {secs[th]:.1f} s"
                         for th, _ in legs)
    return {"value": round(res[best_th], 3), "unit": "GiB/s", "cores": best_th, "kind": kind,
            "by_threads": {str(k): round(v, 3) for k, v in sorted(res.items())},
            "seconds_by_threads": {str(k): v for k, v in sorted(secs.items())},
            "seconds_total": round(total, 2),
            "value_1core": round(res[1], 3), **facts,
            "sample": f"{m} frames of the same config ({alg / 1e6:.1f} MB algorithmic), "
                      f"xudp/{'packet.c xudp_checksum_half' if hdr_only else 'checksum.h udp_csum6' if mode == 2 else 'checksum.h udp_checksum'} compiled "
                      f"-O2 from the reference, static frame partition; timed legs: {legs_txt} "
                      f"({total:.1f} s in all with the warm-up and sizing runs); "
                      f"{usable:g} CPUs usable by this job (affinity / cgroup quota), so "
                      f"thread counts above that time-slice; value = the fastest leg"}


def pmc_traffic(cid, layout, flags, sha):
    """HBM bytes per launch from the rocprofv3 PMC summary committed under
    profiles/ (FETCH_SIZE + WRITE_SIZE passes of this bench, tools/pmc_summary.py);
    counters cannot be read inside the timed process itself.  Only counters
    taken on this very kernel are reported: the summary records the kernel
    rocprofv3 measured and the SHA-256 prefix of its machine code
    (kernel_sha16), which must equal the loaded library's; older summaries
    without it are matched on the whole device code (lib_sha16).  Otherwise
    traffic is null and the reason says which code the counters came from.
    Returns (bytes, source, reason, kernel hash)."""
    tag = f"{'_umem' if layout == 'umem' else ''}{'_f%x' % flags if flags else ''}"
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01", ""):
        path = os.path.join(ROOT, "profiles", rnd, f"pmc_config{cid}{tag}.json")
        if not os.path.exists(path):
            continue
        try:
            j = json.load(open(path))
        except Exception:
            continue
        src = os.path.relpath(path, ROOT)
        if j.get("kernel_sha16"):
            kern = (j.get("kernel") or [None])[0]
            mine = kernel_sha16(kern)
            if mine != j["kernel_sha16"]:
                return None, src, (f"counters in {src} were taken on {kern} with code "
                                   f"{j['kernel_sha16']}, this build's is {mine}"), mine
            return j.get("hbm_bytes_per_launch"), src, None, mine
        if j.get("lib_sha16") != sha:
            return None, src, (f"counters in {src} were taken on libxcsum.so "
                               f"{j.get('lib_sha16') or '(unrecorded)'}, not this build {sha}"), None
        return j.get("hbm_bytes_per_launch"), src, None, None
    return None, None, "no PMC summary for this workload under profiles/", None


def gpu_clocks(dev):
    """Current SCLK / MCLK of this GPU from sysfs (the '*' level of
    pp_dpm_sclk / pp_dpm_mclk), or None where not readable."""
    try:
        import torch
        p = torch.cuda.get_device_properties(dev)
        path = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:" \
               f"{p.pci_device_id:02x}.0"
        res = {}
        for k in ("sclk", "mclk", "fclk"):
            try:
                for ln in open(os.path.join(path, f"pp_dpm_{k}")):
                    if "*" in ln:
                        res[k] = ln.split(":", 1)[1].replace("*", "").strip()
            except OSError:
                pass
        return res or None
    except Exception:
        return None


def real_bytes(desc, flags=0):
    """HBM bytes a launch cannot avoid: the union of the 64-byte lines the
    frames touch, plus the 16-byte descriptor and the 2-byte result of every
    frame.  XCSUM_F_IPHDR_ONLY touches only the lines of the IPv4 header
    [eth+14, eth+34)."""
    if len(desc) == 0:
        return 0
    a = desc["addr"].astype(np.int64)
    if flags & X.F_IPHDR_ONLY:
        lo = (a + 14) // 64
        hi = (a + 34 + 63) // 64
    else:
        lo = a // 64
        hi = (a + desc["len"].astype(np.int64) + 63) // 64
    order = np.argsort(lo, kind="stable")
    lo, hi = lo[order], hi[order]
    reach = np.maximum.accumulate(hi)
    start = np.maximum(lo, np.concatenate([[lo[0]], reach[:-1]]))
    lines = int(np.maximum(hi - start, 0).sum())
    return lines * 64 + 18 * len(desc)


def stream_ceiling(torch, dev, bufs, sptr):
    """Same-run streaming-read ceiling over the very buffers the checksum
    kernel reads, rotated the same way: the fastest of tools/libhbmprobe.so's
    dwordx4 grid-stride read (8 blocks/CU, nontemporal; the best setting of
    tools/hbm_probe.py) and its wave-contiguous reads (round 6,
    tools/read_shapes.py: each wave streams its own 8 KiB / 128 KiB region, 8
    / 16 loads of 1 KiB in flight, 1 block/CU, nontemporal -- up to 3.5 %
    faster than the grid stride).  A measuring stick, not the product."""
    path = os.path.join(ROOT, "tools", "libhbmprobe.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    region = getattr(L, "probe_wave_region_read", None)
    if region is not None:
        region.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    scratch = torch.empty(cus * 8 * 256, dtype=torch.int32, device=dev)
    nbytes = (bufs[0].numel() - 64) & ~15
    legs = {"grid_stride_8bpc": lambda buf: L.probe_stream_read(
        buf.data_ptr(), nbytes, scratch.data_ptr(), cus * 8, 1, 1, sptr)}
    if region is not None:
        legs["wave_region_8k_u8_1bpc"] = lambda buf: region(
            buf.data_ptr(), nbytes, 8 << 10, cus, 1, 8, scratch.data_ptr(), sptr)
        legs["wave_region_128k_u16_1bpc"] = lambda buf: region(
            buf.data_ptr(), nbytes, 128 << 10, cus, 1, 16, scratch.data_ptr(), sptr)
    # back-to-back launches between two events, as the checksum launches
    # are timed (K per replay): per-launch events would add the launch gap to
    # every short kernel and understate the ceiling
    per = max(10, len(bufs))
    s = torch.cuda.current_stream(dev)
    ms = {}
    for name, fn in legs.items():
        ts = []
        for r in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for k in range(per):
                if fn(bufs[k % len(bufs)]) != 0:
                    return None
            b.record(s)
            torch.cuda.synchronize(dev)
            ts.append(a.elapsed_time(b) / per)
        ms[name] = float(np.median(ts[1:]))
    best = min(ms, key=ms.get)
    t = ms[best]
    return {"GBps": round(nbytes / (t * 1e-3) / 1e9, 1), "fastest": best,
            "GBps_by_leg": {k: round(nbytes / (v * 1e-3) / 1e9, 1) for k, v in ms.items()},
            "what": f"stream read of the same {nbytes / 1e9:.3f} GB frame buffer"
                    f"{'s' if len(bufs) > 1 else ''} (real bytes, headers and padding "
                    f"included), tools/hbm_probe.hip: the fastest of a grid-stride read and "
                    f"two wave-contiguous reads, {per} back-to-back launches between two events, "
                    f"median of 5"}


def span_ceiling(torch, dev, bufs, d_desc, desc, sptr, real):
    """Like-for-like ceiling of the frame-per-wave access pattern (VERDICT r5
    #3, #6): tools/libhbmprobe.so's probe_frame_spans2 reads what the
    checksum kernel must fetch -- per frame its descriptor and the 128-byte
    lines (or the 16-byte chunks) around its span -- with no arithmetic, one
    wave per frame (64 x 16 B per load instruction), 4 MTU or 2 jumbo frames
    per wave in flight, the frames in one of the kernel's visiting orders (32
    regions of 16-frame tiles: sparse; 8 of 16: MTU; 16 of 4: mixed sizes;
    descriptor order), plain or nontemporal loads; the fastest leg counts.
    For xudp's slots (--layout umem) and for mixed sizes (config 5) the
    contiguous stream read of the whole buffer is not that pattern.  Rates
    over the same real bytes as roofline.real_achieved.  None where the probe
    is missing or a frame's span exceeds 10 KiB."""
    path = os.path.join(ROOT, "tools", "libhbmprobe.so")
    if not os.path.exists(path) or not len(desc):
        return None
    L = ctypes.CDLL(path)
    fn = getattr(L, "probe_frame_spans2", None)
    if fn is None:
        return None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                   ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_void_p]
    a = desc["addr"].astype(np.int64)
    end = a + desc["len"].astype(np.int64)
    max_span = int((((end + 127) & ~127) - (a & ~127)).max())
    if max_span > 10240:
        return None
    # host-side bounds: every line the probe may load lies inside the buffer
    assert int(((end + 127) & ~127).max()) <= bufs[0].numel()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    blocks = cus * (8 if max_span <= 2048 else 4)
    scratch = torch.empty(blocks, dtype=torch.int32, device=dev)
    per = max(10, len(bufs)) if max_span <= 2048 else 4
    s = torch.cuda.current_stream(dev)
    legs = {}
    for rlog, tlog in ((5, 4), (3, 4), (4, 2), (0, 0)):
        for line in (128, 16):
            for nt in (0, 1):
                ts = []
                for r in range(6):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for k in range(per):
                        if fn(bufs[k % len(bufs)].data_ptr(), d_desc.data_ptr(), len(desc), rlog,
                              tlog, line, nt, max_span, scratch.data_ptr(), blocks, sptr) != 0:
                            return None
                    e1.record(s)
                    torch.cuda.synchronize(dev)
                    ts.append(e0.elapsed_time(e1) / per)
                legs[f"order_{rlog}_{tlog}_line{line}{'_nt' if nt else ''}"] = \
                    float(np.median(ts[1:]))
    best = min(legs, key=legs.get)
    t = legs[best]
    return {"ms": round(t, 4), "ms_by_leg": {k: round(v, 4) for k, v in legs.items()},
            "fastest": best, "GBps": round(real / (t * 1e-3) / 1e9, 1),
            "what": "tools/hbm_probe.hip probe_frame_spans2: per frame the 16-byte descriptor "
                    "and the 128-byte lines (or 16-byte chunks) around its span, no arithmetic, "
                    "one wave per frame, 4 MTU / 2 jumbo frames per wave in flight, in one of "
                    "the kernel's visiting orders (regions R,T) or descriptor order, plain or "
                    "nontemporal loads; the fastest leg; rate over the same real bytes as "
                    f"real_achieved; {per} back-to-back launches between two events, median "
                    "of 5"}


def inplace_ceiling(torch, dev, bufs, desc, flags, family, sptr):
    """Same-run ceiling of the in-place pass: tools/libhbmprobe.so's stream
    read of the same buffers plus one 2-byte store per frame into its
    udp->check (and iph->check with IPHDR) field, from the thread that read
    the chunk holding it (probe_stream_read_inplace).  Frames must sit at a
    fixed stride (the bench's layouts do).  Writes garbage into the check
    fields: run it after timing, before the parity pass regenerates the
    frames."""
    path = os.path.join(ROOT, "tools", "libhbmprobe.so")
    a = desc["addr"].astype(np.int64)
    if not os.path.exists(path) or len(a) < 2:
        return None
    fstride = int(a[1] - a[0])
    if fstride <= 0 or not np.all(np.diff(a) == fstride):
        return None
    L = ctypes.CDLL(path)
    fn = L.probe_stream_read_inplace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                   ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    f1 = 60 if family == 6 else 40
    f2 = 24 if (flags & X.F_IPHDR) and family == 4 else f1
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    blocks = cus * 8
    scratch = torch.empty(blocks * 256, dtype=torch.int32, device=dev)
    nbytes = (bufs[0].numel() - 64) & ~15
    per = max(10, len(bufs))
    s = torch.cuda.current_stream(dev)
    by_unroll = {}
    for unroll in (1, 4):           # 1 or 4 chunks in flight per thread, the faster counts
        ts = []
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for k in range(per):
                if fn(bufs[k % len(bufs)].data_ptr(), nbytes, fstride, int(a[0]), len(a), f1, f2,
                      scratch.data_ptr(), blocks, unroll, sptr) != 0:
                    return None
            e1.record(s)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / per)
        by_unroll[unroll] = float(np.median(ts[1:]))
    # the two-pass schedule's probe: the plain read, then the field stores in
    # frame order (probe_stream_read_twopass), both launches between the events
    two = getattr(L, "probe_stream_read_twopass", None)
    if two is not None:
        two.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                        ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                        ctypes.c_int, ctypes.c_void_p]
        ts = []
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for k in range(per):
                if two(bufs[k % len(bufs)].data_ptr(), nbytes, fstride, int(a[0]), len(a), f1, f2,
                       scratch.data_ptr(), blocks, sptr) != 0:
                    return None
            e1.record(s)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / per)
        by_unroll["two_pass"] = float(np.median(ts[1:]))
    t = min(by_unroll.values())
    return {"ms": round(t, 4), "ms_by_unroll": {str(k): round(v, 4) for k, v in by_unroll.items()},
            "GBps_read": round(nbytes / (t * 1e-3) / 1e9, 1),
            "what": f"stream read of the same {nbytes / 1e9:.3f} GB buffer"
                    f"{'s' if len(bufs) > 1 else ''} + a 2-byte store per frame at eth+{f1}"
                    f"{f' and eth+{f2}' if f2 != f1 else ''} from the thread that read it "
                    f"(tools/hbm_probe.hip probe_stream_read_inplace, 1 or 4 chunks in flight "
                    f"per thread), or the stream read followed by a launch storing the fields "
                    f"in frame order (probe_stream_read_twopass); the fastest of the three, "
                    f"{per} back-to-back launches between two events, median of 5"}


def header_ceiling(torch, dev, bufs, d_desc, count, write, sptr):
    """Same-run ceiling of the XCSUM_F_IPHDR_ONLY call: tools/libhbmprobe.so's
    probe_header_touch over the very frames and descriptors -- per frame the
    descriptor, the seven header dwords the kernel loads and, in place, a
    2-byte store at eth+24 -- with none of the kernel's arithmetic.  One
    scattered line read (+ one partial write) per frame is an access pattern
    whose bound is the memory system's transaction rate, not the stream
    rate.  Writes junk into iph->check: run it after timing, before the
    parity pass regenerates the frames."""
    path = os.path.join(ROOT, "tools", "libhbmprobe.so")
    if not os.path.exists(path) or not count:
        return None
    L = ctypes.CDLL(path)
    fn = getattr(L, "probe_header_touch", None)
    if fn is None:
        return None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p]
    scratch = torch.empty(max(1, (count + 1023) // 1024), dtype=torch.int32, device=dev)
    per = max(20, len(bufs))
    s = torch.cuda.current_stream(dev)
    ts = []
    for r in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for k in range(per):
            if fn(bufs[k % len(bufs)].data_ptr(), d_desc.data_ptr(), count, int(write),
                  scratch.data_ptr(), sptr) != 0:
                return None
        e1.record(s)
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1) / per)
    t = float(np.median(ts[1:]))
    return {"ms": round(t, 5),
            "what": f"tools/hbm_probe.hip probe_header_touch over the same frames: per frame the "
                    f"16-byte descriptor and the 28 bytes at (eth+12)&~3"
                    f"{' plus a 2-byte store at eth+24' if write else ''}, no arithmetic; "
                    f"{per} back-to-back launches between two events, median of 5"}


# Visiting orders the same-run A/B times next to the automatic one
# (xcsum_ctx_set_order "R,T": 2^R regions of 2^T-frame tiles; 0,0 = descriptor
# order).  The automatic order of MTU frames is 3,4.
ORDER_AB = [(0, 0), (3, 4), (4, 4), (2, 5)]


def order_ab(torch, dev, eng, bufs, d_desc, count, out_arg, cfg, flags, len_hint, sptr,
             real, ceiling_gbps, calibrated=None, per=10, reps=6):
    """Same-run A/B of dense visiting orders on the timed workload: for each
    order in ORDER_AB and the automatic one, `per` back-to-back eager launches
    between two events, median of `reps` - 1 (the first is a warm-up); the
    per-launch time and its fraction of the same-run stream-read ceiling (real
    bytes, as roofline.frac_vs_ceiling).  `calibrated`: the order
    xcsum_ctx_calibrate_order picked for the timed run, (-1, 0) = automatic;
    a forced pick outside ORDER_AB gets its own leg, and the line says which
    leg the timed run used.  Leaves the timed run's order set."""
    s = torch.cuda.current_stream(dev)
    best_ms = {}
    legs = [None] + ORDER_AB
    if calibrated not in (None, (-1, 0)) and tuple(calibrated) not in ORDER_AB:
        legs.append(tuple(calibrated))
    # two rounds with the legs interleaved, the lower median of each leg:
    # the first leg measured after the ceiling probe ran ~10 % slow once
    for rnd in range(2):
        for order in legs:
            if order is None:
                eng.set_order(-1, 0)
            else:
                eng.set_order(*order)
            ts = []
            for r in range(reps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(per):
                    eng.batch_device(bufs[k % len(bufs)], d_desc, count, out_arg, cfg["mode"],
                                     flags, len_hint, stream=sptr)
                e1.record(s)
                torch.cuda.synchronize(dev)
                ts.append(e0.elapsed_time(e1) / per)
            key = "auto" if order is None else f"{order[0]},{order[1]}"
            best_ms[key] = min(best_ms.get(key, 1e9), float(np.median(ts[1:])))
    res = {}
    for key, ms in best_ms.items():
        res[key] = {"ms": round(ms, 4)}
        if ceiling_gbps:
            res[key]["frac_vs_ceiling"] = round(real / (ms * 1e-3) / 1e9 / ceiling_gbps, 4)
    timed_leg = "auto" if calibrated in (None, (-1, 0)) else f"{calibrated[0]},{calibrated[1]}"
    if timed_leg == "auto":
        eng.set_order(-1, 0)
    else:
        eng.set_order(*calibrated)
    best = min(res, key=lambda k: res[k]["ms"])
    return {"orders": res, "fastest": best, "timed_run_order": timed_leg,
            "auto_vs_fastest": round(res[best]["ms"] / res["auto"]["ms"], 4),
            "timed_vs_fastest": round(res[best]["ms"] / res[timed_leg]["ms"], 4),
            "what": f"{per} back-to-back eager launches per order between two events, median "
                    f"of {reps - 1}, the lower of two interleaved rounds; R,T = 2^R regions of "
                    f"2^T-frame tiles (0,0 = descriptor order), auto = the library's choice"}


def parse_shard(text):
    """--shard r/N -> (r, N), or None for ''."""
    if not text:
        return None
    try:
        r, n = (int(v) for v in text.split("/"))
    except ValueError:
        raise SystemExit(f"--shard {text!r}: expected r/N, e.g. 0/8")
    if not (n >= 1 and 0 <= r < n):
        raise SystemExit(f"--shard {text!r}: need 0 <= r < N")
    return r, n


def digest_check(cfg, out, count, world, rank, dist, sdev, field="sha256_out", shard=None):
    """SHA-256 of the timed output against the digest the REFERENCE produced
    over the same synthetic frames (tests/golden/digests.json, made by
    tests/golden/make_golden.py with the compiled checksum.h).  Config 5 is
    one job sharded by bytes: every rank's output is gathered to rank 0 and
    the concatenation must equal the single-job digest.  Weak-scaling configs
    give rank r frames r*n..: rank 0's batch is the digested one.  `shard`
    (r, N): one process timing shard r of N alone (--shard) -- its output
    against the reference's digest of exactly that shard
    (sha256_out_shards{N}[r])."""
    import hashlib
    path = os.path.join(ROOT, "tests", "golden", "digests.json")
    key = f"config{cfg['id']}"
    if not os.path.exists(path):
        return None
    rec = json.load(open(path)).get(key, {})
    import torch
    mine = out[:count].view(torch.uint8) if count else out[:0].view(torch.uint8)
    if shard is not None and cfg["shard"]:
        if field != "sha256_out":
            return None
        want = (rec.get(f"sha256_out_shards{shard[1]}") or [None] * shard[1])[shard[0]]
        if not want:
            return None
        return {"ok": hashlib.sha256(d2h(torch, mine).tobytes()).hexdigest() == want,
                "what": f"{key} sha256_out_shards{shard[1]}[{shard[0]}] over this shard's "
                        f"timed output"}
    want = rec.get(field)
    if not want:
        return None
    if cfg["shard"] and dist.is_initialized():
        cnt = torch.tensor([count], dtype=torch.int64, device=sdev)
        cnts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(cnts, cnt)
        cmax = max(int(c) for c in cnts)
        pad = torch.zeros(2 * cmax, dtype=torch.uint8, device=sdev)
        pad[:2 * count] = mine.to(sdev)
        parts = [torch.zeros_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
        if rank != 0:
            return None
        blob = b"".join(d2h(torch, p[:2 * int(c)]).tobytes() for p, c in zip(parts, cnts))
        what = f"{key} {field} over the concatenated outputs of {world} ranks"
    else:
        if rank != 0:
            return None
        blob = d2h(torch, mine).tobytes()
        what = f"{key} {field} over rank 0's timed output"
    return {"ok": hashlib.sha256(blob).hexdigest() == want, "what": what}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--geometry", default="", help="G,U,K override (tuning)")
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"],
                    help="frames packed at 8-byte boundaries (default) or one per 4096-byte "
                         "chunk as in xudp's TX UMEM")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches")
    ap.add_argument("--dist-init", action="store_true",
                    help="form the process group and run every collective even at one rank "
                         "(exercises the RCCL branch on a one-GPU box)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process group for the barrier / timing reductions (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (1-GPU box)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--reps", type=int, default=5,
                    help="timed repetitions of the K steps (the median is reported)")
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed back-to-back K-step bodies before timing (clock ramp)")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the same-run streaming-read ceiling probe")
    ap.add_argument("--no-calibrate", dest="calibrate", action="store_false",
                    help="keep the automatic visiting order (no xcsum_ctx_calibrate_order)")
    ap.add_argument("--no-order-ab", dest="order_ab", action="store_false",
                    help="skip the same-run A/B of dense visiting orders (configs 2 and 4)")
    ap.add_argument("--inplace-schedule", default="auto", choices=["auto", "fused", "two_pass"],
                    help="how --flags inplace writes the check fields (xcsum_ctx_set_inplace)")
    ap.add_argument("--flags", default="",
                    help="comma list of inplace,iphdr,rfc,verify,iphdr_only (XCSUM_F_*); with "
                         "inplace the checks go into the frames and no result array is written, "
                         "as libxudp's TX path does (tx.c:696-726); libxudp's IPv4 call is "
                         "inplace,iphdr_only (iph->check only), its IPv6 call inplace on config 4")
    ap.add_argument("--shard", default="",
                    help="r/N: one process times shard r of N of a sharded config (config 5) "
                         "alone -- one rank's share of the N-GPU job -- with the full roofline "
                         "and that shard's reference digest")
    args = ap.parse_args()
    flags = parse_flags(args.flags)
    shard = parse_shard(args.shard)
    # in place: the check fields go into the frames, no result array
    with_out = not (flags & X.F_INPLACE) or bool(flags & X.F_VERIFY)

    # N > 1 without a launcher: start the N ranks here, before torch or any
    # GPU call (a bare `bench.py --gpus 8` ran one rank)
    plan, msg = launch_plan(args.gpus, os.environ)
    if plan == "error":
        print(f"bench: {msg}", file=sys.stderr)
        sys.exit(2)
    if plan == "launch":
        if shard is not None:
            print("bench: --shard times one shard in one process; use --gpus 1", file=sys.stderr)
            sys.exit(2)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world, rank, local = dist_env()
    if shard is not None and (world != 1 or not CONFIGS[args.config]["shard"]):
        print("bench: --shard needs --gpus 1 and a sharded config (5)", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()
    if not args.same_device and local >= ndev:
        print(f"bench: rank {rank} wants cuda:{local} but {ndev} GPU(s) are visible "
              f"(--same-device rehearses N ranks on one GPU)", file=sys.stderr)
        sys.exit(2)
    dev = torch.device(f"cuda:{0 if args.same_device else local}")
    torch.cuda.set_device(dev)
    use_dist = world > 1 or args.dist_init
    if use_dist:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    def barrier():
        if use_dist:
            dist.barrier()

    cfg = dict(CONFIGS[args.config], id=args.config, layout=args.layout)
    eng = X.Engine(dev.index)
    if args.geometry:
        eng.set_geometry(*[int(v) for v in args.geometry.split(",")])
    eng.set_inplace({"auto": X.INPLACE_AUTO, "fused": X.INPLACE_FUSED,
                     "two_pass": X.INPLACE_TWO_PASS}[args.inplace_schedule])
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    # --shard r/N: this process's batch is shard r of the N-way split
    srank, sworld = shard if shard is not None else (rank, world)
    desc, d_desc, bufs, out, first, count = build_batch(cfg, srank, sworld, torch, dev, eng, sptr,
                                                        flags)
    alg = alg_bytes_flags(desc, cfg["family"], flags, with_out)
    len_hint = int(desc["len"].mean()) if count else 0
    out_arg = out if with_out else None

    def step(k):
        eng.batch_device(bufs[k % len(bufs)], d_desc, count, out_arg, cfg["mode"], flags,
                         len_hint, stream=sptr)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    # The library's once-per-context order calibration (xcsum_ctx_calibrate_order)
    # on this rank's batch, as libxudp would run it once its UMEM is set up:
    # the automatic order unless a forced one is >= 1 % faster on this box.
    # Before the graph capture, which bakes the order into the launches.
    calibrated = None
    if args.calibrate and count and not args.geometry:
        calibrated = eng.calibrate_order(bufs[0], d_desc, count, out_arg, cfg["mode"], flags,
                                         len_hint, stream=sptr)

    # The K timed launches are captured once into a HIP graph and replayed:
    # the host enqueues one graph instead of K ctypes launches, so short
    # kernels (config 3) are not host-bound.  Every replay runs all K
    # checksum launches.  --no-graph times eager launches instead.
    graph = None
    if not args.no_graph:
        try:
            graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(stream)
            with torch.cuda.graph(graph, stream=cap):
                cptr = torch.cuda.current_stream(dev).cuda_stream
                for k in range(args.steps):
                    eng.batch_device(bufs[k % len(bufs)], d_desc, count, out_arg, cfg["mode"],
                                     flags, len_hint, stream=cptr)
            stream.wait_stream(cap)
            torch.cuda.synchronize(dev)
        except Exception as e:  # capture unsupported: fall back to eager launches
            print(f"note: graph capture failed ({e}); timing eager launches", file=sys.stderr)
            graph = None

    def run_k():
        """the K steps, enqueued on `stream`"""
        if graph is not None:
            graph.replay()
        else:
            for k in range(args.steps):
                step(k)

    # Clock ramp (untimed): the GPU's clocks take tens of milliseconds of
    # sustained load to reach their working point; a few warm-up launches
    # (the driver's --warmup 5 is ~1 ms of work) leave the timed region on a
    # ramping clock (round 1: 274 us first replays vs 241 us steady).  So the
    # K-step body runs back to back for at least --ramp-ms of wall time
    # before anything is timed, whatever --warmup says.
    # It ends once --ramp-ms have passed AND the last three bodies agree
    # within 1 % (event-timed), or after 4 s: some boxes were still speeding
    # up after 300 ms (round 3: repetitions 0.268 -> 0.235 ms on one box).
    torch.cuda.synchronize(dev)
    t_r = time.perf_counter()
    n_ramp = 0
    body_ms = []
    while True:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run_k()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        body_ms.append(e0.elapsed_time(e1))
        n_ramp += 1
        ramp_ms = (time.perf_counter() - t_r) * 1e3
        last = body_ms[-3:]
        steady = len(last) == 3 and max(last) <= 1.01 * min(last)
        if (ramp_ms >= args.ramp_ms and n_ramp >= 2 and (steady or args.ramp_ms <= 0)) \
                or ramp_ms >= max(4000.0, args.ramp_ms):
            break
    # clocks while the kernel is running: enqueue ~40 ms more, sample, drain
    per_body = ramp_ms / n_ramp
    for _ in range(max(1, int(40.0 / max(per_body, 1e-3)))):
        run_k()
    clocks_load = gpu_clocks(dev)
    torch.cuda.synchronize(dev)

    # Timed region: R repetitions of exactly K steps, each bracketed by a
    # barrier and a device synchronize on both sides; the reported step time
    # is the median repetition (max over ranks per repetition).
    reps = max(1, args.reps)
    walls, kms = [], []
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for r in range(reps):
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev[r][0].record(stream)
        run_k()
        ev[r][1].record(stream)
        torch.cuda.synchronize(dev)
        barrier()
        t1 = time.perf_counter()
        walls.append(t1 - t0)
    for r in range(reps):
        # HIP events around the K launches on the stream they run on; per
        # launch = region / K (includes the ~1 us graph node boundaries)
        kms.append(ev[r][0].elapsed_time(ev[r][1]) / args.steps)
    clocks_after = gpu_clocks(dev)

    # whole-job numbers: per repetition the max elapsed over ranks, then the
    # median repetition; bytes summed over ranks
    sdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    wt = torch.tensor(walls, dtype=torch.float64, device=sdev)
    tot = torch.tensor([float(alg), float(count)], dtype=torch.float64, device=sdev)
    kern_ms = float(np.median(kms))
    # per rank: its kernel's median launch time, algorithmic bytes and frames
    mine = torch.tensor([kern_ms, float(alg), float(count)], dtype=torch.float64, device=sdev)
    per_rank = [mine]
    if use_dist:
        dist.all_reduce(wt, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        per_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
    per_rank = [[float(x) for x in t.cpu()] for t in per_rank]
    walls_max = [float(x) for x in wt.cpu()]
    elapsed_max = float(np.median(walls_max))
    alg_all, frames_all = float(tot[0]), float(tot[1])

    ceiling = inplace = orders = hdr_probe = spans = None
    if rank == 0 and not args.no_ceiling:
        ceiling = stream_ceiling(torch, dev, bufs, sptr)
        if (args.layout == "umem" or cfg["id"] == 5) and \
                not flags & (X.F_INPLACE | X.F_IPHDR_ONLY):
            # xudp's slots, mixed sizes: the loads the kernel must make, in
            # its orders, one wave per frame
            spans = span_ceiling(torch, dev, bufs, d_desc, desc, sptr, real_bytes(desc, flags))
        if flags & X.F_IPHDR_ONLY:
            hdr_probe = header_ceiling(torch, dev, bufs, d_desc, count,
                                       bool(flags & X.F_INPLACE) and not flags & X.F_VERIFY,
                                       sptr)
        if flags & X.F_INPLACE and with_out is False and not flags & X.F_IPHDR_ONLY:
            inplace = inplace_ceiling(torch, dev, bufs, desc, flags, cfg["family"], sptr)
        if args.order_ab and cfg["id"] in (2, 4) and not flags and not args.geometry:
            # after the in-place probe (none here: no flags), before the
            # parity pass: the order never changes results
            orders = order_ab(torch, dev, eng, bufs, d_desc, count, out_arg, cfg, flags,
                              len_hint, sptr, real_bytes(desc, flags),
                              ceiling["GBps"] if ceiling else None, calibrated)

    if not with_out and count:
        # the in-place passes rewrote the check fields of every buffer (and the
        # probe wrote garbage there): regenerate the frames, then one pass with
        # the result array as well, which the parity checks read
        eng.gen_fill_device(bufs[0], d_desc, count, cfg["family"], SEED_BASE ^ cfg["id"], first,
                            stream=sptr)
        eng.batch_device(bufs[0], d_desc, count, out, cfg["mode"], flags, len_hint, stream=sptr)
        torch.cuda.synchronize(dev)
    else:
        # the last timed pass may have read another buffer: one more on bufs[0]
        step(0)
        torch.cuda.synchronize(dev)

    # parity spot check of the output (and, in place, of the frame bytes)
    ok = None
    if rank == 0 and count:
        import oracle  # checker only
        m = min(count, 4096)
        got = d2h(torch, out[:m]).view(np.uint16)
        ubytes = int(desc["addr"][m - 1]) + int(desc["len"][m - 1])
        hu = d2h(torch, bufs[0][:ubytes])
        if flags & X.F_INPLACE and not flags & X.F_VERIFY and flags & X.F_IPHDR_ONLY:
            # libxudp's IPv4 call: iph->check written, udp->check still 0
            fresh = hu.copy()
            for k in range(m):
                a0 = int(desc["addr"][k])
                fresh[a0 + 24:a0 + 26] = 0
            exp = oracle.batch(fresh, desc[:m], cfg["mode"], flags & ~X.F_INPLACE)
            ok = bool(np.array_equal(got, exp))
            for k in range(m):
                a0 = int(desc["addr"][k])
                ok = ok and int(hu[a0 + 24:a0 + 26].view("<u2")[0]) == int(exp[k]) \
                    and not hu[a0 + 40:a0 + 42].any()
        elif flags & X.F_INPLACE and not flags & X.F_VERIFY:
            fresh = hu.copy()
            off = 60 if cfg["family"] == 6 else 40
            for k in range(m):       # the pristine frames, check fields 0
                a0 = int(desc["addr"][k])
                fresh[a0 + off:a0 + off + 2] = 0
                if flags & X.F_IPHDR and cfg["family"] == 4:
                    fresh[a0 + 24:a0 + 26] = 0
            exp = oracle.batch(fresh, desc[:m], cfg["mode"], flags & ~X.F_INPLACE)
            ok = bool(np.array_equal(got, exp))
            for k in range(m):
                a0 = int(desc["addr"][k])
                ok = ok and int(hu[a0 + off:a0 + off + 2].view("<u2")[0]) == int(exp[k])
                if flags & X.F_IPHDR and cfg["family"] == 4:
                    f = fresh[a0:a0 + int(desc["len"][k])]
                    ok = ok and int(hu[a0 + 24:a0 + 26].view("<u2")[0]) == oracle.ip_header_rfc(f)
        else:
            ok = bool(np.array_equal(got, oracle.batch(hu, desc[:m], cfg["mode"], flags)))
    # IPHDR_ONLY: the reference's xudp_checksum_half over the same frames
    digest = None if flags & X.F_VERIFY else digest_check(
        cfg, out, count, world, rank, dist, sdev,
        "sha256_iphdr" if flags & X.F_IPHDR_ONLY else "sha256_out", shard)

    parity_ok = True
    if rank == 0:
        value = alg_all * args.steps / elapsed_max / 2**30
        # the slowest rank's kernel sets the fraction (at N = 1: this one)
        slow = max(per_rank, key=lambda r: r[0])
        achieved = slow[1] / (slow[0] * 1e-3) / 1e9  # GB/s
        sha = lib_sha16()
        traffic, traffic_src, why, ksha = pmc_traffic(args.config, args.layout, flags, sha)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": traffic_src}
        if ksha:
            roof["traffic_kernel_sha16"] = ksha   # the counted kernel's code, this build
        if why:
            roof["traffic_note"] = why
        if traffic is not None and cfg["shard"] and (world > 1 or shard is not None):
            # the counters were taken on the whole 8M-frame job; this line's
            # launches are shards of it: no per-launch bytes to report, only
            # the whole job's ratio to its algorithmic bytes
            try:
                j = json.load(open(os.path.join(ROOT, traffic_src)))
                roof["traffic_over_alg_whole_job"] = j.get("traffic_over_alg")
            except (OSError, ValueError):
                pass
            roof["traffic"] = None
            roof["traffic_note"] = (f"counters in {traffic_src} were taken on the whole "
                                    f"{cfg['n']}-frame job, this line's launches are shards")
        # bytes the kernel must move per launch (every 64-byte line holding a
        # frame byte, once, + 16-byte descriptors + 2-byte results): the
        # apples-to-apples numerator for the stream-read ceiling
        real = real_bytes(desc, flags)
        roof["real_bytes_per_launch"] = real
        roof["real_achieved"] = round(real / (kern_ms * 1e-3) / 1e9, 1)
        if ceiling:
            roof["ceiling_measured"] = ceiling["GBps"]
            roof["ceiling_GBps_by_leg"] = ceiling.get("GBps_by_leg")
            roof["frac_vs_ceiling"] = round(roof["real_achieved"] / ceiling["GBps"], 4)
            roof["ceiling_probe"] = ceiling["what"]
            # The layout's own bound: a launch must move `real` bytes to
            # deliver `alg` algorithmic ones (config 3: a 106-byte frame in
            # 112 bytes + a 16-byte descriptor per 82 algorithmic bytes), so
            # at the same-run ceiling the algorithmic rate tops out at
            # ceiling x alg / real.  layout_bound_frac = that bound over the
            # 8 TB/s peak; frac_of_layout_bound = achieved over that bound.
            alg_launch = slow[1]
            bound = ceiling["GBps"] * alg_launch / real
            roof["layout_alg_over_real"] = round(alg_launch / real, 4)
            roof["layout_bound_GBps"] = round(bound, 1)
            roof["layout_bound_frac"] = round(bound / HBM_PEAK_GBS, 4)
            roof["frac_of_layout_bound"] = round(achieved / bound, 4)
        if spans:
            # the layout's like-for-like bound: the same loads, no arithmetic
            roof["span_probe_ms"] = spans["ms"]
            roof["span_probe_GBps"] = spans["GBps"]
            roof["span_probe_ms_by_leg"] = spans["ms_by_leg"]
            roof["frac_vs_span_probe"] = round(spans["ms"] / kern_ms, 4)
            roof["span_probe"] = spans["what"]
        if orders:
            roof["order_ab"] = orders
        if hdr_probe:
            # the same descriptor, header and field accesses, no arithmetic:
            # the bound of one scattered line read (+ write) per frame
            roof["header_probe_ms"] = hdr_probe["ms"]
            roof["frac_vs_header_probe"] = round(hdr_probe["ms"] / kern_ms, 4)
            roof["header_probe"] = hdr_probe["what"]
        if inplace:
            # same buffers, same reads, the same stores per frame, no arithmetic
            roof["inplace_probe_ms"] = inplace["ms"]
            roof["inplace_probe_ms_by_unroll"] = inplace["ms_by_unroll"]
            roof["frac_vs_inplace_probe"] = round(inplace["ms"] / kern_ms, 4)
            roof["inplace_probe"] = inplace["what"]
        parity_ok = ok is not False and (digest is None or digest.get("ok") is not False)
        fl = ",".join(k for k, v in FLAG_NAMES.items() if flags & v)
        line = {
            "metric": (f"device-resident IPv4 header checksum GiB/s, libxudp's IPv4 TX call "
                       f"(iph->check only, packet.c:43-66; config {args.config} frames)"
                       if flags & X.F_IPHDR_ONLY else
                       "device-resident UDP checksum GiB/s + %HBM-peak, 1M x 1472B IPv4 packets"
                       if args.config == 2 else f"device-resident UDP checksum GiB/s (config "
                                                f"{args.config})")
                      + (f" [flags {fl}]" if flags else ""),
            "value": round(value, 2) if parity_ok else None,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if cfg["shard"] else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SplitMix64 frames generated on device, xudp_packet_udp layout)",
            "config": {"workload": cfg["name"], "frames_per_gpu": count,
                       "frames_total": int(frames_all), "payload_bytes": [cfg["pmin"], cfg["pmax"]],
                       "family": cfg["family"], "mode": MODE_NAMES[cfg["mode"]],
                       "flags": fl or "none",
                       "result_array": with_out,
                       "reference_call": reference_call(cfg, flags),
                       "inplace_schedule": (args.inplace_schedule if flags & X.F_INPLACE
                                            and not flags & X.F_VERIFY else None),
                       "layout": "packed, 8-byte aligned frames" if args.layout == "packed"
                       else "xudp TX UMEM: one frame per 4096-byte chunk",
                       "visiting_order": "automatic (32 regions of 16-frame tiles if the batch "
                                         "is sparse in the UMEM, else the geometry's dense "
                                         "order: 8 regions of 16-frame tiles at MTU, 16 of "
                                         "4-frame tiles for mixed sizes)"
                       if calibrated in (None, (-1, 0)) else
                       f"forced by xcsum_ctx_calibrate_order: 2^{calibrated[0]} regions of "
                       f"2^{calibrated[1]}-frame tiles (>= 1 % faster than automatic here)",
                       "order_calibration": (None if calibrated is None else
                                             "auto" if calibrated == (-1, 0) else
                                             f"{calibrated[0]},{calibrated[1]}"),
                       "rotating_buffers": len(bufs),
                       "alg_bytes_per_step": int(alg_all), "parallelism": f"dp{world}",
                       "shard": (None if shard is None else
                                 f"{shard[0]}/{shard[1]}: frames {first}..{first + count - 1} "
                                 f"of the job, one rank's byte-balanced share, timed alone")},
            "pct_hbm_peak": round(100 * achieved / HBM_PEAK_GBS, 2),
            "mpps": round(frames_all * args.steps / elapsed_max / 1e6, 1),
            "kernel_ms": round(kern_ms, 4),
            "per_rank": {"ranks": world,
                         "kernel_ms": [round(r[0], 4) for r in per_rank],
                         "achieved_GBps": [round(r[1] / (r[0] * 1e-3) / 1e9, 1) for r in per_rank],
                         "kernel_ms_min_median_max": [round(min(r[0] for r in per_rank), 4),
                                                      round(float(np.median([r[0] for r in
                                                                             per_rank])), 4),
                                                      round(slow[0], 4)],
                         "frac_from": "the slowest rank's kernel"},
            "lib_sha16": sha,   # of the kernels (.hip_fatbin), see lib_sha16()
            "kernel_ms_reps": [round(x, 4) for x in kms],
            "wall_ms_reps": [round(x * 1e3, 4) for x in walls_max],
            "timing": (f"median of {reps} repetitions of the K steps "
                       f"({'hipGraph replay' if graph is not None else 'eager launches'}), "
                       f"each bracketed by barrier + synchronize"),
            "clock_ramp_ms": round(ramp_ms, 1),
            "ramp_bodies_ms_last3": [round(x, 3) for x in body_ms[-3:]],
            "clocks": {"under_load": clocks_load, "after_timing": clocks_after},
            "parity_spot_check": ok,
            "parity_digest": digest,
            "parity_ok": parity_ok,
            "roofline": roof,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds, flags)
        print(json.dumps(line), flush=True)

    eng.close()
    if use_dist:
        dist.destroy_process_group()
    if rank == 0 and not parity_ok:
        print("bench: the output differs from the reference; value withheld", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
