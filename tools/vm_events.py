"""Kernel memory-management events around a command (read-only diagnostic).

Prints the box's NUMA-balancing and transparent-huge-page settings, then the
/proc/vmstat counters that move when the kernel unmaps, migrates, collapses or
splits pages of a process (each such change invalidates any GPU mapping of a
registered host range: amdgpu's MMU notifier evicts the range and the
process's queues), sampled before and after `-- <command>`, which runs as a
child process.  The counters are machine-wide: other processes on the host
move them too, so a zero delta is the informative result.

    python tools/vm_events.py -- python -m pytest tests/test_gpu_resident.py -q
"""
import subprocess
import sys

KEYS = ("numa_pte_updates", "numa_hint_faults", "numa_pages_migrated", "pgmigrate_success",
        "pgmigrate_fail", "thp_collapse_alloc", "thp_split_pmd", "thp_fault_alloc",
        "compact_migrate_scanned", "compact_stall", "thp_migration_success")
SETTINGS = ("/proc/sys/kernel/numa_balancing", "/sys/kernel/mm/transparent_hugepage/enabled",
            "/sys/kernel/mm/transparent_hugepage/defrag",
            "/sys/kernel/mm/transparent_hugepage/khugepaged/defrag",
            "/proc/sys/vm/compaction_proactiveness", "/proc/sys/vm/compact_unevictable_allowed")


def vmstat():
    out = {}
    with open("/proc/vmstat") as f:
        for ln in f:
            k, v = ln.split()
            if k in KEYS:
                out[k] = int(v)
    return out


def main():
    argv = sys.argv[1:]
    cmd = argv[argv.index("--") + 1:] if "--" in argv else []
    for p in SETTINGS:
        try:
            print(f"{p}: {open(p).read().strip()}")
        except OSError as e:
            print(f"{p}: unreadable ({e.strerror})")
    before = vmstat()
    rc = subprocess.call(cmd) if cmd else 0
    after = vmstat()
    for k in KEYS:
        if k in before:
            print(f"vmstat {k}: {after[k] - before[k]:+d} (now {after[k]})")
    sys.exit(rc)


if __name__ == "__main__":
    main()
