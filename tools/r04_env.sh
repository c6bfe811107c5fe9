#!/bin/bash
# Read-only facts about the GPU box that bear on registered (userptr) host
# memory: memlock limit, THP and compaction settings, kernel, NUMA balancing.
# Nothing is changed.
set -u
echo "uname: $(uname -r)"
echo "ulimit -l: $(ulimit -l)"
for f in /sys/kernel/mm/transparent_hugepage/enabled \
         /sys/kernel/mm/transparent_hugepage/defrag \
         /sys/kernel/mm/transparent_hugepage/khugepaged/defrag \
         /sys/kernel/mm/transparent_hugepage/khugepaged/scan_sleep_millisecs \
         /proc/sys/vm/compact_unevictable_allowed \
         /proc/sys/kernel/numa_balancing \
         /sys/module/amdgpu/parameters/noretry \
         /sys/module/amdgpu/parameters/mtype_local \
         /sys/module/amdgpu/parameters/vm_fragment_size; do
  [ -r "$f" ] && echo "$f: $(cat "$f" 2>/dev/null)"
done
python3 -c "import numpy, numpy.core.multiarray as m; print('numpy', numpy.__version__, 'madvise_hugepage', m._get_madvise_hugepage() if hasattr(m, '_get_madvise_hugepage') else '?')" 2>&1
grep -E 'thp_|compact_(migrate|stall|success)|pgmigrate' /proc/vmstat 2>/dev/null | tr '\n' ' '; echo
