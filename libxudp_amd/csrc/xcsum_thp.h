/* xcsum_thp.h -- can the kernel move the pages of a host range under a GPU
 * mapping?  The registration policy of xcsum_register_umem:
 * the registered-memory faults of rounds 2-4 all hit memory eligible for
 * transparent huge pages (numpy's heap, madvise(MADV_HUGEPAGE) by numpy for
 * arrays of 4 MiB and up: VmFlags "hg"); none hit libxudp's UMEM mapping
 * (anon_map, MAP_SHARED | MAP_LOCKED | MAP_POPULATE, include/common.h:37-41,
 * not THP-eligible under THP "madvise"), and the same suite ran clean with
 * THP disabled for the process.
 *
 * Plain C++ over a /proc/<pid>/smaps stream and the THP sysfs modes, so the
 * parser is tested on synthetic input on the CPU (tests/test_thp_policy.py).
 * Eligible: a VMA overlapping [lo, hi) that is
 *   - private (no "sh" flag): THP not "never", and flagged "hg", or THP
 *     "always" and not flagged "nh";
 *   - shared ("sh": shmem, anon_map's MAP_SHARED | MAP_ANONYMOUS): not "nh",
 *     and shmem_enabled "always" / "force" / "within_size", or "advise" with
 *     "hg".
 * The policy is read once, at registration (include/xcsum.h). */
#ifndef XCSUM_THP_H
#define XCSUM_THP_H

#include <stdint.h>
#include <stdio.h>
#include <string.h>

namespace xcsum {

struct ThpModes {
	bool never;       /* transparent_hugepage/enabled = [never] */
	bool always;      /* ... = [always] */
	bool sh_always;   /* shmem_enabled = [always] / [force] / [within_size] */
	bool sh_advise;   /* shmem_enabled = [advise] */
};

/* does this VmFlags line ("VmFlags: rd wr ... hg") carry flag fl? */
static inline bool vmflag(const char *line, const char *fl)
{
	const size_t n = strlen(fl);
	for (const char *p = strstr(line, fl); p; p = strstr(p + 1, fl))
		if (p[-1] == ' ' && (p[n] == ' ' || p[n] == '\n' || p[n] == '\0'))
			return true;
	return false;
}

/* the smaps stream `f`: is any VMA overlapping [lo, hi) THP-eligible? */
static inline bool thp_eligible_smaps(FILE *f, uintptr_t lo, uintptr_t hi, const ThpModes &m)
{
	char line[512];
	uintptr_t s = 0, e = 0;
	bool eligible = false;
	while (fgets(line, sizeof line, f)) {
		unsigned long a, b;
		/* a VMA header: "start-end perms ..." (the '-' before the first
		 * blank, which no "Key: value" line has) */
		const char *dash = strchr(line, '-'), *blank = strchr(line, ' ');
		if (dash && blank && dash < blank && sscanf(line, "%lx-%lx ", &a, &b) == 2) {
			s = a;
			e = b;
			continue;
		}
		if (strncmp(line, "VmFlags:", 8) != 0 || !(s < hi && e > lo))
			continue;
		const bool hg = vmflag(line, "hg"), nh = vmflag(line, "nh");
		if (vmflag(line, "sh"))
			eligible |= !nh && (m.sh_always || (m.sh_advise && hg));
		else
			eligible |= !m.never && (hg || (m.always && !nh));
	}
	return eligible;
}

} /* namespace xcsum */

#endif
