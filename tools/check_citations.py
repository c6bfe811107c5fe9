#!/usr/bin/env python3
"""Every profiles/ path DESIGN.md, README.md and INTEGRATION.md cite exists
(bundle sections: 'x.bundle.txt: name' -> a '===== name' header inside, with
shell-style wildcards).  Exit 1 and list the misses."""
import fnmatch
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
miss = []
for doc in ("DESIGN.md", "README.md", "INTEGRATION.md", "profiles/README.md"):
    p = os.path.join(ROOT, doc)
    if not os.path.exists(p):
        continue
    text = open(p).read().replace("\n", " ")
    for m in re.finditer(r"(profiles/[A-Za-z0-9_./{}*,\-]+?)(?=[`\s,;):]|$)(?::\s*([^`)]*))?", text):
        path = m.group(1).rstrip(".")
        cands = [path]
        br = re.match(r"(.*)\{([^}]*)\}(.*)", path)
        if br:
            cands = [br.group(1) + x + br.group(3) for x in br.group(2).split(",")]
        for c in cands:
            full = os.path.join(ROOT, c)
            if "*" in c:
                import glob
                ok = bool(glob.glob(full))
            else:
                ok = os.path.exists(full)
            if not ok:
                miss.append(f"{doc}: {c}")
                continue
            if c.endswith(".bundle.txt") and m.group(2):
                heads = re.findall(r"^===== (.*) =====$", open(full).read(), re.M)
                for sec in re.split(r",\s+", m.group(2).strip()):
                    sec = sec.strip().rstrip(".")
                    if not sec:
                        continue
                    secs = [sec]
                    b2 = re.match(r"(.*)\{([^}]*)\}(.*)", sec)
                    if b2:
                        secs = [b2.group(1) + x + b2.group(3) for x in b2.group(2).split(",")]
                    for s2 in secs:
                        if not any(fnmatch.fnmatch(h, s2) or fnmatch.fnmatch(h, s2 + "*")
                                   or h.startswith(s2) for h in heads):
                            miss.append(f"{doc}: {c}: {s2}")
print("\n".join(miss) or "all cited profile paths exist")
sys.exit(1 if miss else 0)
