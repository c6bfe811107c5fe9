#!/usr/bin/env python3
"""Fold a profiles/ subtree into one text bundle (round-3 prune: VERDICT r2
asked for < 150 tracked files under profiles/).  Every file of the subtree is
concatenated verbatim, in path order, under a '===== relative/path =====' header,
into <subtree>.bundle.txt next to it; the originals are removed with git rm.
A citation 'profiles/r02/x/y.log' becomes 'profiles/r02/x.bundle.txt' (section
'y.log').

    python tools/bundle_profiles.py profiles/r02/session2/order_dense [...]
    python tools/bundle_profiles.py --loose profiles/r01   # the files directly in it
"""
import os
import subprocess
import sys


def tracked(path):
    out = subprocess.run(["git", "ls-files", path], capture_output=True, text=True, check=True)
    return sorted(out.stdout.split())


def bundle(root, loose=False):
    root = root.rstrip("/")
    files = tracked(root)
    if loose:
        files = [f for f in files if os.path.dirname(f) == root]
        dest = os.path.join(root, "loose.bundle.txt")
        base = root
    else:
        dest = root + ".bundle.txt"
        base = root
    files = [f for f in files if f != dest]
    if not files:
        return
    with open(dest, "w") as out:
        out.write(f"# bundle of {base}/{' (files directly in it)' if loose else ''}: "
                  f"{len(files)} files concatenated verbatim in path order\n")
        for f in files:
            out.write(f"\n===== {os.path.relpath(f, base)} =====\n")
            with open(f, errors="replace") as inp:
                out.write(inp.read())
    subprocess.run(["git", "rm", "-q", *files], check=True)
    subprocess.run(["git", "add", dest], check=True)
    print(f"{dest}: {len(files)} files")


if __name__ == "__main__":
    args = sys.argv[1:]
    loose = "--loose" in args
    for a in (x for x in args if x != "--loose"):
        bundle(a, loose)
