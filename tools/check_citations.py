#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Resolve every `file.c:N-M` citation in this repo against the mounted
reference (/root/reference) and against the repo's own files.

A citation is `name.c:RANGES` / `name.h:RANGES` (optionally with a path
prefix), RANGES = N, N-M, comma separated. A bare `:RANGES` continues the
file cited last on its line, else the last main citation (not inside
parentheses) of the 40 lines above.

Prints one line per citation whose line range does not exist in the file it
names (or, with --show, every citation with the first cited line's text, for
reading the restatement side by side with the reference). Exit 1 when a
citation is out of range. Used by tests/test_citations.py; needs
/root/reference (study only: nothing under it is executed or imported).
"""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

SCAN = [
    "include", "grout_amd/csrc", "grout_amd/graph", "grout_amd", "oracle", "tests", "bench.py",
    "DESIGN.md", "INTEGRATION.md", "__graft_entry__.py",
]
EXT = (".c", ".h", ".cpp", ".hip", ".py", ".md")

EXPLICIT = re.compile(r"((?:[\w.-]+/)*[\w-]+(?:\.[\w-]+)*\.(?:c|h|cpp|hip)):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")
BARE = re.compile(r"(?:^|[\s(,;])(?<![\w.]):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")


def index_files(top, skip=()):
    by_name = {}
    for d, dirs, files in os.walk(top):
        dirs[:] = [x for x in dirs if not x.startswith(".") and x not in skip]
        for f in files:
            by_name.setdefault(f, []).append(os.path.join(d, f))
    return by_name


def n_lines(path, cache={}):
    if path not in cache:
        with open(path, "rb") as fh:
            cache[path] = fh.read().decode("utf-8", "replace").split("\n")
    return cache[path]


def ranges(spec):
    out = []
    for part in spec.replace(" ", "").split(","):
        if "-" in part:
            a, b = part.split("-")
            out.append((int(a), int(b)))
        else:
            out.append((int(part), int(part)))
    return out


def candidates(name, ref_idx, repo_idx):
    base = os.path.basename(name)
    repo = repo_idx.get(base, [])
    ref = ref_idx.get(base, [])
    if "/" in name:
        ref = [p for p in ref if p.endswith("/" + name)] or ref
        repo = [p for p in repo if p.endswith("/" + name)]
    # a repo file of that name that the reference lacks: the citation is ours
    if repo and not ref:
        return repo, "repo"
    return ref, "ref"


def scan_file(path):
    rel = os.path.relpath(path, ROOT)
    with open(path, encoding="utf-8", errors="replace") as fh:
        lines = fh.read().split("\n")
    last = None  # (file, line number) of the last explicit citation
    for no, text in enumerate(lines, 1):
        spans = []
        for m in EXPLICIT.finditer(text):
            spans.append((m.start(), m.group(1), m.group(2)))
        for m in BARE.finditer(text):
            spans.append((m.start(1) - 1, None, m.group(1)))
        spans.sort()
        here = None  # the last explicit citation on this line
        for pos, name, spec in spans:
            if name is None:
                # a bare range: the file cited just before it on this line,
                # else the main citation of the lines above, nearby
                if here is not None:
                    name = here
                elif last is None or no - last[1] > 40:
                    continue
                else:
                    name = last[0]
                yield rel, no, name, spec
                continue
            here = name
            if text[:pos].count("(") <= text[:pos].count(")"):
                # a main citation: bare ranges after it continue it (one in
                # parentheses is a side note and does not)
                last = (name, no)
            yield rel, no, name, spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--show", action="store_true", help="print every citation with the cited line")
    ap.add_argument("paths", nargs="*")
    a = ap.parse_args()
    if not os.path.isdir(REF):
        print("no reference mounted", file=sys.stderr)
        return 2
    ref_idx = index_files(REF, skip={"subprojects"})
    repo_idx = index_files(ROOT, skip={"gpurun_out", "build", "__pycache__"})
    paths = a.paths or SCAN
    files = []
    for p in paths:
        full = os.path.join(ROOT, p)
        if os.path.isdir(full):
            for f in sorted(os.listdir(full)):
                if f.endswith(EXT) and os.path.isfile(os.path.join(full, f)):
                    files.append(os.path.join(full, f))
        elif os.path.isfile(full):
            files.append(full)
    bad = 0
    seen = set()
    for f in files:
        if f in seen:
            continue
        seen.add(f)
        for rel, no, name, spec in scan_file(f):
            cands, where = candidates(name, ref_idx, repo_idx)
            if not cands:
                continue  # DPDK or another file absent from the reference
            rs = ranges(spec)
            ok_paths = [c for c in cands if all(1 <= a <= b <= len(n_lines(c)) for a, b in rs)]
            if not ok_paths:
                bad += 1
                print(f"BAD {rel}:{no}: {name}:{spec} (file has {len(n_lines(cands[0]))} lines: {cands[0]})")
            elif a.show:
                c = ok_paths[0]
                first = n_lines(c)[rs[0][0] - 1].strip()
                amb = f" [+{len(ok_paths) - 1} more]" if len(ok_paths) > 1 else ""
                print(f"{rel}:{no}: {name}:{spec}{amb} -> {os.path.relpath(c, REF if where == 'ref' else ROOT)}: {first[:90]}")
    print(f"{bad} citation(s) out of range", file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
