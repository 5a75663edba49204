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
reading the restatement side by side with the reference).

Content: the identifiers on the citing line and the line above it (names with
an underscore, ALL_CAPS names, camelCase) that the cited file holds are the
ones the citation talks about; at least one of them must appear in the cited
lines (case-insensitively, as a word prefix, so the edge name
"ip_input_bad_length" is found as BAD_LENGTH in ip_input.c and a call as the
function's name). Not informative, so not required: the cited file's own
stem (a node cited by its file), other grout node names (the context names
the next node), and identifiers common to many reference files (data_len,
vrf_id ...). A citation with no informative identifier is only range-checked.

Exit 1 when a citation is out of range or its content does not match. Used
by tests/test_citations.py; needs /root/reference (study only: nothing under
it is executed or imported).
"""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

SCAN = [
    "include", "grout_amd/csrc", "grout_amd/module", "tests/standin", "grout_amd", "oracle", "tests", "bench.py",
    "DESIGN.md", "INTEGRATION.md", "__graft_entry__.py",
]
EXT = (".c", ".h", ".cpp", ".hip", ".py", ".md")

EXPLICIT = re.compile(r"((?:[\w.-]+/)*[\w-]+(?:\.[\w-]+)*\.(?:c|h|cpp|hip|sh)):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")
BARE = re.compile(r"(?:^|[\s(,;])(?<![\w.]):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")


IDENT = re.compile(r"\b[A-Za-z_][A-Za-z0-9_]*\b")
FILE_REF = re.compile(r"[\w./-]+\.(?:c|h|cpp|hip|py|md|sh|json)\b")
# acronyms and words of the prose, not identifiers
PROSE = {
    "ABI", "API", "ARP", "BGP", "CPU", "DPDK", "ECMP", "FIB", "GPU", "HBM", "HIP", "ICMP", "IPIP", "LDS", "MAC",
    "MTU", "NDP", "QSBR", "RCU", "RSS", "SNAT", "DNAT", "TCP", "TTL", "UDP", "VLAN", "VRF", "SPDX", "BSD", "TODO",
    "FIXME", "NOTE", "XXX", "LOCAL", "NEXT", "CHAIN", "NULL",
}
COMMON_IN = 12  # an identifier found in this many reference files or more is common


# IPv4 / IPv6 addresses and prefixes: what a smoke script's cited line configures or pings
ADDR = re.compile(r"(?<![\w.:])(?:(?:\d{1,3}\.){3}\d{1,3}|[0-9a-f]{1,4}(?::[0-9a-f]{0,4}){2,7})(?:/\d+)?(?![\w.:])")


def identifiers(text):
    out = set()
    for w in IDENT.findall(FILE_REF.sub(" ", text)):
        if w in PROSE or re.fullmatch(r"u?int\d+_t|size_t|ssize_t", w):
            continue
        if "_" in w.strip("_") or (w.isupper() and len(w) >= 3) or re.match(r"[a-z]+[A-Z]", w):
            out.add(w)
    return out


class Content:
    """The content check's view of the reference: grout's node names and the
    identifiers common to many of its files."""

    def __init__(self, ref_idx):
        self.nodes = set()
        self.common = set()
        self.df = {}
        counts = {}
        for name, paths in ref_idx.items():
            if not name.endswith((".c", ".h")):
                continue
            for p in paths:
                text = "\n".join(n_lines(p))
                for w in set(IDENT.findall(text)):
                    counts[w] = counts.get(w, 0) + 1
                for m in re.finditer(r'\.name\s*=\s*"(\w+)"', text):
                    self.nodes.add(m.group(1))
                for m in re.finditer(r'\[\w+\]\s*=\s*"(\w+)"', text):
                    self.nodes.add(m.group(1))
        self.common = {w for w, c in counts.items() if c >= COMMON_IN}
        fx = os.path.join(ROOT, "tests", "golden", "graph_svg.json")
        if os.path.isfile(fx):
            import json
            with open(fx) as fh:
                d = json.load(fh)
            self.nodes |= set(d["nodes"]) | set(d["registered"])

    def informative(self, ids, path):
        stem = os.path.basename(path).rsplit(".", 1)[0]
        whole = "\n".join(n_lines(path))
        out = []
        for i in ids:
            edge_name = i.lower().startswith(stem.lower() + "_")  # the cited node's own edge
            if i == stem or i in self.common or (i in self.nodes and not edge_name):
                continue
            if re.search(r"\b%s" % re.escape(i), whole, re.I):
                out.append(i)
        return out, stem

    def check(self, ids, path, rs):
        """None: nothing to check; else whether the cited lines hold one of the ids."""
        fid, stem = self.informative(ids, path)
        if not fid:
            return None
        L = n_lines(path)
        body = "\n".join("\n".join(L[a - 1:b]) for a, b in rs) + "\n" + enclosing(L, rs[0][0])
        if path.endswith(".sh") and "$" in body:
            return None  # a templated line (addresses built from $n): not comparable
        for i in fid:
            alts = [i]
            if i.lower().startswith(stem.lower() + "_"):
                alts.append(i[len(stem) + 1:])  # an edge name: its enum constant
            # a word prefix, or a part of a name after an underscore (LOOPBACK in ETH_DOMAIN_LOOPBACK)
            if any(re.search(r"(?<![A-Za-z0-9])%s" % re.escape(x), body, re.I) for x in alts):
                return True
        return False


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


def enclosing(L, a):
    """The definition line a cited range sits in (a C function's or struct's
    first line at column 0), for citations that name the function."""
    for k in range(a - 2, max(-1, a - 400), -1):
        t = L[k]
        if t and not t[0].isspace() and t[0] not in "}#/*" and not re.match(r"\w+:\s*$", t):
            return t  # (a goto label at column 0 is not a definition)
    return ""


SCRIPT = re.compile(r"\b([\w-]+\.sh)\b")
COMMENT = re.compile(r"//|/\*|(?:^|\s)#\s")


def after_comment(text):
    """The comment part of a line of code (all of it when it has no marker)."""
    ms = list(COMMENT.finditer(text))
    return text[ms[-1].end():] if ms else text


def scan_file(path):
    """(rel, line, file, ranges, context identifiers) per citation. The
    context of a citation is the text between it and the citation before it
    (on this line, else the tail of the line above), in the comment part of
    a line of code, and the rest of its line up to the next citation."""
    rel = os.path.relpath(path, ROOT)
    with open(path, encoding="utf-8", errors="replace") as fh:
        lines = fh.read().split("\n")
    last = None  # (file, line number) of the last explicit citation
    prev_tail = ""
    prose_prev = False
    in_doc = False
    for no, text in enumerate(lines, 1):
        # prose: Markdown, a docstring, a comment line; the tail of the line
        # above carries over to this one only from prose to prose
        st = text.strip()
        prose = path.endswith(".md") or in_doc or st.startswith(("#", "//", "*", "/*", '"""'))
        if path.endswith(".py") and text.count('"""') % 2:
            in_doc = not in_doc
        carry = prev_tail if prose and prose_prev else ""
        spans = []
        for m in EXPLICIT.finditer(text):
            spans.append((m.start(), m.end(), m.group(1), m.group(2)))
        for m in BARE.finditer(text):
            spans.append((m.start(1) - 1, m.end(), None, m.group(1)))
        for m in SCRIPT.finditer(text):
            if not text[m.end():m.end() + 1] == ":" or not text[m.end() + 1:m.end() + 2].isdigit():
                spans.append((m.start(), m.end(), m.group(1), None))  # a script named without lines
        spans.sort()
        here = None  # the last explicit citation on this line
        for k, (pos, end, name, spec) in enumerate(spans):
            before = text[spans[k - 1][1]:pos] if k else carry + "\n" + after_comment(text[:pos])
            nxt = spans[k + 1][0] if k + 1 < len(spans) else len(text)
            # what follows a citation, up to the end of its clause
            m = re.search(r"[;,]|\)\s", text[end:nxt])
            nxt = end + m.start() if m else nxt
            ctx = identifiers(before + "\n" + text[end:nxt])
            # a smoke script's line: the code around the citation says what it holds
            sh = set(ADDR.findall(text[spans[k - 1][1] if k else 0:pos])) or set(ADDR.findall(text[end:nxt]))
            if spec is None:
                last = (name, no)  # the bare ranges below are the script's lines
                here = name
                continue
            if name is None:
                # a bare range: the file cited just before it on this line,
                # else the main citation of the lines above, nearby
                if here is not None:
                    name = here
                elif last is None or no - last[1] > 40:
                    continue
                else:
                    name = last[0]
                yield rel, no, name, spec, sh if name.endswith(".sh") else ctx
                continue
            here = name
            if text[:pos].count("(") <= text[:pos].count(")"):
                # a main citation: bare ranges after it continue it (one in
                # parentheses is a side note and does not)
                last = (name, no)
            yield rel, no, name, spec, sh if name.endswith(".sh") else ctx
        prev_tail = after_comment(text[spans[-1][1]:] if spans else text)
        prose_prev = prose


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
    content = Content(ref_idx)
    bad = mismatched = 0
    seen = set()
    for f in files:
        if f in seen:
            continue
        seen.add(f)
        for rel, no, name, spec, ctx in scan_file(f):
            cands, where = candidates(name, ref_idx, repo_idx)
            if not cands:
                continue  # DPDK or another file absent from the reference
            rs = ranges(spec)
            ok_paths = [c for c in cands if all(1 <= a <= b <= len(n_lines(c)) for a, b in rs)]
            if not ok_paths:
                bad += 1
                print(f"BAD {rel}:{no}: {name}:{spec} (file has {len(n_lines(cands[0]))} lines: {cands[0]})")
                continue
            verdicts = [content.check(ctx, c, rs) for c in ok_paths]
            if False in verdicts and True not in verdicts:
                mismatched += 1
                fid, _ = content.informative(ctx, ok_paths[0])
                print(f"MISMATCH {rel}:{no}: {name}:{spec} holds none of {sorted(fid)}")
            elif a.show:
                c = ok_paths[0]
                first = n_lines(c)[rs[0][0] - 1].strip()
                amb = f" [+{len(ok_paths) - 1} more]" if len(ok_paths) > 1 else ""
                print(f"{rel}:{no}: {name}:{spec}{amb} -> {os.path.relpath(c, REF if where == 'ref' else ROOT)}: {first[:90]}")
    print(f"{bad} citation(s) out of range, {mismatched} not holding what they cite", file=sys.stderr)
    return 1 if bad or mismatched else 0


if __name__ == "__main__":
    sys.exit(main())
