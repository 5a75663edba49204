# SPDX-License-Identifier: BSD-3-Clause
"""Generate tests/golden/graph_svg.json from the reference tree (not run on
the GPU box): the node -> node edges of grout's documented datapath graph,
docs/graph.svg, extracted the way smoke/graph_svg_test.sh:6-9 extracts them
(the <title> of each class="edge" group, "&#45;&gt;" read as " -> ", sorted,
unique), its nodes, and every node name grout's sources register (".name =",
GR_DROP_REGISTER; the svg is `grcli graph show brief`, which leaves the drop
nodes out).

    python tests/golden/make_graph_svg.py [/root/reference]"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "graph_svg.json")


def svg_edges(text):
    lines = text.splitlines()
    titles = []
    for i, line in enumerate(lines):
        if 'class="edge"' in line and i + 1 < len(lines):  # grep -A1 'class="edge"'
            m = re.match(r"^<title>(.+)</title>$", lines[i + 1])
            if m:
                titles.append(m.group(1).replace("&#45;&gt;", " -> ", 1))
    return sorted(set(titles))


def svg_nodes(text):
    return sorted(set(re.findall(r'<g id="node\d+" class="node">\n<title>([^<]+)</title>', text)))


def registered(root):
    names = set()
    for d, _, files in os.walk(os.path.join(root, "modules")):
        for f in files:
            if f.endswith(".c"):
                t = open(os.path.join(d, f), encoding="utf-8", errors="replace").read()
                names |= set(re.findall(r'\.name = "([a-z0-9_]+)"', t))
                names |= set(re.findall(r"GR_DROP_REGISTER\((\w+)\)", t))
    return sorted(names | {"port_rx", "port_tx"})  # RX_NODE_BASE / TX_NODE_BASE (rxtx.h:20-23)


def build(root):
    text = open(os.path.join(root, "docs", "graph.svg"), encoding="utf-8").read()
    return {"source": "docs/graph.svg, smoke/graph_svg_test.sh:6-9", "edges": svg_edges(text),
            "nodes": svg_nodes(text), "registered": registered(root)}


if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump(build(REF), f, indent=0)
        f.write("\n")
    print(OUT)
