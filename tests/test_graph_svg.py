# SPDX-License-Identifier: BSD-3-Clause
"""grout's documented datapath graph (docs/graph.svg, which
smoke/graph_svg_test.sh:6-15 holds grout's runtime graph to) against the
fast path's node: every edge that leaves the nodes the GPU replaces is one of
the node's verdict edges, or is reached through one of the two CPU
continuation nodes; every verdict edge names a grout node.

The edges are a committed fixture (tests/golden/graph_svg.json, made by
tests/golden/make_graph_svg.py from the reference tree); when the reference
is mounted the fixture is checked against it."""
import json
import os

import pytest

from grout_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
# the nodes whose work the GPU does (enum gr_hip_node)
REPLACED = {"iface_input", "eth_input", "ip_input", "ip_forward", "ip_output", "eth_output", "iface_output",
            "ip6_input", "ip6_forward", "ip6_output"}
# CPU continuation nodes (gpu_fwd4_cpu_nodes.c): the verdict edge that stops
# at grout's conntrack / SNAT hook, and the grout nodes they go on to
CONTINUATIONS = {"ip_input_local_ct": {"ip_input_local", "dnat44_dynamic"},
                 "ip_output_snat": {"eth_output", "ip_output_drop"}}
# edges inside the replaced sub-graph, walked by the kernel (fwd4_chain.h)
INTERNAL = {("iface_input", "eth_input"), ("eth_input", "ip_input"), ("eth_input", "ip6_input"),
            ("ip_input", "ip_forward"), ("ip_input", "ip_output"), ("ip_forward", "ip_output"),
            ("ip_output", "eth_output"), ("eth_output", "iface_output"), ("ip6_input", "ip6_forward"),
            ("ip6_input", "ip6_output"), ("ip6_forward", "ip6_output"), ("ip6_output", "eth_output")}


def fixture():
    with open(os.path.join(HERE, "golden", "graph_svg.json")) as f:
        return json.load(f)


def edges():
    return [tuple(e.split(" -> ")) for e in fixture()["edges"]]


@pytest.mark.skipif(not os.path.isfile(REF + "/docs/graph.svg"), reason="reference not mounted")
def test_fixture_is_the_reference_graph():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_graph_svg", os.path.join(HERE, "golden", "make_graph_svg.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.build(REF) == fixture()


def test_edges_leaving_the_replaced_nodes_are_verdicts():
    names = set(abi.EDGE_NAMES)
    via = {}
    for a, b in edges():
        if a not in REPLACED:
            continue
        if b in REPLACED:
            assert (a, b) in INTERNAL, (a, b)
            continue
        if b in names:
            continue
        cont = [c for c, after in CONTINUATIONS.items() if b in after and c in names]
        assert cont, "%s -> %s: neither a verdict edge nor behind a continuation node" % (a, b)
        via[(a, b)] = cont[0]
    assert via == {("ip_input", "dnat44_dynamic"): "ip_input_local_ct"}  # conntrack hit (ip_input.c:170-185)
    # and the kernel walks every internal edge the graph documents
    documented = {(a, b) for a, b in edges() if a in REPLACED and b in REPLACED}
    assert documented == INTERNAL


def test_verdict_edges_name_grout_nodes():
    fx = fixture()
    grout = set(fx["nodes"]) | set(fx["registered"])
    ours = {"iface_input_cpu"} | set(CONTINUATIONS)  # grout's iface_input renamed; the continuation nodes
    for e in abi.EDGE_NAMES:
        name = "iface_input_cpu" if e == "punt" else e
        assert name in grout or name in ours, name
    # every edge of the documented graph out of the replaced nodes has a verdict or a continuation
    out = {b for a, b in edges() if a in REPLACED and b not in REPLACED}
    assert out <= set(abi.EDGE_NAMES) | set().union(*CONTINUATIONS.values())


def test_node_edges_match_the_fixture():
    """The compiled node's next nodes (libgrout_gpu_fwd4.so, loaded by the stand-in library) carry those names."""
    from test_graph_walk import edges_of, lib
    assert lib().gh_register() == 0
    got = edges_of("iface_input")
    assert got[0] == "iface_input_cpu" and got[1:] == abi.EDGE_NAMES[1:]
    for c, after in CONTINUATIONS.items():
        assert after <= set(edges_of(c)), c
