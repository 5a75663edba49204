# SPDX-License-Identifier: BSD-3-Clause
"""The changes a grout maintainer makes to grout's own files, as committed
patches, applied to the reference tree in a dry run:

* integration/grout-gpu_module-build.patch adds modules/gpu to grout's build
  behind a meson option (-Dgrout_amd=<checkout>): its meson.build
  (grout_amd/module/meson.build) compiles the module's sources in place and
  links libgrout_hip.so; without the option grout builds as before;
* integration/grout-iface_input_cpu.patch names grout's iface_input node
  iface_input_cpu (the fast path's PUNT target) when the module is built;
* integration/grout-gpu_fwd4-datapath.patch adds datapath hooks to grout's
  worker loop (datapath.h, main_loop.c): the module registers them; grout
  without it runs as before;
* integration/grout-gpu_fwd4-control.patch adds grout's internal event
  channel (main/event.c) and pushes on it wherever grout changes a nexthop
  or a route without a public event, for the control-plane mirror
  (grout_amd/module/gpu_fwd4_control.c).

Each patch must apply cleanly. The module files include grout's and DPDK's
headers by name (the stand-ins' names here): each name is a file of grout's
tree that declares what the module uses, and the module compiles with
grout's own warning flags. Its library exports the module's API only."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
MOD = os.path.join(ROOT, "grout_amd", "module")
STANDIN_INC = os.path.join(ROOT, "tests", "standin", "include")
PATCHES = ["grout-gpu_module-build.patch", "grout-iface_input_cpu.patch", "grout-gpu_fwd4-datapath.patch",
           "grout-gpu_fwd4-control.patch"]
MODULE_SRC = ["gpu_fwd4_node.c", "gpu_fwd4_control.c", "gpu_fwd4_cpu_nodes.c"]
have_ref = pytest.mark.skipif(not os.path.isdir(REF + "/modules") or shutil.which("patch") is None,
                              reason="reference tree or patch(1) not available")


def _patch_ok(name):
    return subprocess.run(["patch", "-p1", "--dry-run", "-s", "-d", REF, "-i", os.path.join(ROOT, "integration", name)],
                          capture_output=True, text=True)


@have_ref
@pytest.mark.parametrize("name", PATCHES)
def test_patch_applies_to_grout(name):
    r = _patch_ok(name)
    assert r.returncode == 0, r.stdout + r.stderr


@have_ref
def test_patches_apply_together(tmp_path):
    """All four on one copy of the files they touch, in order."""
    text = "".join(open(os.path.join(ROOT, "integration", p)).read() for p in PATCHES)
    files = sorted(set(re.findall(r"^\+\+\+ b/(\S+)", text, re.M)))
    for f in files:
        src = os.path.join(REF, f)
        if os.path.exists(src):
            os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
            shutil.copy(src, tmp_path / f)
    for p in PATCHES:
        r = subprocess.run(["patch", "-p1", "-s", "-d", str(tmp_path), "-i", os.path.join(ROOT, "integration", p)],
                           capture_output=True, text=True)
        assert r.returncode == 0, (p, r.stdout + r.stderr)
    # the module's build file as the patch creates it is the repo's own
    assert open(tmp_path / "modules/gpu/meson.build").read() == open(os.path.join(MOD, "meson.build")).read()


def test_build_patch_binds_the_module():
    text, added = _added("grout-gpu_module-build.patch")
    assert "+++ b/modules/gpu/meson.build" in text
    assert re.search(r"^\+subdir\('gpu'\)$", text, re.M)
    assert "'grout_amd', type: 'string', value: ''" in added  # off unless given
    assert "gpu_deps = []" in added and "+ gpu_deps," in added
    meson = open(os.path.join(MOD, "meson.build")).read()
    assert "if grout_amd_dir != ''" in meson and "find_library(\n    'grout_hip'" in meson
    for f in MODULE_SRC:  # the sources it compiles are the module's
        assert "'%s'" % f in meson and os.path.exists(os.path.join(MOD, f)), f
    # the flag the iface_input patch keys on is the one the build sets
    assert "grout_cflags += ['-DGR_GPU_FWD4']" in meson
    _, ii = _added("grout-iface_input_cpu.patch")
    assert "#ifdef GR_GPU_FWD4" in ii and '"iface_input_cpu"' in ii and '#define IFACE_INPUT_NODE "iface_input"' in ii


def test_datapath_patch_adds_hooks_not_module_calls():
    """grout's worker loop calls registered hooks, never the module: grout
    without modules/gpu builds and runs as before. The hooks are called where
    the module needs them, and the stand-in's declaration (which the module
    compiles against here) is the patch's."""
    text, added = _added("grout-gpu_fwd4-datapath.patch")
    assert not re.search(r"gpu_fwd4|GPU_FWD4", added)
    assert "void gr_datapath_hooks_register(struct gr_datapath_hooks *);" in added
    # graph_leave before the worker leaves its graph (reconfiguration, shutdown)
    assert re.search(r"if \(atomic_load\(&w->shutdown\) \|\| atomic_load\(&w->next_config\) != cur\) \{\n"
                     r"(\+[^\n]*\n)*\+\s*int n = hook->graph_leave \? hook->graph_leave\(graph\) : 0;\n"
                     r"(\+[^\n]*\n)* \s*worker_active_dec\(\);", text)
    # stats_flush at the housekeeping tick, right after rte_graph's own counters,
    # and what the hooks' nodes hold summed there
    assert re.search(r"\n \s*rte_graph_cluster_stats_get\(ctx\.stats, false\);\n\+\s*held = 0;\n\+\s*STAILQ_FOREACH "
                     r"\(hook, &datapath_hooks, next\) \{\n\+\s*if \(hook->stats_flush != NULL\)\n\+\s*hook->stats_flush\("
                     r"graph, rte_lcore_id\(\), hook_node_stats, &ctx\);\n(\+[^\n]*\n)*\+\s*held \+= "
                     r"hook->holding\(graph\);", text)
    # a window whose nodes hold packets is not idle: no micro-sleep, no block
    # on RX interrupts (main_loop.c:478-508)
    assert re.search(r"\n\+\s*if \(ctx\.last_count == 0 && held == 0\n \s*&& \+\+airq_empty >= "
                     r"ADAPTIVE_IRQ_EMPTY_WINDOWS\) \{", text)
    assert re.search(r"\n\+\s*if \(ctx\.last_count \|\| held\)\n \s*airq_empty = 0;", text)
    assert re.search(r"\n\+\s*if \(ctx\.last_count == 0 && held == 0 && max_sleep_us > 0\) \{", text)
    assert "const uint32_t readers = RTE_MAX_LCORE + hooks_rcu_readers;" in added
    body = re.search(r"struct gr_datapath_hooks \{(.*?)\};", added, re.S).group(1)
    mine = re.search(r"struct gr_datapath_hooks \{(.*?)\};", open(os.path.join(STANDIN_INC, "gr_datapath_min.h")).read(),
                     re.S).group(1)
    strip = lambda b: [l.strip() for l in b.splitlines() if l.strip() and not l.strip().startswith("//")]
    assert strip(body) == strip(mine)
    # the module registers its hooks with what the node provides
    node = open(os.path.join(MOD, "gpu_fwd4_node.c")).read()
    assert "gr_datapath_hooks_register(&gpu_hooks);" in node
    assert ".graph_leave = gpu_fwd4_drain," in node and ".stats_flush = gpu_fwd4_stats_flush," in node
    assert ".holding = gpu_fwd4_holding," in node


def _quoted_includes(path):
    return re.findall(r'^#include "([^"]+)"', open(path).read(), re.M)


def test_module_includes_grouts_headers():
    """The module files include grout's headers by grout's names (no stand-in
    header name), each a stand-in here."""
    for f in MODULE_SRC:
        for h in _quoted_includes(os.path.join(MOD, f)):
            if h.startswith("gpu_fwd4_"):
                continue
            assert not h.endswith("_min.h"), (f, h)
            assert os.path.exists(os.path.join(STANDIN_INC, h)), (f, h)


# where grout declares what the module uses (file of grout's tree: symbols)
GROUT_DECLS = {
    "modules/infra/control/graph.h": ["GR_NODE_CTX_TYPE", "GR_NODE_REGISTER", "struct gr_node_info", "GR_NODE_T_L2"],
    "main/module.h": ["void module_register"],
    "modules/infra/datapath/rcu.h": ["gr_datapath_rcu"],
    "modules/infra/datapath/mbuf.h": ["GR_MBUF_PRIV_DATA_TYPE(mbuf_data", "gr_mbuf_is_traced"],
    "modules/infra/datapath/rxtx.h": ["GR_MBUF_PRIV_DATA_TYPE(iface_mbuf_data"],
    "modules/infra/datapath/eth.h": ["eth_domain_t", "eth_input_mbuf_data", "eth_output_mbuf_data"],
    "modules/infra/datapath/l3.h": ["l3_mbuf_data"],
    "modules/infra/control/iface.h": ["iface_get_stats", "int iface_get_eth_addr", "struct __rte_cache_aligned iface {"],
    "modules/infra/control/nexthop.h": ["nexthop_info_l3", "nexthop_info_group"],
    "main/event.h": ["void event_subscribe"],
    "modules/infra/control/vrf.h": ["iface_info_vrf"],
    "modules/infra/control/port.h": ["iface_info_port"],
    "modules/infra/control/vlan.h": ["iface_info_vlan"],
    "modules/policy/control/conntrack.h": ["gr_conn_parse_key", "gr_conn_lookup", "conn_mbuf_data"],
    "modules/policy/datapath/nat_datapath.h": ["snat44_process", "NAT_VERDICT_DROP"],
}


@have_ref
def test_grouts_headers_declare_what_the_module_uses():
    """Each header name the module includes is a file of grout's tree, and
    grout declares each symbol the module takes from it there (the control
    patch moves route4_event / route6_event into ip4.h / ip6.h, the datapath
    patch adds the hooks to datapath.h)."""
    names = set()
    for f in MODULE_SRC:
        names |= {h for h in _quoted_includes(os.path.join(MOD, f)) if not h.startswith("gpu_fwd4_")}
    found = {}
    for d in ("modules", "main"):
        for dp, _, fs in os.walk(os.path.join(REF, d)):
            for x in fs:
                if x in names:
                    found.setdefault(x, []).append(os.path.relpath(os.path.join(dp, x), REF))
    assert names <= set(found), names - set(found)
    for path, syms in GROUT_DECLS.items():
        assert os.path.basename(path) in names, path
        assert path in found[os.path.basename(path)], (path, found[os.path.basename(path)])
        text = open(os.path.join(REF, path)).read()
        for sym in syms:
            assert sym in text, (path, sym)
    _, ctl = _added("grout-gpu_fwd4-control.patch")
    assert "struct route4_event {" in ctl and "struct route6_event {" in ctl
    _, dp = _added("grout-gpu_fwd4-datapath.patch")
    assert "struct gr_datapath_hooks {" in dp


CLANG = "/opt/rocm/lib/llvm/bin/clang"
# grout's own C flags (meson.build: project_c_flags, add_project_arguments, optional_c_args, c_std)
GROUT_CFLAGS = ["-std=gnu2x", "-DALLOW_EXPERIMENTAL_API", "-D_GNU_SOURCE", "-fms-extensions", "-Wno-microsoft",
                "-Wmissing-prototypes", "-Wstrict-aliasing=2", "-fstrict-aliasing", "-Wcalloc-transposed-args",
                "-Wmissing-variable-declarations", "-Wno-format-truncation", "-DGR_GPU_FWD4"]


@pytest.mark.skipif(not os.path.exists(CLANG), reason="clang not available")
@pytest.mark.parametrize("src", MODULE_SRC)
def test_module_compiles_with_grouts_flags(src, tmp_path):
    flags = [x for x in GROUT_CFLAGS if x != "-Wcalloc-transposed-args"]  # not in this clang
    r = subprocess.run([CLANG] + flags + ["-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror", "-O2", "-fPIC",
                                          "-I" + os.path.join(ROOT, "include"), "-I" + MOD, "-I" + STANDIN_INC, "-c",
                                          os.path.join(MOD, src), "-o", str(tmp_path / "m.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_module_library_exports_its_api_only():
    """libgrout_gpu_fwd4.so, the module as built here, defines gpu_fwd4_*
    and nothing of grout's or DPDK's: those it leaves to grout (here: to the
    stand-in library that loads it)."""
    lib = os.path.join(ROOT, "grout_amd", "libgrout_gpu_fwd4.so")
    if not os.path.exists(lib) or shutil.which("nm") is None:
        pytest.skip("module library not built")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    syms = [l.split()[-1] for l in out.splitlines() if l.strip()]
    assert syms and all(x.startswith("gpu_fwd4_") for x in syms), [x for x in syms if not x.startswith("gpu_fwd4_")]
    und = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True, check=True).stdout
    assert "rte_node_from_name" in und and "module_register" in und  # grout's / DPDK's, left undefined


def _added(name):
    text = open(os.path.join(ROOT, "integration", name)).read()
    return text, "\n".join(l[1:] for l in text.splitlines() if l.startswith("+") and not l.startswith("+++"))


def test_control_patch_feeds_the_mirror():
    """Every event the patch pushes on the internal channel is one the mirror
    subscribes to there; the stand-in the tests drive pushes them at the same
    places (its "patch:" sites), with the same event objects."""
    text, added = _added("grout-gpu_fwd4-control.patch")
    pushed = set(re.findall(r"event_push_internal\((GR_EVENT_\w+)", added))
    assert pushed == {"GR_EVENT_NEXTHOP_NEW", "GR_EVENT_NEXTHOP_UPDATE", "GR_EVENT_NEXTHOP_DELETE",
                      "GR_EVENT_IP_ROUTE_ADD", "GR_EVENT_IP_ROUTE_DEL", "GR_EVENT_IP6_ROUTE_ADD",
                      "GR_EVENT_IP6_ROUTE_DEL", "GR_EVENT_NEXTHOP_PRE_DELETE"}, pushed
    mirror = open(os.path.join(MOD, "gpu_fwd4_control.c")).read()
    subs = mirror[mirror.index("obj_evs[] = {"):]
    subs = subs[:subs.index("};")]
    assert "event_subscribe_internal(obj_evs[k]" in mirror
    subscribed = set(re.findall(r"GR_EVENT_\w+", subs)) | set(
        re.findall(r"event_subscribe_internal\((GR_EVENT_\w+)", mirror))
    assert pushed <= subscribed, pushed - subscribed
    # the pre-delete event, before nexthop_destroy's synchronize, in the patch and the stand-in
    nh_hunk = text[text.index("+++ b/modules/infra/control/nexthop.c"):]
    assert nh_hunk.index("event_push_internal(GR_EVENT_NEXTHOP_PRE_DELETE") < nh_hunk.index(
        "rte_rcu_qsbr_synchronize(gr_datapath_rcu()")
    assert "#define GR_EVENT_NEXTHOP_PRE_DELETE GR_MSG_TYPE(GR_INFRA_MODULE, 0x30ff)" in added
    stand_in = open(os.path.join(ROOT, "tests", "standin", "gr_control_min.c")).read()
    assert pushed <= set(re.findall(r"event_push_internal\((GR_EVENT_\w+)", stand_in))
    # the internal channel's API and the event objects as the patch declares them
    hdr = open(os.path.join(STANDIN_INC, "gr_control_min.h")).read()
    for decl in ("void event_subscribe_internal(uint32_t ev_type, event_sub_cb_t callback);",
                 "void event_push_internal(uint32_t ev_type, const void *obj);"):
        assert decl in added and decl in hdr, decl
    for struct in ("route4_event", "route6_event"):
        body = re.search(r"struct %s \{(.*?)\};" % struct, added, re.S).group(1)
        fields = re.findall(r"(\w+);", body)
        mine = re.findall(r"(\w+);", re.search(r"struct %s \{(.*?)\};" % struct, hdr, re.S).group(1))
        assert fields == mine, (struct, fields, mine)
    # every INTERNAL-origin branch grout has for these events now pushes internally
    for f in ("modules/infra/control/nexthop.c", "modules/ip/control/route.c", "modules/ip6/control/route.c"):
        assert "+++ b/" + f in text, f


# ---- the stand-ins' prototypes against grout's and DPDK's ---------------------
# What the module calls that grout declares, and where (grout's tree, or the
# lines an integration patch adds).
GROUT_PROTOS = {
    "event_subscribe": "main/event.h",
    "event_subscribe_internal": "grout-gpu_fwd4-control.patch",
    "gr_conn_lookup": "modules/policy/control/conntrack.h",
    "gr_conn_parse_key": "modules/policy/control/conntrack.h",
    "gr_datapath_hooks_register": "grout-gpu_fwd4-datapath.patch",
    "gr_datapath_rcu": "modules/infra/datapath/rcu.h",
    "gr_mbuf_is_traced": "modules/infra/datapath/mbuf.h",
    "iface_get_eth_addr": "modules/infra/control/iface.h",
    "iface_get_stats": "modules/infra/control/iface.h",
    "module_register": "main/module.h",
    "snat44_process": "modules/policy/datapath/nat_datapath.h",
}
# DPDK 25.11 (subprojects/dpdk-25.11.wrap) and libevent 2.1 are not in the
# reference tree: their published prototypes, restated (inline?, return, params)
EXTERNAL_PROTOS = {
    "rte_graph_walk": (True, "void", ["struct rte_graph *"]),
    "rte_node_enqueue": (True, "void", ["struct rte_graph *", "struct rte_node *", "rte_edge_t", "void * *",
                                        "uint16_t"]),
    "rte_node_enqueue_x1": (True, "void", ["struct rte_graph *", "struct rte_node *", "rte_edge_t", "void *"]),
    "rte_node_from_name": (False, "rte_node_t", ["const char *"]),
    "rte_pktmbuf_free": (True, "void", ["struct rte_mbuf *"]),
    "rte_prefetch0": (True, "void", ["const volatile void *"]),
    "rte_rcu_qsbr_thread_online": (True, "void", ["struct rte_rcu_qsbr *", "unsigned int"]),
    "rte_rcu_qsbr_thread_offline": (True, "void", ["struct rte_rcu_qsbr *", "unsigned int"]),
    "rte_rcu_qsbr_thread_register": (False, "int", ["struct rte_rcu_qsbr *", "unsigned int"]),
    "rte_rcu_qsbr_thread_unregister": (False, "int", ["struct rte_rcu_qsbr *", "unsigned int"]),
    "event_new": (False, "struct event *", ["struct event_base *", "evutil_socket_t", "short", "event_callback_fn",
                                            "void *"]),
    "event_add": (False, "int", ["struct event *", "const struct timeval *"]),
    "event_del": (False, "int", ["struct event *"]),
    "event_free": (False, "void", ["struct event *"]),
}
_QUAL = {"const", "volatile", "struct", "enum", "union", "signed", "unsigned", "restrict"}
_STORAGE = {"static", "inline", "extern", "__rte_always_inline", "__rte_experimental"}


def _c_strip(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def _c_type(tokens):
    return " ".join(tokens)


def _c_param(p):
    toks = re.findall(r"\w+|\*", p)
    if len(toks) > 1 and re.match(r"\w+$", toks[-1]) and any(t == "*" or t not in _QUAL for t in toks[:-1]):
        toks = toks[:-1]  # the parameter's name
    return _c_type(toks)


def _c_proto(text, name):
    """(inline, return type, parameter types) of `name`'s declaration or
    definition in C text, or None."""
    m = re.search(r"^([ \t\w\*]*?)\b%s\s*\(([^()]*)\)\s*[;{]" % re.escape(name), _c_strip(text), re.M)
    if m is None:
        return None
    pre = re.findall(r"\w+|\*", m.group(1))
    inline = any(t in ("inline", "__rte_always_inline") for t in pre)
    ret = _c_type([t for t in pre if t not in _STORAGE])
    params = [_c_param(p) for p in m.group(2).split(",") if p.strip()]
    return inline, ret, params if params != ["void"] else []


def _module_calls():
    txt = _c_strip("".join(open(os.path.join(MOD, f)).read() for f in MODULE_SRC))
    return set(re.findall(r"\b([a-z_]\w*)\s*\(", txt))


def _standin_proto(name):
    for dp, _, fs in os.walk(STANDIN_INC):
        for f in sorted(fs):
            p = _c_proto(open(os.path.join(dp, f)).read(), name)
            if p is not None:
                return p
    return None


def test_standin_prototypes_parse():
    """The prototype reader on the forms grout writes (names or none, const
    typedefs, pointers, static inline, a declaration over several lines)."""
    assert _c_proto("static inline struct iface_stats *iface_get_stats(uint16_t lcore_id, uint16_t ifid) {",
                    "iface_get_stats") == (True, "struct iface_stats *", ["uint16_t", "uint16_t"])
    assert _c_proto("bool gr_conn_parse_key(\n\tconst struct iface *,\n\tconst addr_family_t,\n"
                    "\tconst struct rte_mbuf *,\n\tstruct conn_key *\n);", "gr_conn_parse_key") == (
        False, "bool", ["const struct iface *", "const addr_family_t", "const struct rte_mbuf *", "struct conn_key *"])
    assert _c_proto("struct rte_rcu_qsbr *gr_datapath_rcu(void);", "gr_datapath_rcu") == (
        False, "struct rte_rcu_qsbr *", [])


def test_standin_prototypes_match_grouts():
    """Every function the module calls that grout declares has, in the
    stand-ins it is compiled against here, grout's prototype: the same return
    type, parameter types, and static inline or not (iface.h:117-119,
    nat_datapath.h:57-67, conntrack.h:50-56, ...); every DPDK or libevent
    function it calls, the published prototype (EXTERNAL_PROTOS). A mismatch
    would otherwise surface only when a grout maintainer builds the module."""
    calls = _module_calls()
    for name, where in sorted(GROUT_PROTOS.items()):
        assert name in calls, name  # the table lists only what the module uses
        mine = _standin_proto(name)
        assert mine is not None, name
        if where.endswith(".patch"):
            theirs = _c_proto(_added(where)[1], name)
        elif os.path.isdir(REF + "/modules"):
            theirs = _c_proto(open(os.path.join(REF, where)).read(), name)
        else:
            continue  # the reference tree is not mounted: nothing to compare with
        assert theirs is not None, (name, where)
        assert mine == theirs, (name, where, mine, theirs)
    for name, want in sorted(EXTERNAL_PROTOS.items()):
        mine = _standin_proto(name)
        assert mine is not None, name
        assert mine == want, (name, mine, want)
    # every DPDK / libevent function the module calls is in the table
    ext = {c for c in calls if c.startswith(("rte_", "event_"))} - set(GROUT_PROTOS)
    ext -= {"rte_pktmbuf_mtod"}  # a macro in DPDK and here
    assert ext <= set(EXTERNAL_PROTOS), ext - set(EXTERNAL_PROTOS)
