# SPDX-License-Identifier: BSD-3-Clause
"""The product's host RIB + DIR24_8 painter (grout_amd/csrc/fib4.c) against
the oracle's longest-prefix match, on CPU: random add / replace / delete
sequences, tbl8 exhaustion, and the 1M-route full view of fib_inject."""
import ctypes

import numpy as np
import pytest

import oracle
from grout_amd import abi
from grout_amd import topology as T


class HostFib:
    def __init__(self, max_routes=1 << 20, num_tbl8=256):
        self.L = abi.host()
        self.h = self.L.gr_fib4_new(max_routes, num_tbl8)
        assert self.h

    def __del__(self):
        self.L.gr_fib4_free(self.h)

    def add(self, ip, ln, nh, replace=False):
        return self.L.gr_fib4_add(self.h, ip, ln, nh, 1 if replace else 0)

    def delete(self, ip, ln):
        return self.L.gr_fib4_del(self.h, ip, ln)

    def lookup(self, ip):
        return self.L.gr_fib4_lookup(self.h, ip)

    def tables(self):
        t24 = np.ctypeslib.as_array(ctypes.cast(self.L.gr_fib4_tbl24(self.h), ctypes.POINTER(ctypes.c_uint32)),
                                    shape=(1 << 24,))
        n8 = self.L.gr_fib4_num_tbl8(self.h)
        t8 = np.ctypeslib.as_array(ctypes.cast(self.L.gr_fib4_tbl8(self.h), ctypes.POINTER(ctypes.c_uint32)),
                                   shape=(n8 * 256,))
        return t24, t8


def vec_lookup(t24, t8, ips):
    e = t24[ips >> 8]
    ext = (e & 0x80000000) != 0
    out = e.copy()
    out[ext] = t8[(e[ext] & 0x7FFFFFFF).astype(np.int64) * 256 + (ips[ext] & 0xFF)]
    return out


def mask(ln):
    return 0 if ln == 0 else ((1 << 32) - 1) ^ ((1 << (32 - ln)) - 1)


def oracle_for(routes):
    t = T.base_ports(max_routes=1 << 20, num_tbl8=4096)
    for k in range(40):
        t.add_nexthop(T.PORT_IFACE[1], f"172.16.1.{k + 2}", "02:00:00:01:00:2d")
    for (ip, ln), nh in routes.items():
        t.add_route(1, f"{T.ipaddress.IPv4Address(ip)}/{ln}", nh)
    return oracle.Oracle(t, build_dir24=False)


def probes_for(routes, rng, n=4000):
    p = [int(x) for x in rng.integers(0, 2**32, n)]
    for ip, ln in list(routes)[:500]:
        p += [ip, ip + (1 << (32 - ln)) - 1, (ip - 1) & 0xFFFFFFFF, (ip + (1 << (32 - ln))) & 0xFFFFFFFF]
    return p


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_add_replace_delete(seed):
    rng = np.random.default_rng(seed)
    fib = HostFib(num_tbl8=512)
    routes = {}
    lens = [0, 1, 4, 8, 12, 15, 16, 20, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32]
    base = int(rng.integers(0, 2**32)) & 0xFF000000
    for step in range(1500):
        ln = int(rng.choice(lens))
        # cluster addresses so prefixes overlap a lot
        ip = (base | int(rng.integers(0, 1 << 20)) << 4) & mask(ln) if ln >= 8 else \
            int(rng.integers(0, 2**32)) & mask(ln)
        op = rng.random()
        if op < 0.65:
            nh = int(rng.integers(1, 40))
            r = fib.add(ip, ln, nh, replace=bool(rng.random() < 0.5))
            if (ip, ln) in routes and r == -17:  # -EEXIST without replace
                continue
            assert r == 0, (step, ip, ln, r)
            routes[(ip, ln)] = nh
        elif routes:
            k = list(routes)[int(rng.integers(0, len(routes)))]
            assert fib.delete(*k) == 0
            del routes[k]
        else:
            assert fib.delete(ip, ln) == -2  # -ENOENT
        if step % 250 == 249:
            o = oracle_for(routes)
            for p in probes_for(routes, rng, 1000):
                assert fib.lookup(p) == o.lpm(1, p, "hash"), (step, hex(p))
    o = oracle_for(routes)
    for p in probes_for(routes, rng):
        assert fib.lookup(p) == o.lpm(1, p, "hash"), hex(p)
    # delete everything: the table must return to empty and free every tbl8
    for k in list(routes):
        assert fib.delete(*k) == 0
    t24, _ = fib.tables()
    assert not t24.any()
    assert fib.L.gr_fib4_tbl8_used(fib.h) == 0
    assert fib.L.gr_fib4_n_routes(fib.h) == 0


def test_exists_and_replace():
    fib = HostFib()
    assert fib.add(T.ip4("10.0.0.0"), 8, 3) == 0
    assert fib.add(T.ip4("10.1.2.3"), 8, 4) == -17  # host bits masked: same prefix
    assert fib.lookup(T.ip4("10.9.9.9")) == 3
    assert fib.add(T.ip4("10.0.0.0"), 8, 4, replace=True) == 0
    assert fib.lookup(T.ip4("10.9.9.9")) == 4
    assert fib.delete(T.ip4("10.0.0.0"), 9) == -2
    assert fib.delete(T.ip4("10.0.0.0"), 8) == 0
    assert fib.lookup(T.ip4("10.9.9.9")) == 0


def test_tbl8_exhaustion_is_atomic():
    fib = HostFib(num_tbl8=4)
    for k in range(4):
        assert fib.add(T.ip4(f"10.0.{k}.1"), 32, 5) == 0
    assert fib.L.gr_fib4_tbl8_used(fib.h) == 4
    assert fib.add(T.ip4("10.0.9.1"), 32, 6) == -28  # -ENOSPC, like rte_fib_add
    assert fib.lookup(T.ip4("10.0.9.1")) == 0
    assert fib.L.gr_fib4_n_routes(fib.h) == 4
    assert fib.add(T.ip4("10.0.0.0"), 16, 7) == 0
    assert fib.lookup(T.ip4("10.0.9.1")) == 7
    assert fib.lookup(T.ip4("10.0.1.1")) == 5
    assert fib.lookup(T.ip4("10.0.1.2")) == 7


def test_max_routes():
    fib = HostFib(max_routes=3)
    for k in range(3):
        assert fib.add(T.ip4(f"10.{k}.0.0"), 16, 1) == 0
    assert fib.add(T.ip4("10.9.0.0"), 16, 1) == -28
    assert fib.add(T.ip4("10.0.0.0"), 16, 2, replace=True) == 0


def test_fullview_matches_oracle():
    """1M fib_inject routes: every packet destination and 2M random IPs."""
    t = T.config_fullview()
    routes = t.route_array()
    fib = HostFib(max_routes=len(routes) + 10, num_tbl8=max(256, (len(routes) + 10) // 500))
    for r in routes:
        assert fib.add(int(r["ip"]), int(r["prefixlen"]), int(r["nh"])) == 0
    o = oracle.Oracle(t)
    t24, t8 = fib.tables()
    rng = np.random.default_rng(11)
    ips = rng.integers(0, 1 << 32, 1 << 21, dtype=np.uint64).astype(np.uint32)
    sel = routes[rng.integers(0, len(routes), 1 << 20)]
    m = np.array([mask(int(x)) for x in range(33)], dtype=np.uint64)
    host_ips = ((sel["ip"].astype(np.uint64) & m[sel["prefixlen"]]) |
                (rng.integers(0, 1 << 32, len(sel), dtype=np.uint64) & ~m[sel["prefixlen"]] & 0xFFFFFFFF))
    ips = np.concatenate([ips, host_ips.astype(np.uint32)])
    got = vec_lookup(t24, t8, ips)
    # oracle DIR24_8 restatement (cross-checked against brute force in the KAT)
    want = np.array([o.lpm(1, int(i), "dir24") for i in ips[:200000]], dtype=np.uint32)
    assert np.array_equal(got[:200000], want)
    want2 = np.array([o.lpm(1, int(i), "dir24") for i in ips[-200000:]], dtype=np.uint32)
    assert np.array_equal(got[-200000:], want2)
    assert fib.L.gr_fib4_n_routes(fib.h) == len(routes)
