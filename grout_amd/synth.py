# SPDX-License-Identifier: BSD-3-Clause
"""Synthetic packet streams and hand-crafted frames."""
import ctypes
import ipaddress

import numpy as np

from . import abi
from .topology import PORT_IFACE, PORT_MAC, SRC_MAC, mac_bytes

SEED_SINGLE = 0x67720001
SEED_FULLVIEW = 0x67720002
SEED_IMIX = 0x67720003
SEED_FULLVIEW6 = 0x67720006
SEED_GPU_BASE = 0x67721000

DST_RANGE, DST_ROUTES = 0, 1
SIZE_64, SIZE_IMIX = 0, 1


def stream(n, seed, *, routes=None, dst_range=None, imix=False, stride=64, lines_only=False,
           in_iface=PORT_IFACE[0], dst_mac=PORT_MAC[0], src_mac=SRC_MAC, ttl=64):
    """n frames (n x stride bytes) and their metadata, from the C generator."""
    s = abi.SynthStream()
    s.seed = seed
    s.size_mode = SIZE_IMIX if imix else SIZE_64
    keep = None
    if routes is not None:
        keep = np.ascontiguousarray(routes, dtype=abi.ROUTE_DT)
        s.dst_mode = DST_ROUTES
        s.routes = keep.ctypes.data
        s.n_routes = len(keep)
    else:
        lo, hi = dst_range
        s.dst_mode = DST_RANGE
        s.dst_lo, s.dst_hi = lo, hi
    s.in_iface = in_iface
    s.dst_mac[:] = list(mac_bytes(dst_mac))
    s.src_mac[:] = list(mac_bytes(src_mac))
    s.ttl = ttl
    frames = np.zeros((n, stride), dtype=np.uint8)
    meta = np.zeros(n, dtype=abi.META_DT)
    abi.check("gr_synth_packets", abi.host().gr_synth_packets(
        ctypes.byref(s), n, stride, 1 if lines_only else 0, frames.ctypes.data, meta.ctypes.data))
    return frames, meta


def ip4_cksum(hdr):
    """RFC 791 header checksum of bytes `hdr` (checksum field treated as 0)."""
    b = bytearray(hdr)
    b[10:12] = b"\0\0"
    s = sum(int.from_bytes(b[i:i + 2], "big") for i in range(0, len(b), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def frame(dst_mac=PORT_MAC[0], src_mac=SRC_MAC, ethertype=0x0800, *, version=4, ihl=5, tos=0,
          total_len=None, ident=1, flags_frag=0, ttl=64, proto=17, src="198.18.0.1",
          dst="16.1.0.1", cksum=None, options=b"", payload_len=None, length=60, raw=None):
    """One Ethernet/IPv4 frame as bytes (length = bytes in buffer, >= 14)."""
    if raw is not None:
        return bytes(raw)
    eth = mac_bytes(dst_mac) + mac_bytes(src_mac) + ethertype.to_bytes(2, "big")
    hl = ihl * 4
    if total_len is None:
        total_len = max(length - 14, 20)
    ip = bytearray(max(hl, 20))
    ip[0] = ((version & 0xF) << 4) | (ihl & 0xF)
    ip[1] = tos
    ip[2:4] = (total_len & 0xFFFF).to_bytes(2, "big")
    ip[4:6] = ident.to_bytes(2, "big")
    ip[6:8] = flags_frag.to_bytes(2, "big")
    ip[8] = ttl & 0xFF
    ip[9] = proto
    ip[12:16] = int(ipaddress.IPv4Address(src)).to_bytes(4, "big")
    ip[16:20] = int(ipaddress.IPv4Address(dst)).to_bytes(4, "big")
    if options:
        ip[20:20 + len(options)] = options
    if cksum is None:
        c = ip4_cksum(bytes(ip[:hl])) if hl >= 2 else 0xFFFF
        ip[10:12] = c.to_bytes(2, "big")
    else:
        ip[10:12] = cksum.to_bytes(2, "big")
    f = eth + bytes(ip)
    if len(f) < length:
        f += bytes(length - len(f))
    return f[:max(length, 14)] if length >= len(eth) else f[:length]


def frame6(dst_mac=PORT_MAC[0], src_mac=SRC_MAC, ethertype=0x86DD, *, version=6, tc=0, flow=0,
           payload_len=None, next_header=17, hop=64, src="2001:db8:ff::1", dst="2001:db8:100::1",
           length=64):
    """One Ethernet/IPv6 frame as bytes (RFC 8200 header, zero payload)."""
    eth = mac_bytes(dst_mac) + mac_bytes(src_mac) + ethertype.to_bytes(2, "big")
    ip = bytearray(40)
    vtc = ((version & 0xF) << 28) | ((tc & 0xFF) << 20) | (flow & 0xFFFFF)
    ip[0:4] = vtc.to_bytes(4, "big")
    if payload_len is None:
        payload_len = max(length - 54, 0)
    ip[4:6] = (payload_len & 0xFFFF).to_bytes(2, "big")
    ip[6] = next_header
    ip[7] = hop & 0xFF
    ip[8:24] = ipaddress.IPv6Address(src).packed
    ip[24:40] = ipaddress.IPv6Address(dst).packed
    f = eth + bytes(ip)
    if len(f) < length:
        f += bytes(length - len(f))
    return f[:length]


def stream6(n, seed, routes6, *, stride=64, in_iface=PORT_IFACE[0], dst_mac=PORT_MAC[0], src_mac=SRC_MAC,
            hop=64, pkt_len=64):
    """n IPv6 frames: dst = a uniformly picked route, random host bits under
    its mask (the IPv6 analogue of SURVEY.md §8d's full-view stream); src from
    2001:db8:ff::/48, hop limit `hop`, UDP next header, random rss."""
    rng = np.random.default_rng(seed)
    r = np.ascontiguousarray(routes6, dtype=abi.ROUTE6_DT)
    pick = rng.integers(0, len(r), size=n)
    pfx = r["ip"][pick]  # n x 16
    plen = r["prefixlen"][pick].astype(np.int32)
    host = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    bits = np.arange(16)[None, :] * 8
    keep = np.clip(plen[:, None] - bits, 0, 8)  # prefix bits per byte
    mask = (0xFF00 >> keep).astype(np.uint8)
    dst = (pfx & mask) | (host & ~mask)
    frames = np.zeros((n, stride), dtype=np.uint8)
    frames[:, 0:6] = np.frombuffer(mac_bytes(dst_mac), np.uint8)
    frames[:, 6:12] = np.frombuffer(mac_bytes(src_mac), np.uint8)
    frames[:, 12] = 0x86
    frames[:, 13] = 0xDD
    frames[:, 14] = 0x60
    payload = max(pkt_len - 54, 0)
    frames[:, 18] = payload >> 8
    frames[:, 19] = payload & 0xFF
    frames[:, 20] = 17
    frames[:, 21] = hop
    frames[:, 22:38] = np.frombuffer(ipaddress.IPv6Address("2001:db8:ff::").packed, np.uint8)
    frames[:, 32:38] = rng.integers(0, 256, size=(n, 6), dtype=np.uint8)
    frames[:, 38:54] = dst
    meta = np.zeros(n, dtype=abi.META_DT)
    meta["iface"] = in_iface
    meta["pkt_len"] = pkt_len
    meta["rss"] = rng.integers(0, 65536, size=n, dtype=np.uint16)
    return frames, meta


def pack(frames, stride=64, iface=PORT_IFACE[0], vlan=0, ck=abi.CKSUM_UNKNOWN, rss=0, pkt_lens=None):
    """List of frame bytes -> (n x stride frames array, meta)."""
    n = len(frames)
    arr = np.zeros((n, stride), dtype=np.uint8)
    meta = np.zeros(n, dtype=abi.META_DT)
    for i, f in enumerate(frames):
        b = np.frombuffer(f[:stride], np.uint8)
        arr[i, :len(b)] = b
        meta[i]["iface"] = iface[i] if isinstance(iface, (list, np.ndarray)) else iface
        v = vlan[i] if isinstance(vlan, (list, np.ndarray)) else vlan
        c = ck[i] if isinstance(ck, (list, np.ndarray)) else ck
        meta[i]["vlan_ck"] = (v & 0xFFF) | (c << 12)
        meta[i]["pkt_len"] = pkt_lens[i] if pkt_lens is not None else len(f)
        meta[i]["rss"] = rss[i] if isinstance(rss, (list, np.ndarray)) else rss
    return arr, meta
