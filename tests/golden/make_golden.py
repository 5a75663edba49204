# SPDX-License-Identifier: BSD-3-Clause
"""Regenerate the golden fixtures (inputs + expected outputs) from the oracle.

    python tests/golden/make_golden.py

The reference cannot run here, so expected outputs come from
the oracle restatement; they are pinned by tests/test_oracle_kat.py (the
reference's own ip_input known answers and hand-derived cases). Fixtures:
  corpus.npz     every terminal edge (tests/scenarios.py), stride 128
  single.npz     config 2 stream, 2048 x 64 B
  fullview.npz   config 3 stream over the 1M-route view, 4096 x 64 B
  imix.npz       config 4 stream (IMIX), 512 packets, header lines only
  fullview6.npz  IPv6 stream over fib_inject -6's 200k-route view, 4096 x 64 B
  eth_cache.npz  graph walks through eth_output's source-MAC cache (corpus topology)
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
import scenarios as SC  # noqa: E402
from grout_amd import synth as S  # noqa: E402
from grout_amd import topology as T  # noqa: E402


def digest(t):
    h = hashlib.sha256()
    h.update(t.ifaces.tobytes())
    h.update(t.nh[:t.n_nh + 1].tobytes())
    h.update(t.reta.tobytes())
    h.update(t.route_array().tobytes())
    h.update(t.route6_array().tobytes())
    return h.hexdigest()


def save(name, t, frames, meta, labels=None, lines_only=False):
    out, v, st = oracle.Oracle(t).process(frames, meta, lines_only=lines_only)
    nz = np.nonzero(st["rx_packets"] | st["tx_packets"])[0]
    np.savez_compressed(os.path.join(HERE, name), frames=frames, meta=meta, out=out, verdicts=v,
                        stats_ifaces=nz, stats=st[nz], topo_sha256=np.array(digest(t)),
                        labels=np.array(labels if labels else [], dtype=object).astype(str),
                        lines_only=np.array(lines_only))


def main():
    t, _ = SC.corpus_topology()
    frames, meta, labels = SC.corpus_arrays()
    save("corpus.npz", t, frames, meta, labels)

    t = T.config_single_route()
    fr, me = S.stream(2048, S.SEED_SINGLE, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    save("single.npz", t, fr, me)

    t = T.config_fullview()
    fr, me = S.stream(4096, S.SEED_FULLVIEW, routes=t.route_array())
    save("fullview.npz", t, fr, me)

    fr, me = S.stream(512, S.SEED_IMIX, routes=t.route_array(), imix=True, lines_only=True)
    save("imix.npz", t, fr, me, lines_only=True)

    t = T.config_fullview6()
    fr, me = S.stream6(4096, S.SEED_FULLVIEW6, t.route6_array())
    save("fullview6.npz", t, fr, me)

    t, _ = SC.corpus_topology()
    frames, meta, labels, _ = SC.eth_output_cache_arrays()
    save("eth_cache.npz", t, frames, meta, labels)


if __name__ == "__main__":
    main()
