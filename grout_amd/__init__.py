# SPDX-License-Identifier: BSD-3-Clause
"""MI355X-native IPv4 forwarding fast path for grout (DPDK graph router).

grout_amd.fwd.FastPath drives libgrout_hip.so (include/grout_hip.h); the
topology / synth modules build grout-shaped control-plane objects and
synthetic packet streams. Importing this package does not load the HIP
library; constructing a FastPath does, and raises if it is not built.
"""
from . import abi  # noqa: F401

__all__ = ["abi", "fwd", "topology", "synth"]
