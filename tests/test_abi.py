# SPDX-License-Identifier: BSD-3-Clause
"""The C-ABI library loads and exports every symbol include/grout_hip.h
declares (no device calls: this runs without a GPU)."""
import pytest
import ctypes
import os
import re
import subprocess

from grout_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(ROOT, header)).read()
    return sorted(set(re.findall(r"^\w[\w \*]*?\b(gr_hip_\w+)\s*\(", text, re.M)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_symbols_exported():
    names = declared("include/grout_hip.h")
    assert len(names) >= 30
    syms = exported(abi.LIB_HIP)
    missing = [n for n in names if n not in syms]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(declared("include/grout_hip.h")) == set(abi.HIP_API)


def test_library_loads_and_reports_abi():
    lib = abi.hip()
    assert lib.gr_hip_abi_version() == abi.ABI_VERSION == 3
    assert isinstance(ctypes.CDLL(abi.LIB_HIP), ctypes.CDLL)


def test_init_without_gpu_fails_cleanly():
    """No device here: init must return -errno, never abort."""
    import torch
    if torch.cuda.is_available():
        return
    h = ctypes.c_void_p()
    r = abi.hip().gr_hip_init(0, 1024, 1024, ctypes.byref(h))
    assert r < 0 and not h.value


def test_code_object_is_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", abi.LIB_HIP], capture_output=True, text=True)
    blob = open(abi.LIB_HIP, "rb").read()
    assert b"gfx950" in blob, out.stdout[:200]


def test_struct_sizes_match_header():
    # sizes asserted in abi.py; check the edge enum count against the header
    text = open(os.path.join(ROOT, "include/grout_hip.h")).read()
    body = text[text.index("enum gr_hip_edge {"):text.index("GR_HIP_E_COUNT")]
    assert len(re.findall(r"\bGR_HIP_E_\w+", body)) == abi.E_COUNT


def test_queue_refuses_null_stream():
    """A queue never silently gets a private stream when the caller meant to
    share torch's default (null) stream."""
    from grout_amd.fwd import Queue

    class _FP:
        lib = None
        h = None

    with pytest.raises(ValueError):
        Queue(_FP(), 0)


def test_product_fails_loudly_without_the_hip_library(monkeypatch):
    """No fallback: without libgrout_hip.so the package refuses to run (the
    oracle is never a stand-in for the product path)."""
    from grout_amd import abi as A
    monkeypatch.setattr(A, "LIB_HIP", "/nonexistent/libgrout_hip.so")
    monkeypatch.setattr(A, "_hip", None)
    with pytest.raises(ImportError, match="not built"):
        A.hip()
    from grout_amd.fwd import FastPath
    with pytest.raises(ImportError):
        FastPath(0)
