#!/usr/bin/env python3
"""What the HIP runtime reports for host memory that was registered and then
unregistered (round 5's illegal-address fault).

No copy and no kernel touches the memory under test: the probe only asks
hipPointerGetAttributes / hipHostGetDevicePointer and our own library's
registry (gr_hip_host_dev_addr) about each address, after each step:

  fresh        a numpy buffer never registered
  registered   gr_hip_host_register (context A)
  unregistered gr_hip_host_unregister (context A)
  reused       the buffer freed and a new one of the same size allocated
               (same virtual address when the allocator hands it back)
  unaligned    a buffer whose data pointer is not page-aligned, registered and
               unregistered: the page base and the last page asked as well
  two_ctx      contexts A and B register the same buffer (B finds it pinned
               and records A's device address), A unregisters: what B's
               registry and the runtime then say

One JSON line per step on stdout.
"""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from grout_amd import abi  # noqa: E402
from grout_amd.fwd import FastPath  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def attrs(p):
    a = Attr()
    e = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    if e:
        hip.hipGetLastError()
    dp = ctypes.c_void_p()
    e2 = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(p), 0)
    if e2:
        hip.hipGetLastError()
    return dict(err=e, type=a.type, dev=a.devicePointer or 0, host=a.hostPointer or 0, flags=a.allocationFlags,
                hgdp_err=e2, hgdp=dp.value or 0)


def our_addr(fp, p):
    d = ctypes.c_uint64()
    r = fp.lib.gr_hip_host_dev_addr(fp.h, ctypes.c_void_p(p), ctypes.byref(d))
    return r if r < 0 else d.value


def emit(step, **kw):
    print(json.dumps(dict(step=step, **kw)), flush=True)


def main():
    n = 32 << 20
    A = FastPath()
    B = FastPath()
    x = np.zeros(n, np.uint8)
    px = x.ctypes.data
    emit("fresh", ptr=px, page_off=px & 4095, attrs=attrs(px))
    abi.check("gr_hip_host_register", A.lib.gr_hip_host_register(A.h, ctypes.c_void_p(px), n))
    emit("registered", attrs=attrs(px), attrs_last=attrs(px + n - 1), ours_A=our_addr(A, px))
    abi.check("gr_hip_host_unregister", A.lib.gr_hip_host_unregister(A.h, ctypes.c_void_p(px)))
    emit("unregistered", attrs=attrs(px), attrs_base=attrs(px & ~4095), attrs_last=attrs(px + n - 1),
         ours_A=our_addr(A, px))
    del x
    y = np.zeros(n, np.uint8)
    py = y.ctypes.data
    emit("reused", ptr=py, same_va=py == px, attrs=attrs(py), attrs_last=attrs(py + n - 1))
    # a sub-range of the reused buffer registered again, then the whole of it
    abi.check("gr_hip_host_register", A.lib.gr_hip_host_register(A.h, ctypes.c_void_p(py), n))
    emit("re_registered", attrs=attrs(py), ours_A=our_addr(A, py))
    abi.check("gr_hip_host_unregister", A.lib.gr_hip_host_unregister(A.h, ctypes.c_void_p(py)))
    emit("re_unregistered", attrs=attrs(py))
    del y

    # two contexts, one buffer
    z = np.zeros(n, np.uint8)
    pz = z.ctypes.data
    abi.check("gr_hip_host_register", A.lib.gr_hip_host_register(A.h, ctypes.c_void_p(pz), n))
    rb = B.lib.gr_hip_host_register(B.h, ctypes.c_void_p(pz), n)
    emit("two_ctx_registered", rb=rb, attrs=attrs(pz), ours_A=our_addr(A, pz), ours_B=our_addr(B, pz))
    abi.check("gr_hip_host_unregister", A.lib.gr_hip_host_unregister(A.h, ctypes.c_void_p(pz)))
    emit("two_ctx_A_unregistered", attrs=attrs(pz), ours_A=our_addr(A, pz), ours_B=our_addr(B, pz))
    rb2 = B.lib.gr_hip_host_unregister(B.h, ctypes.c_void_p(pz))
    emit("two_ctx_B_unregistered", rb=rb2, attrs=attrs(pz), ours_B=our_addr(B, pz))
    del z
    B.close()
    A.close()


if __name__ == "__main__":
    main()
