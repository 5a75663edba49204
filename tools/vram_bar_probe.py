#!/usr/bin/env python3
"""Can the host store straight into device memory here (a doorbell in VRAM the
resident kernel polls locally)? Each flag's allocation is asked
for its host-visible address (hipPointerGetAttributes), and a child process
stores a word through it and reads it back (a CPU fault ends only the child).
No kernel runs. One JSON line per allocation flag."""
import ctypes
import json
import os
import sys

hip = ctypes.CDLL("libamdhip64.so")
FLAGS = {"default": 0x0, "finegrained": 0x1, "uncached": 0x3}  # hipDeviceMallocDefault / Finegrained / Uncached


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def main():
    hip.hipSetDevice(0)
    for name, fl in FLAGS.items():
        p = ctypes.c_void_p()
        e = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(1 << 16), ctypes.c_uint(fl))
        a = Attr()
        ea = hip.hipPointerGetAttributes(ctypes.byref(a), p)
        res = dict(flag=name, alloc_err=e, attr_err=ea, type=a.type, dev=p.value or 0, host=a.hostPointer or 0)
        addr = a.hostPointer or p.value  # unified addressing: the device address itself, if the CPU maps it
        if e == 0 and addr:
            res["tried"] = "host" if a.hostPointer else "device_va"
            pid = os.fork()
            if pid == 0:  # child: no HIP call, a store and a load through the address
                q = ctypes.cast(addr, ctypes.POINTER(ctypes.c_uint64))
                q[0] = 0x1234567890ABCDEF
                os._exit(0 if q[0] == 0x1234567890ABCDEF else 3)
            _, st = os.waitpid(pid, 0)
            res["host_store"] = os.waitstatus_to_exitcode(st)
            back = ctypes.c_uint64()
            hip.hipMemcpy(ctypes.byref(back), p, ctypes.c_size_t(8), 2)  # D2H
            res["device_sees"] = hex(back.value)
        print(json.dumps(res), flush=True)
        if e == 0:
            hip.hipFree(p)


if __name__ == "__main__":
    main()
