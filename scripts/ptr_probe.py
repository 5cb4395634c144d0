"""Prints what hipPointerGetAttributes says about a pageable numpy buffer and
a hipMalloc'd one (no kernel runs).  Exits 1 if a pageable pointer would NOT
be classified unregistered / invalid (then need_gpu_ptr would not reject it)."""
import ctypes
import sys

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")


class Attr(ctypes.Structure):  # hipPointerAttribute_t: type, device, devicePointer, hostPointer, isManaged, allocationFlags
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


a = np.zeros(1 << 20, np.uint8)
at = Attr()
rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(a.ctypes.data))
hip.hipGetLastError()
d = ctypes.c_void_p()
hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(1 << 20))
ad = Attr()
rcd = hip.hipPointerGetAttributes(ctypes.byref(ad), d)
print("pageable: rc=%d type=%d   device: rc=%d type=%d" % (rc, at.type, rcd, ad.type))
hip.hipFree(d)
sys.exit(0 if (rc != 0 or at.type == 0) and rcd == 0 and ad.type == 2 else 1)
