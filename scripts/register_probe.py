"""Cost of pinning a pageable host buffer in place (hipHostRegister) and the
D2H rate into it, against the staged path's legs: a 2.12 GB numpy buffer
(the C5 checkpoint's size), pages touched first.  One JSON line."""
import ctypes
import json
import time

import numpy as np

H = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
H.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
H.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
H.hipHostUnregister.argtypes = [ctypes.c_void_p]
H.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
H.hipDeviceSynchronize.argtypes = []


def main():
    n = 2_120_000_000
    buf = np.empty(n, np.uint8)
    buf[::4096] = 1  # touch
    d = ctypes.c_void_p()
    assert H.hipMalloc(ctypes.byref(d), n) == 0
    res = {}
    for rep in range(3):
        t0 = time.perf_counter()
        rc = H.hipHostRegister(buf.ctypes.data, n, 0)
        t1 = time.perf_counter()
        assert rc == 0, rc
        H.hipMemcpy(buf.ctypes.data, d, n, 2)  # D2H
        t2 = time.perf_counter()
        H.hipMemcpy(d, buf.ctypes.data, n, 1)  # H2D
        t3 = time.perf_counter()
        H.hipHostUnregister(buf.ctypes.data)
        t4 = time.perf_counter()
        res.setdefault("register_ms", []).append((t1 - t0) * 1e3)
        res.setdefault("d2h_GBps", []).append(n / (t2 - t1) / 1e9)
        res.setdefault("h2d_GBps", []).append(n / (t3 - t2) / 1e9)
        res.setdefault("unregister_ms", []).append((t4 - t3) * 1e3)
    t0 = time.perf_counter()
    H.hipMemcpy(buf.ctypes.data, d, n, 2)  # D2H pageable (the runtime's own staging)
    res["d2h_pageable_GBps"] = n / (time.perf_counter() - t0) / 1e9
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
