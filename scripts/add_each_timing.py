"""Times rsk_hll_add_each (PFADD with one reply per element) on 16M keys:
uniform distinct keys vs one key repeated (the skewed case the segmented
scan is for).  Prints one JSON line."""
import ctypes
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from redisson_amd import _lib, devmem  # noqa: E402

L = _lib.load()
eng = _lib.Engine.get(0)
n = 1 << 24
res = {}
uniform = devmem.gen_keys16(eng, 0x5EED0002, 0, n)
one = devmem.DeviceBuffer.from_numpy(eng, np.tile(uniform.to_numpy()[:16], n))
for name, buf in (("uniform", uniform), ("one_key", one)):
    kb = buf.keys_fixed(n, 16)
    ks = kb.as_struct()
    dout = devmem.DeviceBuffer.from_numpy(eng, np.zeros(n, np.uint8))  # replies follow the keys' location
    best = 1e9
    for _ in range(4):
        h = ctypes.c_void_p()
        _lib.check(L.rsk_hll_create(eng.ctx, 1, ctypes.byref(h)))
        eng.sync()
        t0 = time.perf_counter()
        _lib.check(L.rsk_hll_add_each(h, 0, ctypes.byref(ks), dout.ptr))
        eng.sync()
        best = min(best, time.perf_counter() - t0)
        L.rsk_hll_destroy(h)
    res[name] = {"ms": best * 1e3, "keys_per_s": n / best, "replies_1": int(dout.to_numpy().sum())}
print(json.dumps({"add_each_16M_keys_device_resident": res}))
