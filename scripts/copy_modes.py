"""Streaming copy: one wave loads and stores (membench mode 3) against loads
and stores in different waves (mode 7), interleaved rounds, median GB/s of
read + write.  python scripts/copy_modes.py [GiB]"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    nbytes = gib << 30
    buf = devmem.DeviceBuffer(eng, nbytes)
    buf.zero()
    res = {3: [], 7: []}
    for _ in range(5):
        for mode in (3, 7):
            ms = ctypes.c_double()
            _lib.check_diag(D.rsk_diag_membench(eng.ctx, mode, buf.ptr, nbytes, 0, ctypes.byref(ms)))
            res[mode].append(nbytes / ms.value / 1e6)
    for mode, v in res.items():
        print("mode %d (%s): median %.0f GB/s, max %.0f" % (mode, "one wave loads and stores" if mode == 3 else
                                                          "split waves", statistics.median(v), max(v)), flush=True)
    buf.free()


if __name__ == "__main__":
    main()
