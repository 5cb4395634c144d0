"""Random 4-byte gather rate against table size (membench mode 1): the
add()-with-replies reply pass gathers from a 4 B-per-bit first-key table
(38 GB at C3); a 1 B-per-bit table would be 9.6 GB.  Interleaved rounds,
median gathers/s.  python scripts/gather_sizes.py"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402


def main():
    _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    sizes = [1_198_132_298, 4_792_529_192, 9_585_058_377, 19_170_116_754, 38_340_233_508]
    buf = devmem.DeviceBuffer(eng, sizes[-1] + 64)
    buf.zero()
    ops = 1 << 30
    res = {s: [] for s in sizes}
    for _ in range(3):
        for s in sizes:
            ms = ctypes.c_double()
            _lib.check_diag(D.rsk_diag_membench(eng.ctx, 1, buf.ptr, s, ops, ctypes.byref(ms)))
            res[s].append(ops / ms.value * 1e3)
    for s, v in res.items():
        print("table %6.1f GB: %.3g gathers/s" % (s / 1e9, statistics.median(v)), flush=True)
    buf.free()


if __name__ == "__main__":
    main()
