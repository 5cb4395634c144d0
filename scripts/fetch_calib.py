"""FETCH_SIZE calibration (MI355X_MICROARCH.md HBM: 'calibrate on a known
byte count in your own access pattern').  One launch per pattern over a known
byte count, in a fixed order, so a rocprofv3 --pmc FETCH_SIZE run of this
script gives FETCH per dispatch against the bytes read:

  python scripts/fetch_calib.py            (prints the dispatch order)

dispatches: stream read 4 GiB; scattered segment reads of 256, 512 and 1024 B
(one uint4 per lane: the Bloom apply / rp_apply / hll_gapply record loads);
a 4 B/lane stream (hll_gpart1t's group ids, hll_gapply_extra's records) and
scattered 128 / 256 B segments read one dword per lane (the C5 fine-bin
pass's medium segments: hll_gcount2t / hll_gpart2t)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

CASES = [("stream_read", 0, 0), ("segment_256B", 6, 256), ("segment_512B", 6, 512), ("segment_1KiB", 6, 1024),
         ("stream4_read", 8, 0), ("segment4_128B", 9, 128), ("segment4_256B", 9, 256)]


def gathers():
    """`fetch_calib.py gathers`: 2^30 random 4-byte gathers (membench mode 1)
    over a 16 GiB buffer -- FETCH_SIZE per gather for the reply pass's model."""
    _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    nbytes, nops = 16 << 30, 1 << 30
    buf = devmem.DeviceBuffer(eng, nbytes)
    buf.zero()
    ms = ctypes.c_double()
    _lib.check_diag(D.rsk_diag_membench(eng.ctx, 1, buf.ptr, nbytes, nops, ctypes.byref(ms)))
    print("gather4B buffer=%d ops=%d ms=%.3f gathers/s=%.3e" % (nbytes, nops, ms.value, nops / ms.value * 1e3), flush=True)
    buf.free()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "gathers":
        return gathers()
    _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    nbytes = 4 << 30
    buf = devmem.DeviceBuffer(eng, nbytes)
    buf.zero()
    for name, mode, seg in CASES:
        ms = ctypes.c_double()
        _lib.check_diag(D.rsk_diag_membench(eng.ctx, mode, buf.ptr, nbytes, seg, ctypes.byref(ms)))
        print("%-14s bytes=%d ms=%.3f GB/s=%.0f" % (name, nbytes, ms.value, nbytes / ms.value / 1e6), flush=True)
    buf.free()


if __name__ == "__main__":
    main()
