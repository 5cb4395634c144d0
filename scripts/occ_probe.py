"""Occupancy query as seen with and without torch imported (A/B of bench.py's process context)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from redisson_amd import _lib  # noqa: E402

L = _lib.load()
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401
eng = _lib.Engine(0)
for w in (0, 1):
    pc, err = ctypes.c_int(), ctypes.c_int()
    L.rsk_diag_occupancy(w, ctypes.byref(pc), ctypes.byref(err))
    print(sys.argv[1:] or ["plain"], "kernel", w, "per_cu", pc.value, "hip_error", err.value, flush=True)
