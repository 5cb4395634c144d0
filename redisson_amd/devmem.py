"""HBM buffers owned through the C ABI (rsk_dev_alloc), so that keys stay
resident on the GPU across calls.  librsketch runs on the system ROCm
runtime; it does not share a process with torch.cuda ("Runtime")."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .keys import KeyBatch

RSK_H2D, RSK_D2H, RSK_D2D = 0, 1, 2


class DeviceBuffer:
    def __init__(self, engine, nbytes: int):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _lib.check(_lib.load().rsk_dev_alloc(engine.ctx, self.nbytes, ctypes.byref(p)), "rsk_dev_alloc")
        self.ptr = p.value

    def free(self):
        if self.ptr:
            _lib.load().rsk_dev_free(self.engine.ctx, self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.free()
        except Exception:
            pass

    @staticmethod
    def from_numpy(engine, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = DeviceBuffer(engine, max(1, arr.nbytes))
        if arr.nbytes:
            _lib.check(_lib.load().rsk_memcpy(engine.ctx, b.ptr, arr.ctypes.data, arr.nbytes, RSK_H2D))
        return b

    def to_numpy(self, dtype=np.uint8, count: int | None = None, offset: int = 0) -> np.ndarray:
        item = np.dtype(dtype).itemsize
        if count is None:
            count = (self.nbytes - offset) // item
        out = np.empty(count, dtype=dtype)
        if count:
            _lib.check(_lib.load().rsk_memcpy(self.engine.ctx, out.ctypes.data, self.ptr + offset, count * item,
                                              RSK_D2H))
        return out

    def zero(self):
        _lib.check(_lib.load().rsk_memset(self.engine.ctx, self.ptr, 0, self.nbytes))

    # key batches over this buffer (device resident)
    def keys_fixed(self, n: int, fixed_len: int, offset: int = 0) -> KeyBatch:
        return KeyBatch(self.ptr + offset, None, n, fixed_len, _lib.RSK_MEM_DEVICE, (self,))

    def keys_var(self, offsets: "DeviceBuffer", n: int) -> KeyBatch:
        return KeyBatch(self.ptr, offsets.ptr, n, 0, _lib.RSK_MEM_DEVICE, (self, offsets))


def gen_keys16(engine, seed: int, start: int, n: int) -> DeviceBuffer:
    b = DeviceBuffer(engine, 16 * n)
    _lib.check_diag(_lib.diag().rsk_gen_keys16(engine.ctx, seed, start, n, b.ptr))
    return b


def gen_queries16(engine, qseed: int, iseed: int, n_ins: int, start: int, n: int) -> DeviceBuffer:
    b = DeviceBuffer(engine, 16 * n)
    _lib.check_diag(_lib.diag().rsk_gen_queries16(engine.ctx, qseed, iseed, n_ins, start, n, b.ptr))
    return b


def gen_grouped(engine, seed: int, G: int, start: int, n: int):
    g = DeviceBuffer(engine, 4 * n)
    k = DeviceBuffer(engine, 16 * n)
    _lib.check_diag(_lib.diag().rsk_gen_grouped(engine.ctx, seed, G, start, n, g.ptr, k.ptr))
    return g, k


def gen_grouped_zipf(engine, seed: int, G: int, s: float, start: int, n: int):
    g = DeviceBuffer(engine, 4 * n)
    k = DeviceBuffer(engine, 16 * n)
    _lib.check_diag(_lib.diag().rsk_gen_grouped_zipf(engine.ctx, seed, G, s, start, n, g.ptr, k.ptr))
    return g, k


def gen_varlen(engine, seed: int, start: int, n: int):
    offs = DeviceBuffer(engine, 8 * (n + 1))
    tot = ctypes.c_uint64()
    D = _lib.diag()
    _lib.check_diag(D.rsk_gen_varlen(engine.ctx, seed, start, n, offs.ptr, None, 0, ctypes.byref(tot)))
    blob = DeviceBuffer(engine, max(1, tot.value))
    _lib.check_diag(D.rsk_gen_varlen(engine.ctx, seed, start, n, offs.ptr, blob.ptr, blob.nbytes, ctypes.byref(tot)))
    return blob, offs, tot.value
