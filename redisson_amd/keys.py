"""Key batches handed to the C ABI (rsk_keys): fixed stride or blob+offsets,
in host memory or already resident in HBM (redisson_amd.devmem.DeviceBuffer)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


class KeyBatch:
    """Encoded keys plus the buffers that keep them alive while a call runs."""

    def __init__(self, data, offsets, n: int, fixed_len: int, location: int, keepalive=()):
        self.data = data  # int address or None
        self.offsets = offsets
        self.n = int(n)
        self.fixed_len = int(fixed_len)
        self.location = location
        self._keep = keepalive

    @property
    def on_device(self) -> bool:
        return self.location == _lib.RSK_MEM_DEVICE

    def as_struct(self) -> _lib.rsk_keys:
        return _lib.rsk_keys(self.data, self.offsets, self.n, self.fixed_len, self.location)

    def slice(self, start: int, stop: int) -> "KeyBatch":
        """Keys [start, stop) as a new batch over the same buffers."""
        stop = min(stop, self.n)
        if self.offsets is None:
            d = None if self.data is None else self.data + start * self.fixed_len
            return KeyBatch(d, None, stop - start, self.fixed_len, self.location, self._keep)
        return KeyBatch(self.data, self.offsets + 8 * start, stop - start, 0, self.location, self._keep)

    # ---------------------------------------------------------- builders
    @staticmethod
    def from_bytes_list(keys) -> "KeyBatch":
        n = len(keys)
        lens = np.fromiter((len(k) for k in keys), dtype=np.uint64, count=n)
        if n and np.all(lens == lens[0]) and lens[0] > 0:
            blob = np.frombuffer(b"".join(keys), dtype=np.uint8)
            return KeyBatch(blob.ctypes.data, None, n, int(lens[0]), _lib.RSK_MEM_HOST, (blob,))
        offs = np.zeros(n + 1, dtype=np.uint64)
        if n:
            np.cumsum(lens, out=offs[1:])
        joined = b"".join(keys)
        blob = np.frombuffer(joined, dtype=np.uint8) if joined else np.zeros(1, np.uint8)
        return KeyBatch(blob.ctypes.data, offs.ctypes.data, n, 0, _lib.RSK_MEM_HOST, (blob, offs))

    @staticmethod
    def from_numpy(arr: np.ndarray, offsets: np.ndarray | None = None) -> "KeyBatch":
        """uint8 [n, L] fixed keys, or a 1-D blob with uint64 offsets[n+1]."""
        arr = np.ascontiguousarray(arr, dtype=np.uint8)
        if offsets is None:
            if arr.ndim != 2:
                raise ValueError("fixed-length keys must be a 2-D uint8 array [n, L]")
            return KeyBatch(arr.ctypes.data, None, arr.shape[0], arr.shape[1], _lib.RSK_MEM_HOST, (arr,))
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if arr.size == 0:
            arr = np.zeros(1, np.uint8)
        return KeyBatch(arr.ctypes.data, offsets.ctypes.data, offsets.size - 1, 0, _lib.RSK_MEM_HOST, (arr, offsets))


def encode_all(codec, objects) -> KeyBatch:
    if isinstance(objects, KeyBatch):
        return objects
    if isinstance(objects, np.ndarray):
        return KeyBatch.from_numpy(objects)
    return KeyBatch.from_bytes_list([codec.encode(o) for o in objects])


def out_buffer(kb: KeyBatch, n: int, engine=None):
    """Per-key reply buffer in the keys' location (device replies stay in HBM)."""
    if kb.on_device:
        from .devmem import DeviceBuffer

        b = DeviceBuffer(engine, max(n, 1))
        return b, b.ptr
    a = np.zeros(max(n, 1), dtype=np.uint8)
    return a, a.ctypes.data


def ptr_array(values) -> ctypes.Array:
    arr = (ctypes.c_uint64 * len(values))(*values)
    return arr
