"""RBitSet on the gfx950 engine.

Mirror of src/main/java/org/redisson/core/RBitSet.java:25-61, implemented by
RedissonBitSet.java: a Redis string addressed as bits, MSB-first (bit i in
byte i>>3 under mask 0x80>>(i&7)).  On the name of a Bloom filter it is the
filter's bit string (rsk_bloom_bitset), as in Redis where the filter's bits
are the string key of that name.  Every command runs through the rsk_bitset
C ABI on the GPU; only the java.util.BitSet conversions (fromByteArrayReverse /
toByteArrayReverse, :152-173) happen on the host, as in the reference.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


class JavaBitSet:
    """The java.util.BitSet values RBitSet.asBitSet() / set(BitSet) exchange."""

    def __init__(self, indices=()):
        self._s = set(int(i) for i in indices)

    def get(self, i: int) -> bool:
        return i in self._s

    def set(self, i: int):
        self._s.add(int(i))

    def clear(self, i: int):
        self._s.discard(int(i))

    def cardinality(self) -> int:
        return len(self._s)

    def length(self) -> int:
        return max(self._s) + 1 if self._s else 0

    def indices(self):
        return sorted(self._s)

    def __eq__(self, other):
        return isinstance(other, JavaBitSet) and self._s == other._s

    def __str__(self):
        return "{" + ", ".join(str(i) for i in self.indices()) + "}"

    __repr__ = __str__


def from_byte_array_reverse(data: bytes) -> JavaBitSet:
    """RedissonBitSet.fromByteArrayReverse (:152-160)."""
    a = np.frombuffer(data, dtype=np.uint8)
    bits = np.unpackbits(a)  # MSB first per byte
    return JavaBitSet(np.nonzero(bits)[0].tolist())


def to_byte_array_reverse(bs: JavaBitSet) -> bytes:
    """RedissonBitSet.toByteArrayReverse (:163-172): length()/8 + 1 bytes."""
    out = bytearray(bs.length() // 8 + 1)
    for i in bs.indices():
        out[i // 8] |= 1 << (7 - (i % 8))
    return bytes(out)


_OPS = {"AND": 0, "OR": 1, "XOR": 2, "NOT": 3}


class RBitSet:
    def __init__(self, client, name: str):
        self._client = client
        self._name = name

    def getName(self) -> str:
        return self._name

    def _h(self, create=True):
        return self._client._bitset_handle(self._name, create)

    # -- single bits (SETBIT / GETBIT)
    def get(self, bitIndex: int) -> bool:
        h = self._h(False)
        if h is None:
            return False
        offs = (ctypes.c_uint64 * 1)(bitIndex)
        out = (ctypes.c_uint8 * 1)()
        _lib.check(_lib.load().rsk_bitset_getbits(h, offs, 1, _lib.RSK_MEM_HOST, out), "GETBIT")
        return bool(out[0])

    def set(self, *args):
        """set(index) | set(index, value) | set(from, to) | set(from, to, value) | set(BitSet)."""
        if len(args) == 1 and isinstance(args[0], JavaBitSet):
            return self._set_bytes(to_byte_array_reverse(args[0]))
        if len(args) == 1:
            return self._setbits([args[0]], 1)
        if len(args) == 2 and isinstance(args[1], bool):
            return self._setbits([args[0]], 1 if args[1] else 0)
        if len(args) == 2:
            return self._range(args[0], args[1], 1)
        if len(args) == 3:
            return self._range(args[0], args[1], 1 if args[2] else 0)
        raise TypeError("set() takes (index[, value]), (from, to[, value]) or (BitSet)")

    def clear(self, *args):
        """clear() = DEL | clear(index) | clear(from, to)."""
        if not args:
            h = self._h(False)
            if h is not None:
                _lib.check(_lib.load().rsk_bitset_clear(h))
            return None
        if len(args) == 1:
            return self._setbits([args[0]], 0)
        return self._range(args[0], args[1], 0)

    def setBits(self, indices, value: bool = True):
        """Batched SETBIT over many offsets (one GPU launch)."""
        return self._setbits(list(indices), 1 if value else 0)

    def getBits(self, indices):
        h = self._h(False)
        idx = np.ascontiguousarray(indices, dtype=np.uint64)
        if h is None:
            return [False] * idx.size
        out = np.zeros(max(1, idx.size), np.uint8)
        _lib.check(_lib.load().rsk_bitset_getbits(h, idx.ctypes.data, idx.size, _lib.RSK_MEM_HOST, out.ctypes.data))
        return [bool(x) for x in out[: idx.size]]

    def _setbits(self, indices, v):
        idx = np.ascontiguousarray(indices, dtype=np.uint64)
        if (np.asarray(indices, dtype=object) < 0).any():
            raise _lib.RedisException("ERR bit offset is not an integer or out of range")
        _lib.check(_lib.load().rsk_bitset_setbits(self._h(), idx.ctypes.data, idx.size, v, _lib.RSK_MEM_HOST),
                   "SETBIT")

    def _range(self, frm, to, v):
        if frm < 0 or to < 0:
            raise _lib.RedisException("ERR bit offset is not an integer or out of range")
        _lib.check(_lib.load().rsk_bitset_set_range(self._h(), frm, to, v), "SETBIT")

    def _set_bytes(self, data: bytes):
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        _lib.check(_lib.load().rsk_bitset_set_bytes(self._h(), buf, len(data)), "SET")

    # -- whole string
    def size(self) -> int:
        h = self._h(False)
        if h is None:
            return 0
        n = ctypes.c_uint64()
        _lib.check(_lib.load().rsk_bitset_strlen(h, ctypes.byref(n)))
        return 8 * n.value

    def length(self) -> int:
        h = self._h(False)
        if h is None:
            return 0
        n = ctypes.c_uint64()
        _lib.check(_lib.load().rsk_bitset_length(h, ctypes.byref(n)))
        return n.value

    def cardinality(self) -> int:
        h = self._h(False)
        if h is None:
            return 0
        n = ctypes.c_uint64()
        _lib.check(_lib.load().rsk_bitset_bitcount(h, ctypes.byref(n)), "BITCOUNT")
        return n.value

    def toByteArray(self):
        h = self._h(False)
        if h is None:
            return None
        n = ctypes.c_uint64()
        _lib.check(_lib.load().rsk_bitset_strlen(h, ctypes.byref(n)))
        buf = np.zeros(max(1, n.value), np.uint8)
        got = ctypes.c_size_t()
        _lib.check(_lib.load().rsk_bitset_get_bytes(h, buf.ctypes.data, buf.size, ctypes.byref(got)), "GET")
        return buf[: got.value].tobytes() if got.value else None

    def asBitSet(self) -> JavaBitSet:
        return from_byte_array_reverse(self.toByteArray() or b"")

    def __str__(self):
        return str(self.asBitSet())

    def toString(self) -> str:
        return str(self)

    # -- BITOP op self self names...
    def _op(self, op, names):
        srcs = [self._h()] + [self._client._bitset_handle(n, True) for n in names]
        arr = (ctypes.c_void_p * len(srcs))(*srcs)
        _lib.check(_lib.load().rsk_bitset_bitop(_OPS[op], self._h(), arr, len(srcs)), "BITOP")

    def or_(self, *bitSetNames):
        self._op("OR", bitSetNames)

    def and_(self, *bitSetNames):
        self._op("AND", bitSetNames)

    def xor(self, *bitSetNames):
        self._op("XOR", bitSetNames)

    def not_(self):
        self._op("NOT", ())

    def delete(self) -> bool:
        """DEL name.  On a Bloom filter's name that deletes only its bit string
        (the filter stays initialised: {name}__config is another key)."""
        with self._client._lock:
            v = self._client._db.get(self._name)
            if v is not None and v[0] == "bloom":
                existed = self.size() > 0
                _lib.check(_lib.load().rsk_bitset_clear(self._h(False)), "DEL")
                return existed
        return self._client.delete(self._name) > 0


# Java method names that are Python keywords
setattr(RBitSet, "or", RBitSet.or_)
setattr(RBitSet, "and", RBitSet.and_)
setattr(RBitSet, "not", RBitSet.not_)
