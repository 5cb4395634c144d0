"""RBloomFilter on the gfx950 engine.

Mirror of src/main/java/org/redisson/core/RBloomFilter.java:27-58, implemented
by RedissonBloomFilter.java:50-289:

  tryInit(n, p)          (:223-252)  sizes with Java double semantics; False if
                                     the {name}__config hash already exists
  add(obj)               (:80-114)   True iff one of the first k-1 bits was clear
  contains(obj)          (:133-168)  AND of the first k-1 bits
  count()                (:188-199)  (int)(-size/k * ln(1 - bitcount/size))
  getExpectedInsertions / getFalseProbability / getSize / getHashIterations
                         (:258-280)  IllegalStateException when not initialised

Batched extensions for GPU callers: addAll(objs) -> per-key replies in input
order (or None when replies are not wanted), containsAll(objs) -> replies.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .keys import KeyBatch, encode_all, out_buffer

MAX_SIZE = 2147483647 * 2  # RedissonBloomFilter.java:52


def _config_name(name: str) -> str:
    return "{" + name + "}__config"  # RedissonBloomFilter.java:254-256


def _plain(p: float) -> str:
    """BigDecimal.valueOf(p).toPlainString() for the usual probabilities."""
    r = repr(float(p))
    if "e" in r or "E" in r:
        from decimal import Decimal

        r = format(Decimal(r), "f")
    return r


def bloom_params(n: int, p: float, extended: bool = False):
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    mode = _lib.RSK_BLOOM_EXTENDED if extended else _lib.RSK_BLOOM_COMPAT
    _lib.check(_lib.load().rsk_bloom_params(int(n), float(p), mode, ctypes.byref(size), ctypes.byref(k)))
    return size.value, k.value


class RBloomFilter:
    def __init__(self, client, name: str, codec=None):
        self._client = client
        self._name = name
        self.codec = codec or client.codec

    def getName(self) -> str:
        return self._name

    # -- config ({name}__config hash, HMSET at :237-240)
    def _config(self) -> dict:
        return self._client._hash(_config_name(self._name))

    def _filter(self):
        cfg = self._config()
        if cfg.get("hashIterations") is None or cfg.get("size") is None:
            raise _lib.IllegalStateException("Bloom filter is not initialized!")
        return self._client._bloom_handle(self._name, int(cfg["size"]), int(cfg["hashIterations"]))

    def tryInit(self, expectedInsertions: int, falseProbability: float) -> bool:
        size, k = bloom_params(expectedInsertions, falseProbability, self._client.config.bloom_extended)
        cfg = self._config()
        if cfg.get("size") is not None or cfg.get("hashIterations") is not None:
            return False  # Lua assert: 'Bloom filter config has been changed'
        self._client._hmset(_config_name(self._name), {
            "size": str(size), "hashIterations": str(k),
            "expectedInsertions": str(int(expectedInsertions)),
            "falseProbability": _plain(falseProbability)})
        self._client._bloom_handle(self._name, size, k)
        return True

    def getExpectedInsertions(self) -> int:
        return int(self._check(self._config().get("expectedInsertions")))

    def getFalseProbability(self) -> float:
        return float(self._check(self._config().get("falseProbability")))

    def getSize(self) -> int:
        return int(self._check(self._config().get("size")))

    def getHashIterations(self) -> int:
        return int(self._check(self._config().get("hashIterations")))

    @staticmethod
    def _check(v):
        if v is None:
            raise _lib.IllegalStateException("Bloom filter is not initialized!")
        return v

    # -- add / contains
    def add(self, obj) -> bool:
        return bool(self.addAll([obj])[0])

    def addAll(self, objects, replies: bool = True):
        kb = encode_all(self.codec, objects)
        b = self._filter()
        ks = kb.as_struct()
        if not replies:
            _lib.check(_lib.load().rsk_bloom_add(b, ctypes.byref(ks), None), "SETBIT")
            return None
        buf, ptr = out_buffer(kb, kb.n, self._client.engine)
        _lib.check(_lib.load().rsk_bloom_add(b, ctypes.byref(ks), ptr), "SETBIT")
        if kb.on_device:
            return buf  # replies stay in HBM (DeviceBuffer of n bytes)
        return [bool(x) for x in buf[: kb.n]]

    def contains(self, obj) -> bool:
        return bool(self.containsAll([obj])[0])

    def containsAll(self, objects):
        kb = encode_all(self.codec, objects)
        b = self._filter()
        buf, ptr = out_buffer(kb, kb.n, self._client.engine)
        ks = kb.as_struct()
        _lib.check(_lib.load().rsk_bloom_contains(b, ctypes.byref(ks), ptr), "GETBIT")
        if kb.on_device:
            return buf  # replies stay in HBM (DeviceBuffer of n bytes)
        return [bool(x) for x in buf[: kb.n]]

    def count(self) -> int:
        b = self._filter()
        out = ctypes.c_int32()
        _lib.check(_lib.load().rsk_bloom_count(b, ctypes.byref(out)), "BITCOUNT")
        return out.value

    def delete(self) -> bool:
        # DEL name {name}__config (RedissonBloomFilter.java:202-204)
        return self._client.delete(self._name, _config_name(self._name)) > 0

    # -- Redis wire format: the bit string (RBitSet layout, MSB-first)
    def toByteArray(self) -> bytes:
        b = self._filter()
        size = ctypes.c_int64()
        k = ctypes.c_int32()
        _lib.check(_lib.load().rsk_bloom_info(b, ctypes.byref(size), ctypes.byref(k)))
        nbytes = (size.value + 7) // 8
        buf = np.zeros(max(1, nbytes), dtype=np.uint8)
        n = ctypes.c_size_t()
        _lib.check(_lib.load().rsk_bloom_export_bits(b, buf.ctypes.data, buf.size, ctypes.byref(n)))
        return buf[: n.value].tobytes()
