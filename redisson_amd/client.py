"""RedissonClient mirror: the factory and keyspace behind the sketch objects.

Reference: src/main/java/org/redisson/RedissonClient.java (getHyperLogLog
:200,210; getBloomFilter :590,599; createBatch :648) and Redisson.java:276-283,
515-532.  The keyspace plays the role of the Redis db the reference talks to:
name -> HLL sketch (device registers), Bloom filter (device bit string) or
hash (the Bloom {name}__config).  Every sketch computation runs on the GPU.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import threading
from dataclasses import dataclass

from . import _lib
from .bloom import RBloomFilter
from .codec import DEFAULT_CODEC
from .hyperloglog import RHyperLogLog


@dataclass
class Config:
    """The one knob the GPU executor adds (SURVEY.md 5 'Config / flags')."""

    device: int = 0
    codec: object = DEFAULT_CODEC
    bloom_extended: bool = False  # allow filters beyond 2*Integer.MAX_VALUE bits
    threads: int = 4              # async executor (Config.threads analogue)


@dataclass
class _HllSlot:
    pool: ctypes.c_void_p
    id: int


class Redisson:
    """Redisson.create(config) analogue; one GPU engine per client."""

    def __init__(self, config: Config | None = None):
        self.config = config or Config()
        self.codec = self.config.codec
        self.engine = _lib.Engine.get(self.config.device)
        self._db: dict = {}
        self._views: dict = {}  # Bloom filter name -> rsk_bloom_bitset view of its bits
        self._lock = threading.RLock()
        self._pool = cf.ThreadPoolExecutor(max_workers=max(1, self.config.threads))

    @staticmethod
    def create(config: Config | None = None) -> "Redisson":
        return Redisson(config)

    @staticmethod
    def createReactive(config: Config | None = None):
        """Redisson.createReactive(config) -> RedissonReactiveClient analogue."""
        from .reactive import RedissonReactive

        return RedissonReactive(Redisson(config))

    def shutdown(self):
        self._pool.shutdown(wait=True)
        with self._lock:
            for name in list(self._db):
                self._drop(name)

    # -- factories (RedissonClient.java)
    def getHyperLogLog(self, name: str, codec=None) -> RHyperLogLog:
        return RHyperLogLog(self, name, codec)

    def getBloomFilter(self, name: str, codec=None) -> RBloomFilter:
        return RBloomFilter(self, name, codec)

    def getBitSet(self, name: str):
        from .bitset import RBitSet

        return RBitSet(self, name)

    def createBatch(self):
        from .batch import RBatch

        return RBatch(self)

    # -- keyspace
    def _submit(self, fn, *args):
        return self._pool.submit(fn, *args)

    def _drop(self, name):
        v = self._db.pop(name, None)
        if v is None:
            return 0
        kind, obj = v
        if kind == "hll":
            _lib.load().rsk_hll_destroy(obj.pool)
        elif kind == "bloom":
            view = self._views.pop(name, None)
            if view is not None:  # the view of the filter's bits goes first
                _lib.load().rsk_bitset_destroy(view)
            _lib.load().rsk_bloom_destroy(obj)
        elif kind == "bitset":
            _lib.load().rsk_bitset_destroy(obj)
        return 1

    def delete(self, *names) -> int:
        with self._lock:
            return sum(self._drop(n) for n in names)

    def _wrongtype(self, name):
        raise _lib.RedisException("WRONGTYPE Operation against a key holding the wrong kind of value: " + name)

    def _hll_slot(self, name: str, create: bool):
        with self._lock:
            v = self._db.get(name)
            if v is None:
                if not create:
                    return None
                h = ctypes.c_void_p()
                _lib.check(_lib.load().rsk_hll_create(self.engine.ctx, 1, ctypes.byref(h)))
                slot = _HllSlot(h, 0)
                self._db[name] = ("hll", slot)
                return slot
            if v[0] != "hll":
                self._wrongtype(name)
            return v[1]

    def _bloom_handle(self, name: str, size: int, k: int):
        with self._lock:
            v = self._db.get(name)
            if v is not None:
                if v[0] != "bloom":
                    self._wrongtype(name)
                return v[1]
            h = ctypes.c_void_p()
            _lib.check(_lib.load().rsk_bloom_create(self.engine.ctx, size, k, ctypes.byref(h)))
            self._db[name] = ("bloom", h)
            return h

    def _bitset_handle(self, name: str, create: bool):
        """The string of `name` as an rsk_bitset: a plain RBitSet string, or the
        bits of the Bloom filter of that name -- in Redis a filter's bits ARE the
        string key `name` (RedissonBloomFilter SETBITs it), so getBitSet(name)
        reads them (rsk_bloom_bitset)."""
        with self._lock:
            v = self._db.get(name)
            if v is not None:
                if v[0] == "bloom":
                    view = self._views.get(name)
                    if view is None:
                        h = ctypes.c_void_p()
                        _lib.check(_lib.load().rsk_bloom_bitset(v[1], ctypes.byref(h)), "rsk_bloom_bitset")
                        view = self._views[name] = h
                    return view
                if v[0] != "bitset":
                    self._wrongtype(name)
                return v[1]
            if not create:
                return None
            h = ctypes.c_void_p()
            _lib.check(_lib.load().rsk_bitset_create(self.engine.ctx, ctypes.byref(h)))
            self._db[name] = ("bitset", h)
            return h

    def _hash(self, name: str) -> dict:
        with self._lock:
            v = self._db.get(name)
            if v is None:
                return {}
            if v[0] != "hash":
                self._wrongtype(name)
            return dict(v[1])

    def _hmset(self, name: str, mapping: dict):
        with self._lock:
            v = self._db.get(name)
            if v is None:
                self._db[name] = ("hash", dict(mapping))
            elif v[0] != "hash":
                self._wrongtype(name)
            else:
                v[1].update(mapping)

    def getKeys(self):
        with self._lock:
            return list(self._db)
