"""Reactive mirrors of the path's objects: RHyperLogLogReactive
(src/main/java/org/redisson/api/RHyperLogLogReactive.java, implemented by
reactive/RedissonHyperLogLogReactive.java:40-71) and RBitSetReactive
(api/RBitSetReactive.java), from RedissonReactiveClient.getHyperLogLog /
getBitSet (api/RedissonReactiveClient.java:112,122,322).

Every method returns a cold Publisher, as the reference's writeReactive /
readReactive do: nothing runs until subscribe(), each subscription runs the
command once (on the client's executor, the event-loop analogue) and then
signals on_next (not for Publisher<Void>) and on_complete, or on_error.
block() is the BaseReactiveTest.sync() of the reference tests.  The work is
the same GPU call as the synchronous object's (reactive addAll takes the
intended PFADD-of-all-elements semantics, like the sync one)."""
from __future__ import annotations

import concurrent.futures as cf


class Publisher:
    def __init__(self, client, fn, *args, void: bool = False):
        self._client, self._fn, self._args, self._void = client, fn, args, void

    def subscribe(self, on_next=None, on_error=None, on_complete=None) -> cf.Future:
        def run():
            try:
                v = self._fn(*self._args)
            except Exception as e:  # noqa: BLE001 - delivered to the subscriber
                if on_error is None:
                    raise
                on_error(e)
                return None
            if on_next is not None and not self._void:
                on_next(v)
            if on_complete is not None:
                on_complete()
            return None if self._void else v

        return self._client._submit(run)

    def block(self):
        return self.subscribe().result()


class RHyperLogLogReactive:
    def __init__(self, client, hll):
        self._client, self._h = client, hll

    def getName(self) -> str:
        return self._h.getName()

    def add(self, obj) -> Publisher:
        return Publisher(self._client, self._h.add, obj)

    def addAll(self, objects) -> Publisher:
        return Publisher(self._client, self._h.addAll, list(objects))

    def count(self) -> Publisher:
        return Publisher(self._client, self._h.count)

    def countWith(self, *otherLogNames) -> Publisher:
        return Publisher(self._client, self._h.countWith, *otherLogNames)

    def mergeWith(self, *otherLogNames) -> Publisher:
        return Publisher(self._client, self._h.mergeWith, *otherLogNames, void=True)


class RBitSetReactive:
    def __init__(self, client, bs):
        self._client, self._b = client, bs

    def getName(self) -> str:
        return self._b.getName()

    def _p(self, fn, *args, void=False) -> Publisher:
        return Publisher(self._client, fn, *args, void=void)

    def asBitSet(self) -> Publisher:
        return self._p(self._b.asBitSet)

    def toByteArray(self) -> Publisher:
        return self._p(self._b.toByteArray)

    def length(self) -> Publisher:
        return self._p(self._b.length)

    def size(self) -> Publisher:
        return self._p(self._b.size)

    def cardinality(self) -> Publisher:
        return self._p(self._b.cardinality)

    def get(self, bitIndex: int) -> Publisher:
        return self._p(self._b.get, bitIndex)

    def set(self, *args) -> Publisher:
        return self._p(self._b.set, *args, void=True)

    def clear(self, *args) -> Publisher:
        return self._p(self._b.clear, *args, void=True)

    def not_(self) -> Publisher:
        return self._p(self._b.not_, void=True)

    def or_(self, *bitSetNames) -> Publisher:
        return self._p(self._b.or_, *bitSetNames, void=True)

    def and_(self, *bitSetNames) -> Publisher:
        return self._p(self._b.and_, *bitSetNames, void=True)

    def xor(self, *bitSetNames) -> Publisher:
        return self._p(self._b.xor, *bitSetNames, void=True)

    def toString(self) -> str:
        return self._b.toString()

    def __str__(self) -> str:
        return self._b.toString()


setattr(RBitSetReactive, "or", RBitSetReactive.or_)
setattr(RBitSetReactive, "and", RBitSetReactive.and_)
setattr(RBitSetReactive, "not", RBitSetReactive.not_)


class RedissonReactive:
    """RedissonReactiveClient analogue over one engine (Redisson.createReactive)."""

    def __init__(self, client):
        self._client = client

    def getHyperLogLog(self, name: str, codec=None) -> RHyperLogLogReactive:
        return RHyperLogLogReactive(self._client, self._client.getHyperLogLog(name, codec))

    def getBitSet(self, name: str) -> RBitSetReactive:
        return RBitSetReactive(self._client, self._client.getBitSet(name))

    def shutdown(self):
        self._client.shutdown()
