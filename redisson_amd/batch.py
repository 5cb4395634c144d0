"""RBatch for sketches: pipelined commands executed in order on the GPU.

Reference: src/main/java/org/redisson/RedissonBatch.java:55-61,76-83,191,226-233
and core/RBatch.java:166-168,327.  The reference's "pipelined PFADD" baseline
is an RBatch of RHyperLogLog.add calls; here a run of consecutive adds to one
HLL becomes a single rsk_hll_add_each launch whose replies equal the
per-command replies.  RBitSet commands (RBitSetAsync) are queued the same way:
a run of consecutive single-bit SETBITs of one value on one key becomes one
rsk_bitset_setbits launch (later duplicates of an offset win, as in order),
a run of GETBITs one rsk_bitset_getbits launch.
"""
from __future__ import annotations

from concurrent.futures import Future


class _BatchObject:
    kind = ""

    def __init__(self, batch, name, codec=None):
        self._b, self._name, self._codec = batch, name, codec

    def _q(self, op, *args):
        f = Future()
        self._b._ops.append((self.kind, self._name, self._codec, op, args, f))
        return f


class _BatchHLL(_BatchObject):
    kind = "hll"

    def addAsync(self, obj):
        return self._q("add", obj)

    def addAllAsync(self, objs):
        return self._q("addAll", objs)

    def countAsync(self):
        return self._q("count")

    def countWithAsync(self, *names):
        return self._q("countWith", *names)

    def mergeWithAsync(self, *names):
        return self._q("mergeWith", *names)


class _BatchBitSet(_BatchObject):
    """RBitSetAsync (core/RBitSetAsync.java) inside a batch."""

    kind = "bitset"

    def getAsync(self, bitIndex):
        return self._q("get", bitIndex)

    def setAsync(self, *args):
        from .bitset import JavaBitSet

        if len(args) == 1 and not isinstance(args[0], JavaBitSet):
            return self._q("set1", args[0], True)
        if len(args) == 2 and isinstance(args[1], bool):
            return self._q("set1", args[0], args[1])
        return self._q("set", *args)

    def clearAsync(self, *args):
        if len(args) == 1:
            return self._q("set1", args[0], False)
        return self._q("clear", *args)

    def toByteArrayAsync(self):
        return self._q("toByteArray")

    def lengthAsync(self):
        return self._q("length")

    def sizeAsync(self):
        return self._q("size")

    def cardinalityAsync(self):
        return self._q("cardinality")

    def notAsync(self):
        return self._q("not_")

    def orAsync(self, *names):
        return self._q("or_", *names)

    def andAsync(self, *names):
        return self._q("and_", *names)

    def xorAsync(self, *names):
        return self._q("xor", *names)


class RBatch:
    def __init__(self, client):
        self._c = client
        self._ops = []

    def getHyperLogLog(self, name, codec=None):
        return _BatchHLL(self, name, codec)

    def getBitSet(self, name):
        return _BatchBitSet(self, name)

    def _run(self, ops, i, j, fn):
        """ops[i:j] share one launch: fn() returns their replies in order."""
        replies = fn()
        for t, r in zip(range(i, j), replies):
            ops[t][5].set_result(r)
        return list(replies)

    def execute(self):
        """Run every queued command in order; returns their replies (None for void commands)."""
        ops, self._ops = self._ops, []
        results = []
        i = 0
        while i < len(ops):
            kind, name, codec, op, args, fut = ops[i]

            def run_end(pred):
                j = i
                while j < len(ops) and ops[j][0] == kind and ops[j][1] == name and pred(ops[j]):
                    j += 1
                return j

            if kind == "hll":
                hll = self._c.getHyperLogLog(name, codec)
                if op == "add":
                    j = run_end(lambda o: o[3] == "add" and o[2] is codec)
                    results += self._run(ops, i, j, lambda: [bool(r) for r in
                                                             hll.addEach([ops[t][4][0] for t in range(i, j)])])
                    i = j
                    continue
                r = getattr(hll, op)(*args)
            else:
                bs = self._c.getBitSet(name)
                if op == "set1":
                    value = args[1]
                    j = run_end(lambda o: o[3] == "set1" and o[4][1] == value)
                    results += self._run(ops, i, j, lambda: (bs.setBits([ops[t][4][0] for t in range(i, j)], value),
                                                             [None] * (j - i))[1])
                    i = j
                    continue
                if op == "get":
                    j = run_end(lambda o: o[3] == "get")
                    results += self._run(ops, i, j, lambda: bs.getBits([ops[t][4][0] for t in range(i, j)]))
                    i = j
                    continue
                r = getattr(bs, op)(*args)
            fut.set_result(r)
            results.append(r)
            i += 1
        return results
