"""RBatch for sketches: pipelined commands executed in order on the GPU.

Reference: src/main/java/org/redisson/RedissonBatch.java:55-61,76-83,226-233 and
core/RBatch.java.  The reference's "pipelined PFADD" baseline is an RBatch of
RHyperLogLog.add calls; here a run of consecutive adds to one HLL becomes a
single rsk_hll_add_each launch whose replies equal the per-command replies.
"""
from __future__ import annotations

from concurrent.futures import Future


class _BatchHLL:
    def __init__(self, batch, name, codec):
        self._b, self._name, self._codec = batch, name, codec

    def _q(self, op, *args):
        f = Future()
        self._b._ops.append((self._name, self._codec, op, args, f))
        return f

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


class RBatch:
    def __init__(self, client):
        self._c = client
        self._ops = []

    def getHyperLogLog(self, name, codec=None):
        return _BatchHLL(self, name, codec)

    def execute(self):
        """Run every queued command in order; returns their replies."""
        ops, self._ops = self._ops, []
        results = []
        i = 0
        while i < len(ops):
            name, codec, op, args, fut = ops[i]
            hll = self._c.getHyperLogLog(name, codec)
            if op == "add":
                j = i
                while j < len(ops) and ops[j][0] == name and ops[j][2] == "add" and ops[j][1] is codec:
                    j += 1
                replies = hll.addEach([ops[t][3][0] for t in range(i, j)])
                for t, r in zip(range(i, j), replies):
                    ops[t][4].set_result(bool(r))
                    results.append(bool(r))
                i = j
                continue
            r = getattr(hll, op)(*args)
            fut.set_result(r)
            results.append(r)
            i += 1
        return results
