"""RHyperLogLog on the gfx950 engine.

Mirror of the reference interface src/main/java/org/redisson/core/RHyperLogLog.java:20-30
(and RHyperLogLogAsync.java:22-33), implemented by RedissonHyperLogLog.java:30-99,
with the same method names, argument meaning and reply semantics:

  add(obj)            -> PFADD name obj          (:40-43, :65-68)   bool
  addAll(objs)        -> PFADD name o1..on       (:45-48, :70-76)   bool
  count()             -> PFCOUNT name            (:50-53, :78-81)   int
  countWith(*names)   -> PFCOUNT name n1..nk     (:55-58, :83-89)   int
  mergeWith(*names)   -> PFMERGE name n1..nk     (:60-63, :91-97)   None

addAll implements the INTENDED PFADD-of-all-elements semantics; the fork's
varargs bug (the whole collection encoded as one element) is
deliberately not reproduced ("Divergences").
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .keys import KeyBatch, encode_all, out_buffer


class RHyperLogLog:
    def __init__(self, client, name: str, codec=None):
        self._client = client
        self._name = name
        self.codec = codec or client.codec

    # -- RObject
    def getName(self) -> str:
        return self._name

    def _slot(self, create: bool):
        return self._client._hll_slot(self._name, create)

    def delete(self) -> bool:
        return self._client.delete(self._name) > 0

    def isExists(self) -> bool:
        s = self._slot(False)
        if s is None:
            return False
        v = ctypes.c_int()
        _lib.check(_lib.load().rsk_hll_exists(s.pool, s.id, ctypes.byref(v)))
        return bool(v.value)

    # -- PFADD
    def add(self, obj) -> bool:
        return self.addAll([obj])

    def addAll(self, objects) -> bool:
        kb = encode_all(self.codec, objects)
        s = self._slot(True)
        changed = ctypes.c_uint8()
        ks = kb.as_struct()
        _lib.check(_lib.load().rsk_hll_add(s.pool, s.id, ctypes.byref(ks), ctypes.byref(changed)), "PFADD")
        return bool(changed.value)

    def addEach(self, objects):
        """One PFADD per element in order (RBatch of add(); RedissonBatch.java:76-83):
        the list of replies."""
        kb = encode_all(self.codec, objects)
        s = self._slot(True)
        buf, ptr = out_buffer(kb, kb.n, self._client.engine)
        ks = kb.as_struct()
        _lib.check(_lib.load().rsk_hll_add_each(s.pool, s.id, ctypes.byref(ks), ptr), "PFADD")
        if kb.on_device:
            return buf  # replies stay in HBM (DeviceBuffer of n bytes)
        return [bool(x) for x in buf[: kb.n]]

    # -- PFCOUNT
    def count(self) -> int:
        s = self._slot(False)
        if s is None:
            return 0
        out = (ctypes.c_uint64 * 1)()
        ids = (ctypes.c_uint64 * 1)(s.id)
        _lib.check(_lib.load().rsk_hll_count(s.pool, ids, 1, out), "PFCOUNT")
        return int(out[0])

    def countWith(self, *otherLogNames) -> int:
        names = (self._name,) + tuple(otherLogNames)
        slots = [self._client._hll_slot(n, False) for n in names]
        live = [s for s in slots if s is not None]
        if not live:
            return 0
        pools = (ctypes.c_void_p * len(live))(*[s.pool for s in live])
        ids = (ctypes.c_uint64 * len(live))(*[s.id for s in live])
        out = (ctypes.c_uint64 * 1)()
        _lib.check(_lib.load().rsk_hll_count_union(pools, ids, len(live), out), "PFCOUNT")
        return int(out[0])

    # -- PFMERGE
    def mergeWith(self, *otherLogNames) -> None:
        srcs = [self._client._hll_slot(n, False) for n in otherLogNames]
        live = [s for s in srcs if s is not None]
        dst = self._slot(True)
        pools = (ctypes.c_void_p * max(1, len(live)))(*[s.pool for s in live])
        ids = (ctypes.c_uint64 * max(1, len(live)))(*[s.id for s in live])
        _lib.check(_lib.load().rsk_hll_merge(dst.pool, dst.id, pools, ids, len(live)), "PFMERGE")

    # -- async variants (RHyperLogLogAsync): futures on the client executor
    def addAsync(self, obj):
        return self._client._submit(self.add, obj)

    def addAllAsync(self, objects):
        return self._client._submit(self.addAll, objects)

    def countAsync(self):
        return self._client._submit(self.count)

    def countWithAsync(self, *names):
        return self._client._submit(self.countWith, *names)

    def mergeWithAsync(self, *names):
        return self._client._submit(self.mergeWith, *names)

    # -- Redis wire format
    def toRedisBytes(self):
        """GET name: the dense HYLL string (None when the key is absent)."""
        s = self._slot(False)
        if s is None:
            return None
        buf = (ctypes.c_uint8 * _lib.HLL_DENSE_BYTES)()
        n = ctypes.c_size_t()
        _lib.check(_lib.load().rsk_hll_export_redis(s.pool, s.id, buf, len(buf), ctypes.byref(n)))
        return bytes(buf[: n.value]) if n.value else None

    def fromRedisBytes(self, data: bytes) -> None:
        """SET name <HYLL string> (dense or sparse, validated like Redis)."""
        s = self._slot(True)
        b = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        _lib.check(_lib.load().rsk_hll_import_redis(s.pool, s.id, b, len(data)))

    def registers(self) -> np.ndarray:
        s = self._slot(False)
        out = np.zeros(_lib.HLL_REGISTERS, dtype=np.uint8)
        if s is not None:
            _lib.check(_lib.load().rsk_hll_get_registers(s.pool, s.id, out.ctypes.data, _lib.RSK_MEM_HOST))
        return out


class GroupedHyperLogLog:
    """A pool of G sketches addressed by group id (COUNT DISTINCT per group,
    BASELINE config 5): batched add / count / countWith / mergeWith."""

    def __init__(self, engine, n_groups: int):
        self.engine = engine
        self.n = int(n_groups)
        h = ctypes.c_void_p()
        _lib.check(_lib.load().rsk_hll_create(engine.ctx, self.n, ctypes.byref(h)))
        self.pool = h

    def close(self):
        if self.pool:
            _lib.load().rsk_hll_destroy(self.pool)
            self.pool = None

    def clear(self) -> None:
        """DEL of every sketch in the pool (rsk_hll_clear)."""
        _lib.check(_lib.load().rsk_hll_clear(self.pool))

    def add(self, keys: KeyBatch, groups) -> None:
        """groups: uint32 numpy array (host keys) or a DeviceBuffer of uint32 (device keys)."""
        if hasattr(groups, "ptr"):
            gp = groups.ptr
        else:
            groups = np.ascontiguousarray(groups, np.uint32)
            gp = groups.ctypes.data
        ks = keys.as_struct()
        _lib.check(_lib.load().rsk_hll_add_grouped(self.pool, ctypes.byref(ks), gp))

    def count(self, ids=None, out=None) -> np.ndarray:
        """PFCOUNT of every sketch (ids None) or of ids; `out` (uint64, reused
        across calls) receives the counts."""
        n = self.n if ids is None else len(ids)
        if out is None or out.dtype != np.uint64 or out.size < n or not out.flags.c_contiguous:
            out = np.empty(n, dtype=np.uint64)
        if ids is None:
            _lib.check(_lib.load().rsk_hll_count(self.pool, None, self.n, out.ctypes.data))
            return out[:n]
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        _lib.check(_lib.load().rsk_hll_count(self.pool, ids.ctypes.data, ids.size, out.ctypes.data))
        return out[:n]

    def countWith(self, member_ids) -> np.ndarray:
        m = np.ascontiguousarray(member_ids, dtype=np.uint64)
        if m.ndim != 2:
            raise ValueError("member_ids must be [n, arity]")
        out = np.zeros(m.shape[0], dtype=np.uint64)
        _lib.check(_lib.load().rsk_hll_count_union_batch(self.pool, m.ctypes.data, m.shape[1], m.shape[0],
                                                         out.ctypes.data))
        return out

    def mergeWith(self, dst_ids, src_ids) -> None:
        d = np.ascontiguousarray(dst_ids, dtype=np.uint64)
        s = np.ascontiguousarray(src_ids, dtype=np.uint64)
        _lib.check(_lib.load().rsk_hll_merge_batch(self.pool, d.ctypes.data, s.ctypes.data, d.size))

    def registers(self, gid: int) -> np.ndarray:
        out = np.zeros(_lib.HLL_REGISTERS, dtype=np.uint8)
        _lib.check(_lib.load().rsk_hll_get_registers(self.pool, gid, out.ctypes.data, _lib.RSK_MEM_HOST))
        return out

    # -- the pool's Redis strings (checkpoint / restore)
    def exportRedis(self, ids=None, out=None):
        """GET of many keys (rsk_hll_export_redis_batch): returns (data, offsets)
        with key i's "HYLL" string in data[offsets[i]:offsets[i+1]] (empty for
        a missing key).  `out` (a uint8 array) is used when large enough;
        otherwise the call is repeated with an exact buffer."""
        ids = np.arange(self.n, dtype=np.uint64) if ids is None else np.ascontiguousarray(ids, dtype=np.uint64)
        offs = np.empty(ids.size + 1, dtype=np.uint64)  # (every entry written by a call that succeeds or
        offs[-1] = 0                                    # overflows; offs[-1] read only then)
        L = _lib.load()
        if out is None or out.dtype != np.uint8 or not out.flags.c_contiguous:
            out = np.empty(0, np.uint8)
        rc = L.rsk_hll_export_redis_batch(self.pool, ids.ctypes.data, ids.size, out.ctypes.data if out.size else None,
                                          out.size, offs.ctypes.data)
        if rc == _lib.RSK_ERR_INVALID_ARG and int(offs[-1]) > out.size:
            out = np.empty(int(offs[-1]), np.uint8)
            rc = L.rsk_hll_export_redis_batch(self.pool, ids.ctypes.data, ids.size, out.ctypes.data, out.size,
                                              offs.ctypes.data)
        _lib.check(rc)
        return out[: int(offs[-1])], offs

    def importRedis(self, ids, data, offsets) -> None:
        """SET of many keys (rsk_hll_import_redis_batch): key ids[i] := the string
        data[offsets[i]:offsets[i+1]]; all or nothing."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        data = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                    dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        if offs.size != ids.size + 1 or (ids.size and int(offs[-1]) > data.size):
            raise ValueError("offsets must hold n + 1 entries inside data")
        _lib.check(_lib.load().rsk_hll_import_redis_batch(self.pool, ids.ctypes.data, ids.size,
                                                          data.ctypes.data, offs.ctypes.data))

    # -- pipelined forms (the library's async calls, ordered on the context
    # stream like the synchronous ones; each returns a NativeOp to wait on)
    def add_async(self, keys: KeyBatch, groups) -> "_lib.NativeOp":
        if hasattr(groups, "ptr"):
            gp = groups.ptr
        else:
            groups = np.ascontiguousarray(groups, np.uint32)
            gp = groups.ctypes.data
        ks = keys.as_struct()
        op = _lib.NativeOp(keys, groups, ks)
        return op.issued(_lib.load().rsk_hll_add_grouped_async(self.pool, ctypes.byref(ks), gp, op.fn, None), "PFADD")

    def count_async(self, out: np.ndarray, ids=None) -> "_lib.NativeOp":
        """PFCOUNT of every sketch (ids None) or of ids into `out` (uint64),
        written when the op completes."""
        n = self.n if ids is None else len(ids)
        if out.dtype != np.uint64 or out.size < n or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint64 array of at least %d entries" % n)
        idp = None
        if ids is not None:
            ids = np.ascontiguousarray(ids, dtype=np.uint64)
            idp = ids.ctypes.data
        op = _lib.NativeOp(out, ids)
        return op.issued(_lib.load().rsk_hll_count_ids_async(self.pool, idp, n, out.ctypes.data, op.fn, None),
                         "PFCOUNT")

    def countWith_async(self, member_ids, out: np.ndarray) -> "_lib.NativeOp":
        m = np.ascontiguousarray(member_ids, dtype=np.uint64)
        if m.ndim != 2:
            raise ValueError("member_ids must be [n, arity]")
        if out.dtype != np.uint64 or out.size < m.shape[0] or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint64 array of at least %d entries" % m.shape[0])
        op = _lib.NativeOp(m, out)
        return op.issued(_lib.load().rsk_hll_count_union_batch_async(self.pool, m.ctypes.data, m.shape[1], m.shape[0],
                                                                     out.ctypes.data, op.fn, None), "PFCOUNT")

    def mergeWith_async(self, dst_ids, src_ids) -> "_lib.NativeOp":
        d = np.ascontiguousarray(dst_ids, dtype=np.uint64)
        s = np.ascontiguousarray(src_ids, dtype=np.uint64)
        op = _lib.NativeOp(d, s)
        return op.issued(_lib.load().rsk_hll_merge_batch_async(self.pool, d.ctypes.data, s.ctypes.data, d.size, op.fn,
                                                               None), "PFMERGE")
