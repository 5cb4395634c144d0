"""CPU oracle for the Redisson sketch path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  It is the checker, never the
product: ``redisson_amd`` does not import it and fails loudly when its HIP
library is missing.

It wraps ``librsk_oracle.so`` (the C restatement in ``rsk_oracle.c``) and adds
``RedisModel``: a small model of the Redis 3.2.0 commands the reference
issues for this path (PFADD/PFCOUNT/PFMERGE, SETBIT/GETBIT/BITCOUNT, the
Bloom ``{name}__config`` hash), so tests can replay the reference's own JUnit
sequences (``T/RedissonHyperLogLogTest.java``, ``T/RedissonBloomFilterTest.java``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RSK_ORACLE_LIB: an alternative build (the ASan/UBSan one, tests/test_sanitizers.py)
LIB_PATH = os.environ.get("RSK_ORACLE_LIB", os.path.join(HERE, "librsk_oracle.so"))
REGISTERS = 16384
DENSE_SIZE = 16 + 12288
SPARSE_MAX_BYTES = 3000  # Redis hll-sparse-max-bytes default

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "orc_murmur64a": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]),
            "orc_xxh64": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]),
            "orc_farmhash_na64": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_size_t]),
            "orc_farmhash_uo64": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_size_t]),
            "orc_splitmix64": (ctypes.c_uint64, [ctypes.c_uint64]),
            "orc_hll_patlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_long)]),
            "orc_hll_add_raw": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_uint32, ctypes.c_uint64]),
            "orc_hll_add_gen16": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
            "orc_hll_add_gen_varlen": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_int]),
            "orc_hll_add_fixed_mt": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                                            ctypes.c_int]),
            "orc_hll_add_gen_grouped": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_uint64]),
            "orc_hll_add_gen_grouped_subset": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                      ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                      ctypes.c_int]),
            "orc_hll_add_gen_grouped_ids": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                   ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                   ctypes.c_uint64, ctypes.c_int]),
            "orc_hll_dense_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
            "orc_hll_raw_sum": (ctypes.c_double, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
            "orc_hll_dense_sum": (ctypes.c_double, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
            "orc_hll_estimate": (ctypes.c_uint64, [ctypes.c_double, ctypes.c_int]),
            "orc_hll_count_raw": (ctypes.c_uint64, [ctypes.c_void_p]),
            "orc_hll_count_dense_regs": (ctypes.c_uint64, [ctypes.c_void_p]),
            "orc_hll_records": (None, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]),
            "orc_hll_encode_dense": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
            "orc_hll_encode_sparse": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
            "orc_hll_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                              ctypes.POINTER(ctypes.c_int)]),
            "orc_hll_count_string": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u64p]),
            "orc_bloom_optimal_bits": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_double]),
            "orc_bloom_optimal_k": (ctypes.c_int32, [ctypes.c_int64, ctypes.c_int64]),
            "orc_bloom_indexes": (None, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64, _i64p]),
            "orc_bloom_count": (ctypes.c_int32, [ctypes.c_int64, ctypes.c_int, ctypes.c_int64]),
            "orc_bloom_add_batch": (None, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]),
            "orc_bloom_contains_batch": (None, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]),
            "orc_bloom_add_gen16_mt": (None, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
            "orc_bloom_contains_gen_queries_mt": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                                                    ctypes.c_int]),
            "orc_bloom_add_replies_sample_gen16_mt": (None, [ctypes.c_int64, ctypes.c_int, ctypes.c_uint64,
                                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                                             ctypes.c_void_p, ctypes.c_int]),
            "orc_setbit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]),
            "orc_getbit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
            "orc_bitcount": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint64]),
            "orc_gen_keys16": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]),
            "orc_gen_varlen_len": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint64]),
            "orc_gen_varlen_key": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]),
            "orc_zipf_cdf": (None, [ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p]),
            "orc_gen_grouped_zipf": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
            "orc_hll_add_gen_grouped_zipf_subset": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                           ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64,
                                                           ctypes.c_uint64, ctypes.c_int]),
            "orc_gen_grouped_groups": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_void_p, ctypes.c_int]),
            "orc_gen_grouped_zipf_groups": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, ctypes.c_uint64,
                                                   ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]),
            "orc_hll_add_keys_by_groups": (None, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                                  ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
            "orc_gen_grouped": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_void_p]),
            "orc_gen_queries16": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_void_p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- hashes
def murmur64a(b: bytes, seed: int = 0xADC83B19) -> int:
    return lib().orc_murmur64a(b, len(b), seed)


def xxh64(b: bytes, seed: int = 0) -> int:
    return lib().orc_xxh64(b, len(b), seed)


def farmhash_na64(b: bytes) -> int:
    return lib().orc_farmhash_na64(b, len(b))


def farmhash_uo64(b: bytes) -> int:
    return lib().orc_farmhash_uo64(b, len(b))


def splitmix64(x: int) -> int:
    return lib().orc_splitmix64(x & 0xFFFFFFFFFFFFFFFF)


def patlen(b: bytes):
    idx = ctypes.c_long()
    c = lib().orc_hll_patlen(b, len(b), ctypes.byref(idx))
    return idx.value, c


# ----------------------------------------------------------- key batches
def pack_keys(keys):
    """List of bytes -> (blob u8, offsets u64[n+1])."""
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
    blob = np.frombuffer(b"".join(keys), dtype=np.uint8).copy() if keys else np.zeros(1, np.uint8)
    return blob, offs


def gen_keys16(seed: int, start: int, n: int) -> np.ndarray:
    out = np.empty(n * 16, dtype=np.uint8)
    lib().orc_gen_keys16(seed, start, n, _ptr(out))
    return out


def gen_varlen(seed: int, start: int, n: int):
    lens = np.array([lib().orc_gen_varlen_len(seed, start + i) for i in range(n)], dtype=np.uint64)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = np.empty(int(offs[-1]) + 64, dtype=np.uint8)
    tmp = np.empty(64, dtype=np.uint8)
    for i in range(n):
        lib().orc_gen_varlen_key(seed, start + i, _ptr(tmp))
        blob[int(offs[i]):int(offs[i + 1])] = tmp[: int(lens[i])]
    return blob, offs


def gen_grouped(seed: int, G: int, start: int, n: int):
    groups = np.empty(n, dtype=np.uint32)
    keys = np.empty(n * 16, dtype=np.uint8)
    lib().orc_gen_grouped(seed, G, start, n, _ptr(groups), _ptr(keys))
    return groups, keys


def gen_queries16(qseed: int, iseed: int, n_ins: int, start: int, n: int) -> np.ndarray:
    out = np.empty(n * 16, dtype=np.uint8)
    lib().orc_gen_queries16(qseed, iseed, n_ins, start, n, _ptr(out))
    return out


# ------------------------------------------------------------------- HLL
def hll_add(regs: np.ndarray, data: np.ndarray, offsets=None, fixed_len: int = 0, n: int | None = None) -> int:
    assert regs.dtype == np.uint8 and regs.size == REGISTERS
    if n is None:
        n = (offsets.size - 1) if offsets is not None else data.size // fixed_len
    return int(lib().orc_hll_add_raw(_ptr(regs), _ptr(data),
                                     _ptr(offsets) if offsets is not None else None, fixed_len, n))


def hll_records(data: np.ndarray, fixed_len: int, n: int) -> np.ndarray:
    """index << 6 | rank of each key (Redis 3.2.0 hllPatLen)."""
    out = np.empty(n, np.uint32)
    lib().orc_hll_records(_ptr(np.ascontiguousarray(data, dtype=np.uint8)), fixed_len, n, _ptr(out))
    return out


def hll_add_fixed_mt(regs: np.ndarray, data: np.ndarray, fixed_len: int, n: int, nthreads: int):
    assert regs.dtype == np.uint8 and regs.size == REGISTERS and data.size >= n * fixed_len
    lib().orc_hll_add_fixed_mt(_ptr(regs), _ptr(data), fixed_len, n, nthreads)


def hll_add_gen_varlen(regs: np.ndarray, seed: int, start: int, n: int, nthreads: int = 1):
    lib().orc_hll_add_gen_varlen(_ptr(regs), seed, start, n, nthreads)


def hll_add_gen16(regs: np.ndarray, seed: int, start: int, n: int, nthreads: int = 1):
    lib().orc_hll_add_gen16(_ptr(regs), seed, start, n, nthreads)


def zipf_cdf(G: int, s: float) -> np.ndarray:
    cdf = np.zeros(G, np.uint64)
    lib().orc_zipf_cdf(G, s, _ptr(cdf))
    return cdf


def gen_grouped_zipf(seed: int, G: int, s: float, start: int, n: int):
    groups = np.zeros(n, np.uint32)
    keys = np.zeros(16 * n, np.uint8)
    lib().orc_gen_grouped_zipf(seed, G, s, start, n, _ptr(groups), _ptr(keys))
    return groups, keys


def hll_add_gen_grouped_zipf_subset(regs: np.ndarray, G: int, gsub: int, s: float, seed: int, start: int, n: int,
                                    nthreads: int = 1):
    assert regs.dtype == np.uint8 and regs.size == gsub * REGISTERS
    lib().orc_hll_add_gen_grouped_zipf_subset(_ptr(regs), G, gsub, s, seed, start, n, nthreads)


def gen_grouped_groups(seed: int, G: int, start: int, n: int, nthreads: int = 1) -> np.ndarray:
    """The groups of the uniform pair stream (orc_gen_grouped without the keys)."""
    groups = np.zeros(n, np.uint32)
    lib().orc_gen_grouped_groups(seed, G, start, n, _ptr(groups), nthreads)
    return groups


def gen_grouped_zipf_groups(seed: int, G: int, s: float, start: int, n: int, nthreads: int = 1) -> np.ndarray:
    """The groups of the Zipf pair stream (orc_gen_grouped_zipf without the keys)."""
    groups = np.zeros(n, np.uint32)
    lib().orc_gen_grouped_zipf_groups(seed, G, s, start, n, _ptr(groups), nthreads)
    return groups


def hll_add_keys_by_groups(regs: np.ndarray, G: int, groups: np.ndarray, seed: int, start: int, nthreads: int = 1):
    """A whole pool [G][16384] from the pairs whose groups are given and whose
    keys are the grouped streams' (rsk_oracle.c orc_hll_add_keys_by_groups)."""
    assert regs.dtype == np.uint8 and regs.size == G * REGISTERS and groups.dtype == np.uint32
    lib().orc_hll_add_keys_by_groups(_ptr(regs), G, _ptr(groups), seed, start, groups.size, nthreads)


def hll_add_gen_grouped(regs: np.ndarray, G: int, seed: int, start: int, n: int):
    lib().orc_hll_add_gen_grouped(_ptr(regs), G, seed, start, n)


def hll_count_raw(regs: np.ndarray) -> int:
    return int(lib().orc_hll_count_raw(_ptr(np.ascontiguousarray(regs, dtype=np.uint8))))


def hll_count_dense(regs: np.ndarray) -> int:
    return int(lib().orc_hll_count_dense_regs(_ptr(np.ascontiguousarray(regs, dtype=np.uint8))))


def hll_encode_dense(regs: np.ndarray, card: bytes = b"\x00" * 7 + b"\x80") -> bytes:
    out = np.zeros(DENSE_SIZE, dtype=np.uint8)
    c = np.frombuffer(card, dtype=np.uint8).copy()
    n = lib().orc_hll_encode_dense(_ptr(regs), _ptr(c), _ptr(out), out.size)
    assert n == DENSE_SIZE
    return out.tobytes()


def hll_encode_sparse(regs: np.ndarray, card: bytes = b"\x00" * 7 + b"\x80"):
    out = np.zeros(16 + 4 * REGISTERS, dtype=np.uint8)
    c = np.frombuffer(card, dtype=np.uint8).copy()
    n = lib().orc_hll_encode_sparse(_ptr(regs), _ptr(c), _ptr(out), out.size)
    return None if n < 0 else out[:n].tobytes()


def hll_decode(buf: bytes):
    raw = np.zeros(REGISTERS, dtype=np.uint8)
    enc = ctypes.c_int(-1)
    b = np.frombuffer(buf, dtype=np.uint8).copy() if buf else np.zeros(1, np.uint8)
    rc = lib().orc_hll_decode(_ptr(b), len(buf), _ptr(raw), ctypes.byref(enc))
    return rc, raw, enc.value


def hll_count_string(buf: bytes):
    out = ctypes.c_uint64()
    b = np.frombuffer(buf, dtype=np.uint8).copy()
    rc = lib().orc_hll_count_string(_ptr(b), len(buf), ctypes.byref(out))
    return rc, out.value


# ----------------------------------------------------------------- Bloom
def bloom_optimal_bits(n: int, p: float) -> int:
    return int(lib().orc_bloom_optimal_bits(n, p))


def bloom_optimal_k(n: int, m: int) -> int:
    return int(lib().orc_bloom_optimal_k(n, m))


def bloom_indexes(key: bytes, k: int, size: int):
    out = (ctypes.c_int64 * k)()
    lib().orc_bloom_indexes(key, len(key), k, size, out)
    return list(out)


def bloom_count(size: int, k: int, bitcount: int) -> int:
    return int(lib().orc_bloom_count(size, k, bitcount))


def bloom_add_batch(bits: np.ndarray, size: int, k: int, data, offsets=None, fixed_len=0, n=None, want=True):
    if n is None:
        n = (offsets.size - 1) if offsets is not None else data.size // fixed_len
    out = np.zeros(max(n, 1), dtype=np.uint8) if want else None
    lib().orc_bloom_add_batch(_ptr(bits), size, k, _ptr(data), _ptr(offsets) if offsets is not None else None,
                              fixed_len, n, _ptr(out) if want else None)
    return out[:n] if want else None


def bloom_contains_batch(bits: np.ndarray, size: int, k: int, data, offsets=None, fixed_len=0, n=None):
    if n is None:
        n = (offsets.size - 1) if offsets is not None else data.size // fixed_len
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().orc_bloom_contains_batch(_ptr(bits), size, k, _ptr(data), _ptr(offsets) if offsets is not None else None,
                                   fixed_len, n, _ptr(out))
    return out[:n]


def bitcount(bits: np.ndarray) -> int:
    return int(lib().orc_bitcount(_ptr(bits), bits.size))


# ------------------------------------------------------------ Redis model
class WrongType(Exception):
    """Redis -WRONGTYPE reply (RedisException in the reference)."""


class ConfigChanged(Exception):
    """Lua assert 'Bloom filter config has been changed' (RedissonBloomFilter.java:184,235)."""


def _card_bytes(c: int) -> bytes:
    return int(c).to_bytes(8, "little")


class _HLLKey:
    """A Redis 3.2.0 HLL string, held as raw registers + encoding + card[8]."""

    def __init__(self):
        self.regs = np.zeros(REGISTERS, dtype=np.uint8)
        self.dense = False
        self.card = bytearray(8)  # createHLLObject: card zeroed (cache valid, 0)

    def invalidate(self):
        self.card[7] |= 0x80

    def maybe_promote(self):
        if not self.dense:
            if int(self.regs.max()) > 32:
                self.dense = True
            else:
                sp = hll_encode_sparse(self.regs)
                if sp is None or len(sp) > SPARSE_MAX_BYTES:  # sdslen (header included), hllSparseSet
                    self.dense = True

    def to_string(self) -> bytes:
        if self.dense:
            return hll_encode_dense(self.regs, bytes(self.card))
        return hll_encode_sparse(self.regs, bytes(self.card))


class RedisModel:
    """The Redis 3.2.0 commands behind RedissonHyperLogLog / RedissonBloomFilter /
    RedissonBitSet, modelled over the oracle primitives (one logical db)."""

    def __init__(self):
        self.db: dict = {}

    # -- keyspace
    def delete(self, *names) -> int:
        return sum(1 for n in names if self.db.pop(n, None) is not None)

    def _hll(self, name, create=False):
        o = self.db.get(name)
        if o is None:
            if not create:
                return None
            o = _HLLKey()
            self.db[name] = o
            return o
        if not isinstance(o, _HLLKey):
            raise WrongType("WRONGTYPE Key is not a valid HyperLogLog string value.")
        return o

    # -- HLL (hyperloglog.c pfaddCommand / pfcountCommand / pfmergeCommand)
    def pfadd(self, name, *elements: bytes) -> int:
        o = self.db.get(name)
        updated = 0
        if o is None:
            o = self._hll(name, create=True)
            updated += 1
        else:
            o = self._hll(name)
        for e in elements:
            idx, c = patlen(e)
            if c > o.regs[idx]:
                o.regs[idx] = c
                updated += 1
            o.maybe_promote()
        if updated:
            o.invalidate()
        return 1 if updated else 0

    def pfcount(self, *names) -> int:
        if len(names) == 1:
            o = self._hll(names[0])
            if o is None:
                return 0
            rc, v = hll_count_string(o.to_string())
            assert rc == 0
            o.card[:] = _card_bytes(v)
            return v
        mx = np.zeros(REGISTERS, dtype=np.uint8)
        for n in names:
            o = self._hll(n)
            if o is not None:
                np.maximum(mx, o.regs, out=mx)
        return hll_count_raw(mx)

    def pfmerge(self, dest, *sources):
        mx = np.zeros(REGISTERS, dtype=np.uint8)
        for n in (dest,) + tuple(sources):
            o = self._hll(n)
            if o is not None:
                np.maximum(mx, o.regs, out=mx)
        o = self._hll(dest, create=True)
        o.dense = True
        o.regs[:] = mx
        o.invalidate()

    def get(self, name):
        o = self.db.get(name)
        if o is None:
            return None
        if isinstance(o, _HLLKey):
            return o.to_string()
        return bytes(o)

    def set(self, name, value: bytes):
        """SET of an HLL string (import) or a plain string (bitset)."""
        rc, raw, enc = hll_decode(value)
        if rc == 0:
            o = _HLLKey()
            o.regs[:] = raw
            o.dense = enc == 0
            o.card[:] = value[8:16]
            self.db[name] = o
        else:
            self.db[name] = bytearray(value)

    # -- bitops (bitops.c)
    def _bits(self, name, create_len=0):
        o = self.db.get(name)
        if o is None:
            o = bytearray()
            if create_len == 0:
                return o
            self.db[name] = o
        if isinstance(o, _HLLKey):
            raise WrongType("WRONGTYPE Operation against a key holding the wrong kind of value")
        if len(o) < create_len:
            o.extend(b"\x00" * (create_len - len(o)))
        return o

    def setbit(self, name, off: int, v: int) -> int:
        o = self._bits(name, (off >> 3) + 1)
        byte, bit = off >> 3, 7 - (off & 7)
        old = (o[byte] >> bit) & 1
        o[byte] = (o[byte] & ~(1 << bit)) | ((v & 1) << bit)
        return old

    def getbit(self, name, off: int) -> int:
        o = self._bits(name)
        byte = off >> 3
        if byte >= len(o):
            return 0
        return (o[byte] >> (7 - (off & 7))) & 1

    def bitcount(self, name) -> int:
        o = self._bits(name)
        if not o:
            return 0
        a = np.frombuffer(o, dtype=np.uint8)
        return int(lib().orc_bitcount(_ptr(a), a.size))

    def strlen(self, name) -> int:
        return len(self._bits(name))

    def bitop(self, op, dest, *srcs):
        vals = [bytes(self._bits(s)) for s in srcs]
        L = max((len(v) for v in vals), default=0)
        vals = [v + b"\x00" * (L - len(v)) for v in vals]
        if op == "NOT":
            res = bytes((~b) & 0xFF for b in vals[0])
        else:
            res = bytearray(vals[0])
            for v in vals[1:]:
                for i in range(L):
                    if op == "AND":
                        res[i] &= v[i]
                    elif op == "OR":
                        res[i] |= v[i]
                    elif op == "XOR":
                        res[i] ^= v[i]
            res = bytes(res)
        if L == 0:
            self.db.pop(dest, None)
        else:
            self.db[dest] = bytearray(res)
        return L

    # -- hash (Bloom config)
    def hgetall(self, name) -> dict:
        o = self.db.get(name)
        return dict(o) if isinstance(o, dict) else {}

    def hmset(self, name, mapping: dict):
        o = self.db.setdefault(name, {})
        o.update({k: str(v) for k, v in mapping.items()})


class OracleBloomFilter:
    """RedissonBloomFilter.java replayed against RedisModel (the checker for
    the GPU RBloomFilter; same names, argument meaning and exceptions)."""

    MAX_SIZE = 2147483647 * 2

    def __init__(self, redis: RedisModel, name: str, encode):
        self.r, self.name, self.encode = redis, name, encode
        self.size = 0
        self.k = 0

    def _config_name(self):
        return "{" + self.name + "}__config"

    def _read_config(self):
        cfg = self.r.hgetall(self._config_name())
        if cfg.get("hashIterations") is None or cfg.get("size") is None:
            raise RuntimeError("IllegalStateException: Bloom filter is not initialized!")
        self.size, self.k = int(cfg["size"]), int(cfg["hashIterations"])

    def try_init(self, n: int, p: float) -> bool:
        size = bloom_optimal_bits(n, p)
        if size > self.MAX_SIZE:
            raise ValueError("Bloom filter can't be greater than %d. But calculated size is %d" % (self.MAX_SIZE, size))
        k = bloom_optimal_k(n, size)
        if self.r.hgetall(self._config_name()):
            self._read_config()
            return False
        self.size, self.k = size, k
        self.r.hmset(self._config_name(), {"size": size, "hashIterations": k, "expectedInsertions": n,
                                            "falseProbability": repr(p)})
        return True

    def add(self, obj) -> bool:
        if self.size == 0:
            self._read_config()
        idx = bloom_indexes(self.encode(obj), self.k, self.size)
        res = [self.r.setbit(self.name, i, 1) == 0 for i in idx]
        return any(res[: len(res) - 1])

    def contains(self, obj) -> bool:
        if self.size == 0:
            self._read_config()
        idx = bloom_indexes(self.encode(obj), self.k, self.size)
        res = [self.r.getbit(self.name, i) == 1 for i in idx]
        return all(res[: len(res) - 1])

    def count(self) -> int:
        self._read_config()
        return bloom_count(self.size, self.k, self.r.bitcount(self.name))


def bloom_add_gen16_mt(bits: np.ndarray, size: int, k: int, seed: int, start: int, n: int, nthreads: int):
    lib().orc_bloom_add_gen16_mt(_ptr(bits), size, k, seed, start, n, nthreads)


def bloom_contains_gen_queries_mt(bits: np.ndarray, size: int, k: int, qseed: int, iseed: int, n_ins: int,
                                  start: int, n: int, out: np.ndarray | None, nthreads: int) -> int:
    return int(lib().orc_bloom_contains_gen_queries_mt(_ptr(bits), size, k, qseed, iseed, n_ins, start, n,
                                                       _ptr(out) if out is not None else None, nthreads))


def bloom_add_replies_sample_gen16_mt(size: int, k: int, seed: int, n: int, sample: np.ndarray,
                                      nthreads: int) -> np.ndarray:
    """add() replies of keys `sample` (ascending) when C3 stream keys 0..n-1 are
    added in one batch to an empty filter (rsk_oracle.c)."""
    sample = np.ascontiguousarray(sample, dtype=np.uint64)
    out = np.zeros(sample.size, np.uint8)
    lib().orc_bloom_add_replies_sample_gen16_mt(size, k, seed, n, _ptr(sample), sample.size, _ptr(out), nthreads)
    return out


def hll_add_gen_grouped_ids(regs: np.ndarray, G: int, ids: np.ndarray, seed: int, start: int, n: int,
                            nthreads: int = 1):
    """The C5 pair stream's registers for the (distinct) groups `ids` only:
    regs row s = group ids[s]."""
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    assert regs.dtype == np.uint8 and regs.size == ids.size * REGISTERS
    assert np.unique(ids).size == ids.size and (ids.size == 0 or int(ids.max()) < G)
    lib().orc_hll_add_gen_grouped_ids(_ptr(regs), G, _ptr(ids), ids.size, seed, start, n, nthreads)


def hll_add_gen_grouped_subset(regs: np.ndarray, G: int, gsub: int, seed: int, start: int, n: int,
                               nthreads: int = 1):
    assert regs.dtype == np.uint8 and regs.size == gsub * REGISTERS
    lib().orc_hll_add_gen_grouped_subset(_ptr(regs), G, gsub, seed, start, n, nthreads)
