"""ctypes binding of librsketch.so (include/rsketch.h) and of the test /
bench support library librsketch_diag.so (include/rsketch_diag.h: generators,
microbenchmarks, tuning variants, route overrides).

The HIP library is the only compute path: importing this module without the
built library, or creating an Engine without a gfx950 device, raises.  There
is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RSKETCH_LIB", os.path.join(HERE, "librsketch.so"))
DIAG_PATH = os.path.join(HERE, "librsketch_diag.so")

RSK_OK = 0
RSK_ERR_INVALID_ARG = 1
RSK_ERR_NOT_INITIALIZED = 2
RSK_ERR_WRONGTYPE = 3
RSK_ERR_INVALID_HLL = 4
RSK_ERR_DEVICE = 5
RSK_ERR_OUT_OF_MEMORY = 6
RSK_ERR_NO_DEVICE = 7

RSK_MEM_HOST = 0
RSK_MEM_DEVICE = 1
RSK_BLOOM_COMPAT = 0
RSK_BLOOM_EXTENDED = 1
RSK_FETCH_SELF = 1
HLL_REGISTERS = 16384
HLL_DENSE_BYTES = 12304
ABI_VERSION = 2  # include/rsketch.h RSK_ABI_VERSION


class RedissonError(Exception):
    """Base of the errors surfaced by the engine."""


class IllegalArgumentException(RedissonError, ValueError):
    """java.lang.IllegalArgumentException (RedissonBloomFilter.java:175,227)."""


class IllegalStateException(RedissonError, RuntimeError):
    """java.lang.IllegalStateException (RedissonBloomFilter.java:217,284)."""


class RedisException(RedissonError):
    """org.redisson.client.RedisException (-WRONGTYPE / -INVALIDOBJ replies)."""


class EngineError(RedissonError, RuntimeError):
    """HIP runtime, device-memory or no-device failure."""


_STATUS_EXC = {
    RSK_ERR_INVALID_ARG: IllegalArgumentException,
    RSK_ERR_NOT_INITIALIZED: IllegalStateException,
    RSK_ERR_WRONGTYPE: RedisException,
    RSK_ERR_INVALID_HLL: RedisException,
    RSK_ERR_DEVICE: EngineError,
    RSK_ERR_OUT_OF_MEMORY: EngineError,
    RSK_ERR_NO_DEVICE: EngineError,
}


class rsk_options(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("redis_version", ctypes.c_int32), ("staging_bytes", ctypes.c_uint64),
                ("stage_threads", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class rsk_keys(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("n", ctypes.c_uint64),
        ("fixed_len", ctypes.c_uint32),
        ("location", ctypes.c_uint32),
    ]


# name -> (restype, argtypes); every symbol declared in include/rsketch.h.
_vp, _u64, _u32, _i32, _i64, _sz = (ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32,
                                    ctypes.c_int64, ctypes.c_size_t)
_P = ctypes.POINTER
# rsk_done_fn: void (*)(void *user, int status, uint64_t value)
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64)

SIGNATURES = {
    "rsk_init": (ctypes.c_int, [_P(rsk_options), _P(_vp)]),
    "rsk_shutdown": (ctypes.c_int, [_vp]),
    "rsk_last_error": (ctypes.c_char_p, []),
    "rsk_abi_version": (ctypes.c_int, []),
    "rsk_ctx_stream": (_vp, [_vp]),
    "rsk_sync": (ctypes.c_int, [_vp]),
    "rsk_trim": (ctypes.c_int, [_vp]),
    "rsk_host_register": (ctypes.c_int, [_vp, _vp, _u64]),
    "rsk_host_unregister": (ctypes.c_int, [_vp, _vp]),
    "rsk_prof_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rsk_prof_reset": (ctypes.c_int, [_vp]),
    "rsk_prof_read": (ctypes.c_int, [_vp, ctypes.c_char_p, _P(ctypes.c_double), _P(_u64)]),
    "rsk_hll_create": (ctypes.c_int, [_vp, _u64, _P(_vp)]),
    "rsk_hll_destroy": (ctypes.c_int, [_vp]),
    "rsk_hll_size": (_u64, [_vp]),
    "rsk_hll_exists": (ctypes.c_int, [_vp, _u64, _P(ctypes.c_int)]),
    "rsk_hll_delete": (ctypes.c_int, [_vp, _u64]),
    "rsk_hll_clear": (ctypes.c_int, [_vp]),
    "rsk_hll_add": (ctypes.c_int, [_vp, _u64, _P(rsk_keys), _vp]),
    "rsk_hll_add_each": (ctypes.c_int, [_vp, _u64, _P(rsk_keys), _vp]),
    "rsk_hll_add_grouped": (ctypes.c_int, [_vp, _P(rsk_keys), _vp]),
    "rsk_hll_count": (ctypes.c_int, [_vp, _vp, _u64, _vp]),
    "rsk_hll_count_union": (ctypes.c_int, [_vp, _vp, _u32, _vp]),
    "rsk_hll_count_union_batch": (ctypes.c_int, [_vp, _vp, _u32, _u64, _vp]),
    "rsk_hll_merge": (ctypes.c_int, [_vp, _u64, _vp, _vp, _u32]),
    "rsk_hll_merge_batch": (ctypes.c_int, [_vp, _vp, _vp, _u64]),
    "rsk_hll_merge_raw": (ctypes.c_int, [_vp, _u64, _vp, _u32]),
    "rsk_hll_add_async": (ctypes.c_int, [_vp, _u64, _P(rsk_keys), DONE_FN, _vp]),
    "rsk_hll_count_async": (ctypes.c_int, [_vp, _u64, DONE_FN, _vp]),
    "rsk_hll_count_union_async": (ctypes.c_int, [_vp, _vp, _u32, DONE_FN, _vp]),
    "rsk_hll_merge_async": (ctypes.c_int, [_vp, _u64, _vp, _vp, _u32, DONE_FN, _vp]),
    "rsk_hll_merge_batch_async": (ctypes.c_int, [_vp, _vp, _vp, _u64, DONE_FN, _vp]),
    "rsk_hll_add_grouped_async": (ctypes.c_int, [_vp, _P(rsk_keys), _vp, DONE_FN, _vp]),
    "rsk_hll_count_ids_async": (ctypes.c_int, [_vp, _vp, _u64, _vp, DONE_FN, _vp]),
    "rsk_hll_count_union_batch_async": (ctypes.c_int, [_vp, _vp, _u32, _u64, _vp, DONE_FN, _vp]),
    "rsk_hll_get_registers": (ctypes.c_int, [_vp, _u64, _vp, _u32]),
    "rsk_hll_device_registers": (_vp, [_vp]),
    "rsk_hll_export_redis": (ctypes.c_int, [_vp, _u64, _vp, _sz, _P(_sz)]),
    "rsk_hll_import_redis": (ctypes.c_int, [_vp, _u64, _vp, _sz]),
    "rsk_hll_export_redis_batch": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u64, _vp]),
    "rsk_hll_import_redis_batch": (ctypes.c_int, [_vp, _vp, _u64, _vp, _vp]),
    "rsk_bloom_params": (ctypes.c_int, [_i64, ctypes.c_double, _u32, _P(_i64), _P(_i32)]),
    "rsk_bloom_create": (ctypes.c_int, [_vp, _i64, _i32, _P(_vp)]),
    "rsk_bloom_init": (ctypes.c_int, [_vp, _i64, ctypes.c_double, _u32, _P(_vp), _P(_i64), _P(_i32)]),
    "rsk_bloom_destroy": (ctypes.c_int, [_vp]),
    "rsk_bloom_info": (ctypes.c_int, [_vp, _P(_i64), _P(_i32)]),
    "rsk_bloom_add": (ctypes.c_int, [_vp, _P(rsk_keys), _vp]),
    "rsk_bloom_contains": (ctypes.c_int, [_vp, _P(rsk_keys), _vp]),
    "rsk_bloom_count": (ctypes.c_int, [_vp, _P(_i32)]),
    "rsk_bloom_add_async": (ctypes.c_int, [_vp, _P(rsk_keys), _vp, DONE_FN, _vp]),
    "rsk_bloom_contains_async": (ctypes.c_int, [_vp, _P(rsk_keys), _vp, DONE_FN, _vp]),
    "rsk_bloom_bitcount": (ctypes.c_int, [_vp, _P(_u64)]),
    "rsk_hash_to_base64": (ctypes.c_int, [_vp, _P(rsk_keys), _vp]),
    "rsk_bloom_export_bits": (ctypes.c_int, [_vp, _vp, _sz, _P(_sz)]),
    "rsk_bloom_import_bits": (ctypes.c_int, [_vp, _vp, _sz]),
    "rsk_bloom_or_bits": (ctypes.c_int, [_vp, _vp, _sz, _u32]),
    "rsk_bloom_device_bits": (_vp, [_vp]),
    "rsk_bitset_create": (ctypes.c_int, [_vp, _P(_vp)]),
    "rsk_bitset_destroy": (ctypes.c_int, [_vp]),
    "rsk_bitset_strlen": (ctypes.c_int, [_vp, _P(_u64)]),
    "rsk_bitset_setbits": (ctypes.c_int, [_vp, _vp, _u64, ctypes.c_int, _u32]),
    "rsk_bitset_getbits": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp]),
    "rsk_bitset_set_range": (ctypes.c_int, [_vp, _u64, _u64, ctypes.c_int]),
    "rsk_bitset_bitcount": (ctypes.c_int, [_vp, _P(_u64)]),
    "rsk_bitset_length": (ctypes.c_int, [_vp, _P(_u64)]),
    "rsk_bitset_bitop": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _u32]),
    "rsk_bitset_get_bytes": (ctypes.c_int, [_vp, _vp, _sz, _P(_sz)]),
    "rsk_bitset_set_bytes": (ctypes.c_int, [_vp, _vp, _sz]),
    "rsk_bitset_clear": (ctypes.c_int, [_vp]),
    "rsk_bloom_bitset": (ctypes.c_int, [_vp, _P(_vp)]),
    "rsk_dev_alloc": (ctypes.c_int, [_vp, _u64, _P(_vp)]),
    "rsk_dev_free": (ctypes.c_int, [_vp, _vp]),
    "rsk_memcpy": (ctypes.c_int, [_vp, _vp, _vp, _u64, _u32]),
    "rsk_memset": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _u64]),
    "rsk_comm_unique_id": (ctypes.c_int, [_vp]),
    "rsk_comm_init": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp]),
    "rsk_comm_destroy": (ctypes.c_int, [_vp]),
    "rsk_comm_info": (ctypes.c_int, [_vp, _P(ctypes.c_int), _P(ctypes.c_int)]),
    "rsk_hll_allreduce": (ctypes.c_int, [_vp, _u64]),
    "rsk_hll_allreduce_pool": (ctypes.c_int, [_vp]),
    "rsk_hll_reducescatter_pool": (ctypes.c_int, [_vp, _P(_u64), _P(_u64)]),
    "rsk_hll_fetch_rows": (ctypes.c_int, [_vp, _vp, _u64]),
    "rsk_hll_add_grouped_routed": (ctypes.c_int, [_vp, _P(rsk_keys), _vp, _u32, _P(_u64), _P(_u64)]),
    "rsk_hll_fetch_rows_flags": (ctypes.c_int, [_vp, _vp, _u64, _u32]),
    "rsk_plan_shard_range": (ctypes.c_int, [_u64, ctypes.c_int, ctypes.c_int, _P(_u64), _P(_u64)]),
    "rsk_plan_owned_range": (ctypes.c_int, [_u64, ctypes.c_int, ctypes.c_int, _P(_u64), _P(_u64)]),
    "rsk_plan_owner": (ctypes.c_int, [_u64, ctypes.c_int, _u64, _P(ctypes.c_int)]),
    "rsk_plan_bloom_slice_words": (ctypes.c_int, [_u64, ctypes.c_int, _P(_u64)]),
    "rsk_plan_fetch": (ctypes.c_int, [_u64, ctypes.c_int, ctypes.c_int, _vp, _u64, _u32, _vp, _P(_u64), _vp]),
    "rsk_plan_route_recv": (ctypes.c_int, [_vp, _u64, ctypes.c_int, _u64, _u64, _vp, _vp, _vp]),
    "rsk_bloom_allreduce_or": (ctypes.c_int, [_vp]),
    "rsk_bloom_allreduce_or_flags": (ctypes.c_int, [_vp, _u32]),
}

DIAG_SIGNATURES = {
    "rsk_diag_last_error": (ctypes.c_char_p, []),
    "rsk_diag_set_route": (ctypes.c_int, [_vp, ctypes.c_char_p, _i64]),
    "rsk_diag_reply_stats": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "rsk_diag_copy_engine": (ctypes.c_int, [_vp, ctypes.c_int, _P(ctypes.c_int), _P(ctypes.c_float)]),
    "rsk_diag_mark_dead": (ctypes.c_int, [_vp]),
    "rsk_diag_membench": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _u64, _u64, _P(ctypes.c_double)]),
    "rsk_diag_p2p_probe": (ctypes.c_int, [_vp, _u64, ctypes.c_int, _P(_u64), _P(_u64)]),
    "rsk_diag_hll_variant": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _u64, _P(ctypes.c_double)]),
    "rsk_diag_bloom_contains_variant": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _u64, _vp,
                                                       _P(ctypes.c_double)]),
    "rsk_diag_hll_var_variant": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _u64, _P(ctypes.c_double)]),
    "rsk_diag_bloom_contains_probes": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _P(_u64)]),
    "rsk_gen_keys16": (ctypes.c_int, [_vp, _u64, _u64, _u64, _vp]),
    "rsk_gen_grouped": (ctypes.c_int, [_vp, _u64, _u64, _u64, _u64, _vp, _vp]),
    "rsk_gen_grouped_zipf": (ctypes.c_int, [_vp, _u64, _u64, ctypes.c_double, _u64, _u64, _vp, _vp]),
    "rsk_gen_queries16": (ctypes.c_int, [_vp, _u64, _u64, _u64, _u64, _u64, _vp]),
    "rsk_gen_varlen": (ctypes.c_int, [_vp, _u64, _u64, _u64, _vp, _vp, _u64, _P(_u64)]),

}

_lib = None
_diag = None
_lock = threading.Lock()


def load():
    """Load librsketch.so; raises if it has not been built (no fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    "librsketch.so not found at %s: build it with `make` (or __graft_entry__.build()). "
                    "redisson_amd has no CPU fallback." % LIB_PATH)
            L = ctypes.CDLL(LIB_PATH)
            # The HIP runtime dlopens libamd_comgr.so.3 by soname the first time it
            # reads a code object's metadata (occupancy queries, hipcub grid
            # sizing).  torch ships its own copy of that soname: imported first, it
            # would satisfy that dlopen and the system runtime would misread our
            # kernels (hipOccupancyMaxActiveBlocksPerMultiprocessor answered 1,
            # scripts/occ_probe.py).  Binding the system copy now wins the soname.
            comgr = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamd_comgr.so.3")
            if os.path.exists(comgr):
                ctypes.CDLL(comgr, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.rsk_abi_version() != ABI_VERSION:
                raise ImportError("librsketch.so has ABI %d, this binding expects %d: rebuild it"
                                  % (L.rsk_abi_version(), ABI_VERSION))
            _lib = L
    return _lib


def foreign_hip_runtime():
    """Path of a HIP runtime (libamdhip64) mapped into this process from
    outside the ROCm install -- torch's bundled copy, once `import torch` has
    run -- or None."""
    rocm = os.path.realpath(os.environ.get("ROCM_PATH", "/opt/rocm"))
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6 and "libamdhip64" in parts[5]:
                    path = os.path.realpath(parts[5].strip())
                    if not path.startswith(rocm + os.sep) and not path.startswith("/opt/rocm"):
                        return path
    except OSError:
        return None
    return None


def diag():
    """librsketch_diag.so (test / bench support: generators, microbenchmarks,
    tuning variants, route overrides).  Never used by the product path.

    It must be loaded before torch: loaded after torch's own HIP runtime is
    mapped, rocprofv3 crashed through a null dispatch entry (round 3, commit
    c380052).  A late first load is therefore refused."""
    global _diag
    load()  # the product library (and the system comgr) first
    with _lock:
        if _diag is None:
            foreign = foreign_hip_runtime()
            if foreign is not None:
                raise ImportError(
                    "librsketch_diag.so must be loaded before torch: a foreign HIP runtime (%s) is already "
                    "mapped in this process; call redisson_amd._lib.diag() before `import torch`" % foreign)
            if not os.path.exists(DIAG_PATH):
                raise ImportError("librsketch_diag.so not found at %s: build it with `make`" % DIAG_PATH)
            D = ctypes.CDLL(DIAG_PATH)
            for name, (res, args) in DIAG_SIGNATURES.items():
                fn = getattr(D, name)
                fn.restype = res
                fn.argtypes = args
            _diag = D
    return _diag


def check_diag(rc: int, what: str = ""):
    if rc != RSK_OK:
        msg = diag().rsk_diag_last_error().decode(errors="replace")
        exc = _STATUS_EXC.get(rc, EngineError)
        raise exc(msg if not what else "%s: %s" % (what, msg))


def check(rc: int, what: str = ""):
    if rc != RSK_OK:
        msg = load().rsk_last_error().decode(errors="replace")
        exc = _STATUS_EXC.get(rc, EngineError)
        raise exc(msg if not what else "%s: %s" % (what, msg))


class NativeOp:
    """One asynchronous library call (rsk_*_async): `fn` is the completion
    callback to pass, `wait()` blocks until it fired and returns its value.
    Objects in `keep` (input and output buffers) stay referenced until then."""

    def __init__(self, *keep):
        self._ev = threading.Event()
        self.status = None
        self.value = None
        self._keep = keep

        def done(user, status, value):
            self.status = status
            self.value = value
            self._ev.set()

        self.fn = DONE_FN(done)

    def issued(self, rc: int, what: str = "async call"):
        """The call's own status: on failure the callback never fires."""
        if rc != RSK_OK:
            self._keep = None
            check(rc, what)
        return self

    def wait(self, timeout=None):
        if not self._ev.wait(timeout):
            raise TimeoutError("asynchronous call did not complete")
        self._keep = None
        if self.status != RSK_OK:
            raise EngineError("asynchronous call failed with status %d" % self.status)
        return self.value


class Engine:
    """One rsk_ctx: a HIP stream and scratch on one GPU (one process per GPU)."""

    _engines: dict = {}
    _elock = threading.Lock()

    def __init__(self, device: int = 0, staging_bytes: int = 0):
        L = load()
        opts = rsk_options(device, 320, staging_bytes)
        h = ctypes.c_void_p()
        check(L.rsk_init(ctypes.byref(opts), ctypes.byref(h)), "rsk_init")
        self.ctx = h
        self.device = device
        self.lib = L

    @classmethod
    def get(cls, device: int = 0) -> "Engine":
        with cls._elock:
            e = cls._engines.get(device)
            if e is None:
                e = cls._engines[device] = Engine(device)
            return e

    def stream(self) -> int:
        return self.lib.rsk_ctx_stream(self.ctx)

    def sync(self):
        check(self.lib.rsk_sync(self.ctx))

    def host_register(self, arr):
        """Pin a numpy array's memory in place (rsk_host_register): transfers
        to / from it skip the library's pinned stages.  Keep `arr` alive until
        host_unregister(arr)."""
        check(self.lib.rsk_host_register(self.ctx, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr):
        check(self.lib.rsk_host_unregister(self.ctx, arr.ctypes.data))

    def prof_enable(self, on=True):
        check(self.lib.rsk_prof_enable(self.ctx, 1 if on else 0))

    def prof_reset(self):
        check(self.lib.rsk_prof_reset(self.ctx))

    def prof_read(self, name: str):
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        check(self.lib.rsk_prof_read(self.ctx, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def set_route(self, name: str, value: int):
        """Route override of this context (rsk_diag_set_route): tests force
        every pipeline of the library; "reset" restores the automatic routes."""
        check_diag(diag().rsk_diag_set_route(self.ctx, name.encode(), int(value)), "rsk_diag_set_route")

    def reply_stats(self):
        """(groups whose pending reply probes were resolved in LDS, chunks
        answered by the sort-path fallback) of this context (rsk_diag_reply_stats)."""
        pg, fb = ctypes.c_uint64(), ctypes.c_uint64()
        check_diag(diag().rsk_diag_reply_stats(self.ctx, ctypes.byref(pg), ctypes.byref(fb)), "rsk_diag_reply_stats")
        return pg.value, fb.value

    def copy_engine(self, to_host=True):
        """(engine, rates): the SDMA engine of this context's batched-export (to_host) or
        batched-import copies (-2 not measured yet, -1 HIP's copies) and the GB/s measured in
        that direction on engines 0..7 (rsk_diag_copy_engine)."""
        e = ctypes.c_int()
        r = (ctypes.c_float * 8)()
        check_diag(diag().rsk_diag_copy_engine(self.ctx, int(bool(to_host)), ctypes.byref(e), r),
                   "rsk_diag_copy_engine")
        return e.value, [round(float(x), 2) for x in r]

    def routes(self, **kw):
        """Context manager: the given route overrides, then automatic routes."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            for k, v in kw.items():
                self.set_route(k, v)
            try:
                yield self
            finally:
                self.set_route("reset", 0)

        return cm()

    def close(self):
        if self.ctx:
            self.lib.rsk_shutdown(self.ctx)
            self.ctx = None
