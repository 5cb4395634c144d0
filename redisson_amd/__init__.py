"""redisson_amd -- MI355X (gfx950) sketch engine behind Redisson's
RHyperLogLog / RBloomFilter (alexs20/redisson, Redisson 2.2.17).

The compute path is librsketch.so (hand-written HIP kernels + a C ABI,
include/rsketch.h); this package is the host-side mirror of the reference's
Java object API.  It has no CPU fallback: without the built library or a
gfx950 GPU every sketch operation raises.
"""
from ._lib import (EngineError, IllegalArgumentException, IllegalStateException, RedisException,  # noqa: F401
                   RedissonError, Engine)
from .codec import (ByteArrayCodec, JavaInteger, JavaLong, JsonJacksonCodec, LongCodec,  # noqa: F401
                    StringCodec)
from .keys import KeyBatch  # noqa: F401

__all__ = [
    "Redisson", "Config", "RHyperLogLog", "RBloomFilter", "GroupedHyperLogLog", "KeyBatch", "Engine",
    "JsonJacksonCodec", "StringCodec", "LongCodec", "ByteArrayCodec", "JavaLong", "JavaInteger",
    "IllegalArgumentException", "IllegalStateException", "RedisException", "EngineError", "RedissonError", "Hash",
]


def __getattr__(name):
    # Lazy: importing the package must not touch the GPU.
    if name in ("Redisson", "Config"):
        from . import client

        return getattr(client, name)
    if name in ("RHyperLogLog", "GroupedHyperLogLog"):
        from . import hyperloglog

        return getattr(hyperloglog, name)
    if name == "RBloomFilter":
        from . import bloom

        return bloom.RBloomFilter
    if name == "Hash":
        from . import misc

        return misc.Hash
    raise AttributeError(name)
