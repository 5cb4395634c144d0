"""org.redisson.misc.Hash on the GPU (src/main/java/org/redisson/misc/Hash.java:29-40).

hashToBase64(objectState) = Base64(bigEndian(farmUo(bytes)) || bigEndian(xx_r39(bytes)))
without its trailing "==": the 22-character suffix RedissonMultimap (:62) and
RedissonCache (:160) build key names from.  The batched form hashes a whole
KeyBatch in one kernel (the same xxHash64 / FarmHash-uo device code the Bloom
filter uses)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .keys import KeyBatch

B64_LEN = 22


class Hash:
    def __init__(self, engine):
        self.engine = engine

    def hashToBase64All(self, keys) -> list | "object":
        """One 22-char string per key (host keys), or a DeviceBuffer of
        22*n ASCII bytes (device keys)."""
        kb = keys if isinstance(keys, KeyBatch) else KeyBatch.from_bytes_list([bytes(k) for k in keys])
        ks = kb.as_struct()
        if kb.on_device:
            from .devmem import DeviceBuffer

            out = DeviceBuffer(self.engine, max(1, B64_LEN * kb.n))
            _lib.check(_lib.load().rsk_hash_to_base64(self.engine.ctx, ctypes.byref(ks), out.ptr), "hashToBase64")
            return out
        out = np.zeros(max(1, B64_LEN * kb.n), np.uint8)
        _lib.check(_lib.load().rsk_hash_to_base64(self.engine.ctx, ctypes.byref(ks), out.ctypes.data), "hashToBase64")
        raw = out[: B64_LEN * kb.n].tobytes()
        return [raw[B64_LEN * i: B64_LEN * (i + 1)].decode("ascii") for i in range(kb.n)]

    def hashToBase64(self, objectState: bytes) -> str:
        return self.hashToBase64All([objectState])[0]
