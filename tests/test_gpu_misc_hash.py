"""misc/Hash.hashToBase64 on the GPU (src/main/java/org/redisson/misc/Hash.java:29-40)
against an independent CPU form: python-xxhash for xx_r39, the pinned oracle
farmhash for farmUo, big-endian packing and the stdlib Base64."""
import base64
import struct

import numpy as np
import pytest
import xxhash

pytestmark = pytest.mark.gpu


def _ref(orc, b: bytes) -> str:
    h1 = orc.farmhash_uo64(b)
    h2 = xxhash.xxh64_intdigest(b, 0)
    return base64.b64encode(struct.pack(">QQ", h1, h2)).decode()[:-2]


def test_hash_to_base64_host_keys(engine, orc):
    from redisson_amd import Hash

    rng = np.random.default_rng(3)
    keys = [rng.integers(0, 256, int(rng.integers(0, 65)), dtype=np.uint8).tobytes() for _ in range(3000)]
    keys += [b"", b"a", b"\x00" * 64, b'"123"']
    got = Hash(engine).hashToBase64All(keys)
    assert got == [_ref(orc, k) for k in keys]
    assert all(len(s) == 22 for s in got)
    assert Hash(engine).hashToBase64(b"test") == _ref(orc, b"test")


def test_hash_to_base64_device_keys(engine, orc):
    from redisson_amd import Hash, devmem

    n = 100_000
    t = devmem.gen_keys16(engine, 0x5EED0002, 0, n)
    out = Hash(engine).hashToBase64All(t.keys_fixed(n, 16))
    raw = out.to_numpy(count=22 * n).tobytes()
    keys = orc.gen_keys16(0x5EED0002, 0, n).reshape(n, 16)
    for i in range(0, n, 997):
        assert raw[22 * i: 22 * i + 22].decode() == _ref(orc, keys[i].tobytes())
    out.free()
    t.free()
