"""BASELINE configs[0] (the reference's own CPU-runnable case) as a parity case:
RHyperLogLog.addAll of 1M random 8-byte longs + count(), default JsonJacksonCodec
(so each element hashes as ["java.lang.Long",v], JsonJacksonCodec.java:104-106).

The reference's addAll sends ONE element; its intended and
pipelined form is 1M PFADDs, which is what both sides compute here."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_C1 = 0x5EED0001


def _longs(orc, n):
    vals = [orc.splitmix64(SEED_C1 + i) for i in range(n)]
    return [v - (1 << 64) if v >= 1 << 63 else v for v in vals]  # Java signed long


def test_c1_addall_1m_longs_json(client, orc):
    from redisson_amd.codec import JavaLong, JsonJacksonCodec

    n = 1_000_000
    longs = _longs(orc, n)
    hll = client.getHyperLogLog("c1")
    assert hll.addAll([JavaLong(v) for v in longs]) is True
    enc = JsonJacksonCodec()
    blob, offs = orc.pack_keys([enc.encode(JavaLong(v)) for v in longs])
    ref = np.zeros(orc.REGISTERS, np.uint8)
    orc.hll_add(ref, blob, offs)
    assert np.array_equal(hll.registers(), ref)
    assert hll.count() == orc.hll_count_dense(ref)
    # the pipelined form (RBatch of add) gives the same sketch and per-command replies
    batch = client.createBatch()
    b = batch.getHyperLogLog("c1-pipelined")
    for v in longs[:20000]:
        b.addAsync(JavaLong(v))
    replies = batch.execute()
    r = orc.RedisModel()
    want = [bool(r.pfadd("p", enc.encode(JavaLong(v)))) for v in longs[:20000]]
    assert replies == want
    assert client.getHyperLogLog("c1-pipelined").count() == r.pfcount("p")
