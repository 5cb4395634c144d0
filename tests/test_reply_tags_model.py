"""The group-tag rule behind rsk_bloom_reply.hip, restated in Python and
checked against the oracle's sequential SETBITs (RedissonBloomFilter.java:100-107)
on the CPU: T[bit] = (smallest group tag << 1) | (that group probed it once),
NONE where the bit was set before the batch; key i answers true at the first
t < k-1 with T == tag(i) << 1 | 1, and pending bits (T == tag(i) << 1) are
resolved by the smallest (key, t) probe of the group.  Tiny groups and a
small filter make the pending case common here (it is rare at C3)."""
import numpy as np
import pytest

NONE = 0xFFFF


def model_replies(orc, bits, size, k, keys, group):
    n = len(keys)
    probes = [orc.bloom_indexes(x, k, size) for x in keys]
    tag = [i // group for i in range(n)]

    def was_set(b):
        return (bits[b >> 3] >> (7 - (b & 7))) & 1

    # rp_tapply: per bit, (min tag, probes of that tag)
    best = {}
    for i, ps in enumerate(probes):
        for b in ps:
            t, c = best.get(b, (1 << 30, 0))
            if tag[i] < t:
                best[b] = (tag[i], 1)
            elif tag[i] == t:
                best[b] = (t, c + 1)
    T = {b: (NONE if was_set(b) else (t << 1) | (1 if c == 1 else 0)) for b, (t, c) in best.items()}
    out = np.zeros(n, np.uint8)
    pending = []
    for i, ps in enumerate(probes):  # rp_treply
        yes, pend = False, []
        for t in range(k - 1):
            e = T[ps[t]]
            if e >> 1 == tag[i]:
                if e & 1:
                    yes = True
                    break
                pend.append(t)
        out[i] = yes
        if not yes and pend:
            pending.append((i, pend))
    for i, pend in pending:  # the group's smallest (key, t) per pending bit
        g0 = tag[i] * group
        for t in pend:
            b = probes[i][t]
            first = min((j, tt) for j in range(g0, min(n, g0 + group)) for tt, bb in enumerate(probes[j]) if bb == b)
            if first == (i, t):
                out[i] = 1
    for i, ps in enumerate(probes):  # the filter after the batch
        for b in ps:
            bits[b >> 3] |= 0x80 >> (b & 7)
    return out, len(pending)


@pytest.mark.parametrize("size,k,n,group", [(3001, 7, 600, 50), (997, 5, 300, 7), (20011, 9, 800, 64), (64, 3, 200, 16)])
def test_group_tag_rule_matches_sequential_setbits(orc, size, k, n, group):
    rng = np.random.default_rng(size)
    base = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(n)]
    keys = base + base[: n // 5] + [base[3]] * 5  # repeats: bits first probed inside the batch
    rng.shuffle(keys)
    bits = np.zeros((size + 7) // 8, np.uint8)
    pre = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(n // 4)]
    ref = bits.copy()
    orc.bloom_add_batch(ref, size, k, *orc.pack_keys(pre))  # some bits set before the batch
    bits[:] = ref
    got, npend = model_replies(orc, bits, size, k, keys, group)
    blob, offs = orc.pack_keys(keys)
    want = orc.bloom_add_batch(ref, size, k, blob, offs)
    assert np.array_equal(got, want)
    assert np.array_equal(bits, ref)
    assert npend > 0  # the pending path was exercised
