"""Host restatement of the device probe arithmetic (rsk_device.h: fastmod63,
ProbeSeq; and scripts/bloom_chain_bench.hip's fastmod63_big, measured and not
adopted) in Python integers, checked against the plain definition
idx_t = (h_t & Long.MAX_VALUE) % size of RedissonBloomFilter.java:116-131.
The GPU runs the same formulas (the chain bench checks them on the device);
this pins the bounds they rely on: one correction per probe step, one after
fastmod63_big."""
import random

MASK64 = (1 << 64) - 1
MAX63 = (1 << 63) - 1


def fastmod_params(d):
    l = 0
    while (1 << l) < d:
        l += 1
    M = (((1 << (63 + l)) + d - 1) // d) if l else 0
    return d, M, l, (1 << 63) % d


def fastmod63(x, f):
    d, M, l, _ = f
    if l == 0:
        return 0
    q = ((x * M) >> 64) >> (l - 1)
    return x - q * d


def fastmod63_big(x, f):
    d, M, l, _ = f
    p = (x >> 31) * (M >> 32)  # 32 x 32 -> 64
    q = p >> l
    assert q < (1 << 31)
    r = x - q * d
    assert 0 <= r < 2 * d, (x, d)
    return r - d if r >= d else r


def fastmod63_any(x, f):
    return fastmod63_big(x, f) if f[2] >= 33 else fastmod63(x, f)


def probes(h1, h2, f, k):
    d, _, _, r63 = f
    v1, v2 = h1 & MAX63, h2 & MAX63
    r1, r2 = fastmod63(v1, f), fastmod63(v2, f)
    r1c = r1 - r63 if r1 >= r63 else r1 + (d - r63)
    r2c = r2 - r63 if r2 >= r63 else r2 + (d - r63)
    v, idx, out = v1, r1, []
    for t in range(k):
        out.append(idx)
        if t + 1 == k:
            break
        s = v + (v1 if t & 1 else v2)
        c = s >> 63
        x = idx + ((r1c if c else r1) if t & 1 else (r2c if c else r2))
        assert x < 2 * d
        idx = x - d if x >= d else x
        v = s & MAX63
    return out


def reference_probes(h1, h2, d, k):
    h, out = h1, []
    for t in range(k):
        out.append((h & MAX63) % d)
        h = (h + (h2 if t % 2 == 0 else h1)) & MASK64
    return out


SIZES = [1, 2, 3, 1000, 9585058, (1 << 31) - 1, 1 << 31, (1 << 31) + 1, (1 << 32) - 1, 1 << 32, (1 << 32) + 1,
         (1 << 33) - 1, 1 << 33, (1 << 33) + 1, 9585058378, 95850583780, (1 << 40) - 3, (1 << 53) + 1,
         (1 << 62) + 5, MAX63]


def test_fastmod_boundaries():
    rng = random.Random(5)
    for d in SIZES:
        f = fastmod_params(d)
        qmax = MAX63 // d
        xs = [0, 1, MAX63, MAX63 - 1, d - 1, d, d + 1]
        for _ in range(300):
            m = rng.randrange(qmax + 1)
            xs += [m * d + e for e in (-2, -1, 0, 1, 2)]
        xs += [rng.randrange(1 << 63) for _ in range(300)]
        for x in xs:
            if 0 <= x <= MAX63:
                assert fastmod63(x, f) == x % d, (x, d)
                assert fastmod63_any(x, f) == x % d, (x, d)


def test_probe_sequence_matches_definition():
    rng = random.Random(7)
    for d in SIZES:
        f = fastmod_params(d)
        for _ in range(200):
            h1, h2 = rng.getrandbits(64), rng.getrandbits(64)
            for k in (1, 2, 7, 16):
                assert probes(h1, h2, f, k) == reference_probes(h1, h2, d, k)
        # addends near 2^63 (a carry at every step)
        for h1, h2 in ((MAX63, MAX63), (1 << 63, (1 << 63) - 1), (MASK64, MASK64), (0, MAX63)):
            assert probes(h1, h2, f, 9) == reference_probes(h1, h2, d, 9)
