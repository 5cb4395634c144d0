"""Redis 3.2.0 hllCount restated in Python doubles (shared by the CPU pin test
and the GPU estimator-branch test).  Test infrastructure only."""
import numpy as np


def redis32_hllcount_raw(regs: np.ndarray) -> int:
    """hllCount of Redis 3.2.0 (hyperloglog.c), restated line by line in Python
    doubles (IEEE binary64, evaluated in C's order, glibc log) for the raw
    encoding's register order (hllRawSum: u64 words of 8 registers)."""
    import math

    m = 16384.0
    alpha = 0.7213 / (1 + 1.079 / m)
    PE = [1.0] + [1.0 / (1 << j) for j in range(1, 64)]
    E, ez = 0.0, 0
    r = regs.astype(np.int64).tolist()
    for w in range(0, 16384, 8):
        word = r[w:w + 8]
        if not any(word):
            ez += 8
            E += 8.0  # hllRawSum adds 8 (PE[0] * 8) for an all-zero word
            continue
        for v in word:
            if v == 0:
                ez += 1
            E += PE[v]
    E = (1 / E) * alpha * m * m
    branch = "raw"
    if E < m * 2.5 and ez != 0:
        E = m * math.log(m / ez)
        branch = "linear"
    elif m == 16384 and E < 72000:
        bias = 5.9119 * 1.0e-18 * (E * E * E * E) - 1.4253 * 1.0e-12 * (E * E * E) + \
            1.2940 * 1.0e-7 * (E * E) - 5.2921 * 1.0e-3 * E + 83.3216
        E -= E * (bias / 100)
        branch = "bias"
    return int(E), branch
