"""Host-side copy rates on the GPU box: pinned D2H / H2D DMA of 1 GiB (torch,
hipMemcpyAsync underneath) and host memcpy from a pinned buffer to a
pre-touched pageable one (1 and 8 threads) -- the two legs of the staged
export / import copies.  One JSON line."""
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

N = 1 << 30


def rate(fn, reps=5):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return N / best / 1e9


def main():
    dev = torch.empty(N, dtype=torch.uint8, device="cuda")
    dev.fill_(7)
    pin = torch.empty(N, dtype=torch.uint8, pin_memory=True)
    page = np.ones(N, np.uint8)
    out = {}

    def d2h():
        pin.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()

    def h2d():
        dev.copy_(pin, non_blocking=True)
        torch.cuda.synchronize()

    out["d2h_pinned_GBps"] = rate(d2h)
    out["h2d_pinned_GBps"] = rate(h2d)
    src = pin.numpy()
    out["memcpy_1t_GBps"] = rate(lambda: np.copyto(page, src))
    ex = ThreadPoolExecutor(8)
    step = N // 8

    def mt():
        list(ex.map(lambda i: np.copyto(page[i * step:(i + 1) * step], src[i * step:(i + 1) * step]), range(8)))

    out["memcpy_8t_GBps"] = rate(mt)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
