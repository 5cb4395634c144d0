"""The C2 step (addAll of 1B device-resident 16-byte keys + count) alone, with
route overrides, interleaved A/B in one process: ms per step (best of rounds),
kernel time per launch.  One JSON line.

  python scripts/c2_step_ab.py [steps] "route=v,...;route=v,..." """
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    forms = [dict(kv.split("=") for kv in f.split(",") if kv) for f in (sys.argv[2] if len(sys.argv) > 2 else ";").split(";")]
    _lib.load()
    _lib.diag()
    from redisson_amd.client import Config, Redisson

    client = Redisson.create(Config(device=0))
    eng = client.engine
    n = 1_000_000_000
    keys = devmem.gen_keys16(eng, 0x5EED0002, 0, n)
    kb = keys.keys_fixed(n, 16)
    hll = client.getHyperLogLog("c2ab")
    for _ in range(20):
        hll.addAll(kb)
        hll.count()
    res = {str(f): [] for f in forms}
    for rnd in range(3):
        for f in forms:
            eng.set_route("reset", 0)
            for k, v in f.items():
                eng.set_route(k, int(v))
            eng.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                hll.addAll(kb)
                hll.count()
            res[str(f)].append((time.perf_counter() - t0) / steps * 1e3)
    print(json.dumps({"steps": steps, "ms_per_step": {k: min(v) for k, v in res.items()}, "all": res}), flush=True)
    keys.free()
    client.shutdown()


if __name__ == "__main__":
    main()
