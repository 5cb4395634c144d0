"""PFADD of host-resident 16-byte keys (pageable numpy: the JNI direct-buffer
case), host->device copies inside the timed region, with the chunks' copies on
the SDMA engine measured fastest (route io_engine=0) and on HIP's copies (-1),
interleaved.  One JSON line per form.

  python scripts/pcie_probe.py [n_keys] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import KeyBatch, Redisson, devmem  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    client = Redisson.create()
    eng = client.engine
    kd = devmem.gen_keys16(eng, 0x5EED0002, 0, n)
    host = kd.to_numpy()
    kd.free()
    kb = KeyBatch.from_numpy(host.reshape(-1, 16))
    hll = client.getHyperLogLog("pcie-probe")
    res = {}
    for _ in range(reps):
        for form in (0, -1):
            eng.set_route("io_engine", form)
            hll.addAll(kb)  # (warm)
            t0 = time.perf_counter()
            hll.addAll(kb)
            dt = time.perf_counter() - t0
            res.setdefault(form, []).append(round(16 * n / dt / 1e9, 2))
    eng.set_route("reset", 0)
    for form, v in res.items():
        print(json.dumps({"io_engine": form, "keys": n, "GBps_host_to_hbm": v,
                          "h2d_engine": eng.copy_engine(to_host=False)}), flush=True)
    client.shutdown()


if __name__ == "__main__":
    main()
