"""Bloom insert (C3 size, no replies) under diag routes: per-stage times
(interleaved rounds, median) and the resulting filter's popcount, which must
agree across routes.  python scripts/insert_routes.py OUT.json ROUTESPEC...
ROUTESPEC = name=value[,name=value...] or "default"."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

STAGES = ("bloom_st1", "bloom_st_mid", "bloom_st2", "bloom_st_apply", "bloom_add16")


def parse(spec):
    if spec == "default":
        return {}
    return {kv.split("=")[0]: int(kv.split("=")[1]) for kv in spec.split(",")}


def main():
    out_path = sys.argv[1]
    specs = sys.argv[2:] or ["default"]
    n = int(os.environ.get("N_KEYS", 1_000_000_000))
    rounds = int(os.environ.get("ROUNDS", 3))
    L = _lib.load()
    eng = _lib.Engine(0)
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    ins = devmem.gen_keys16(eng, 0x5EED0003, 0, n)
    ks = ins.keys_fixed(n, 16).as_struct()
    res = {s: {st: [] for st in STAGES} for s in specs}
    bits = {}
    for _ in range(rounds):
        for s in specs:
            eng.set_route("reset", 0)
            for name, v in parse(s).items():
                eng.set_route(name, v)
            b = ctypes.c_void_p()
            _lib.check(L.rsk_bloom_create(eng.ctx, size.value, k.value, ctypes.byref(b)))
            eng.prof_reset()
            eng.prof_enable(True)
            _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
            eng.sync()
            eng.prof_enable(False)
            for st in STAGES:
                ms, cnt = eng.prof_read(st)
                res[s][st].append(ms)
            cnt = ctypes.c_uint64()
            _lib.check(L.rsk_bloom_bitcount(b, ctypes.byref(cnt)))
            bits.setdefault(s, set()).add(cnt.value)
            _lib.check(L.rsk_bloom_destroy(b))
    out = {"n": n, "size": size.value, "k": k.value, "routes": {}}
    pops = set().union(*bits.values())
    for s in specs:
        med = {st: statistics.median(v) for st, v in res[s].items()}
        out["routes"][s] = {"median_ms": med, "bitcount": sorted(bits[s])}
        print("%-28s " % s + " ".join("%s=%.2f" % (st.replace("bloom_", ""), med[st]) for st in STAGES),
              sorted(bits[s]), flush=True)
    out["identical_bitcount"] = len(pops) == 1
    print("identical bitcount:", len(pops) == 1)
    json.dump(out, open(out_path, "w"), indent=1)
    ins.free()


if __name__ == "__main__":
    main()
