"""The >2 GB point-to-point probe (VERDICT r05 Weak 7): self send/recv of a
known pattern through a 1-rank RCCL communicator at sizes around 2^31 and
2^32 bytes, as one ncclUint8 transfer, as one ncclUint64 transfer (8x fewer
elements) and in the library's 1 GiB pieces (rsk_diag_p2p_probe).  One JSON
line per case to stdout.

    python scripts/p2p_probe.py [BYTES ...] > gpurun_out/p2p_probe.jsonl
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib  # noqa: E402


def main():
    L = _lib.load()
    D = _lib.diag()
    from redisson_amd import Engine

    eng = Engine.get(0)
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(eng.ctx, 1, 0, uid))
    sizes = [int(a) for a in sys.argv[1:]] or [1 << 30, (1 << 31) - 8, (1 << 31) + 8, 3 << 30, 4_000_000_000,
                                              (1 << 32) + 8]
    for b in sizes:
        for mode in (2, 1, 0):
            bad, first = ctypes.c_uint64(), ctypes.c_uint64()
            t0 = time.perf_counter()
            rc = D.rsk_diag_p2p_probe(eng.ctx, b, mode, ctypes.byref(bad), ctypes.byref(first))
            dt = time.perf_counter() - t0
            rec = {"bytes": b, "mode": ["one uint8 transfer", "one uint64 transfer", "1 GiB uint8 pieces"][mode],
                   "elements": b if mode != 1 else b // 8, "rc": rc, "s": round(dt, 3)}
            if rc == 0:
                rec.update(bad_words=bad.value, first_bad_byte=(first.value * 4 if bad.value else None),
                           correct=bad.value == 0)
            else:
                rec["error"] = D.rsk_diag_last_error().decode(errors="replace")
            print(json.dumps(rec), flush=True)
    _lib.check(L.rsk_comm_destroy(eng.ctx))


if __name__ == "__main__":
    main()
