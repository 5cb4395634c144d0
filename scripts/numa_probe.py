"""Device<->host DMA rate by NUMA placement of the host memory (GPU box only).

Round-6 measurement aid for the checkpoint export's bimodal device->host rate
(DESIGN.md §4 round 6). For every NUMA node the process may run on, the main
thread is pinned to that node's CPUs, host memory is allocated and first-touched
there (hipHostMalloc stages, and a numpy buffer registered with hipHostRegister),
the node of its pages is read back with move_pages(2), and 1 GiB hipMemcpy
D2H/H2D are timed. Plain ctypes on libamdhip64 (no torch import).

Usage: python scripts/numa_probe.py [out.json]
       PROBE_STREAMS=1 [PROBE_TORCH=1] python scripts/numa_probe.py [out.json]  (per-stream rates)
"""
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

GIB = 1 << 30
hip = ctypes.CDLL("libamdhip64.so")
libc = ctypes.CDLL(None, use_errno=True)
SYS_move_pages = 279  # x86_64


def ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def cpulist(s):
    out = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def nodes_of(ptr, nbytes, samples=64):
    """NUMA node of `samples` pages spread over [ptr, ptr+nbytes) (move_pages query)."""
    page = 4096
    step = max(page, (nbytes // samples) // page * page)
    addrs = [ptr + i * step for i in range(samples) if i * step < nbytes]
    arr = (ctypes.c_void_p * len(addrs))(*addrs)
    st = (ctypes.c_int * len(addrs))()
    rc = libc.syscall(ctypes.c_long(SYS_move_pages), ctypes.c_int(0),
                      ctypes.c_ulong(len(addrs)), arr, None, st, ctypes.c_int(0))
    if rc != 0:
        return {"error": ctypes.get_errno()}
    hist = {}
    for v in st:
        hist[int(v)] = hist.get(int(v), 0) + 1
    return hist


def timed_copy(dst, src, nbytes, kind, reps=3):
    out = []
    for _ in range(reps):
        ck(hip.hipDeviceSynchronize(), "sync")
        t = time.perf_counter()
        ck(hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes),
                         ctypes.c_int(kind)), "hipMemcpy")
        out.append(nbytes / (time.perf_counter() - t) / 1e9)
    return [round(x, 1) for x in out]


def stream_probe(nstreams=12, nbytes=256 << 20, reps=3):
    """D2H / H2D rate of hipMemcpyAsync on each of `nstreams` freshly created streams."""
    dev = ctypes.c_void_p()
    ck(hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(nbytes)), "hipMalloc")
    h = ctypes.c_void_p()
    ck(hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(nbytes), ctypes.c_uint(0)), "hostmalloc")
    out = []
    for i in range(nstreams):
        s = ctypes.c_void_p()
        ck(hip.hipStreamCreate(ctypes.byref(s)), "stream")
        r = {"stream": i}
        for kind, dst, src, key in ((2, h, dev, "d2h"), (1, dev, h, "h2d")):
            v = []
            for _ in range(reps):
                ck(hip.hipDeviceSynchronize(), "sync")
                t = time.perf_counter()
                ck(hip.hipMemcpyAsync(dst, src, ctypes.c_size_t(nbytes), ctypes.c_int(kind), s), "cpy")
                ck(hip.hipStreamSynchronize(s), "ssync")
                v.append(round(nbytes / (time.perf_counter() - t) / 1e9, 1))
            r[key] = v
        out.append(r)
        print(json.dumps(r), flush=True)
    return out


def main():
    res = {}
    if os.environ.get("PROBE_STREAMS"):
        if os.environ.get("PROBE_TORCH"):
            import torch
            torch.zeros(1, device="cuda")
        res = {"env": {k: os.environ[k] for k in os.environ if k.startswith(("HSA_", "HIP_", "GPU_", "PROBE_"))},
               "streams": stream_probe()}
        line = json.dumps(res)
        print(line)
        if len(sys.argv) > 1:
            with open(sys.argv[1], "a") as f:
                f.write(line + "\n")
        return
    bus = ctypes.create_string_buffer(64)
    ck(hip.hipDeviceGetPCIBusId(bus, 64, 0), "busid")
    busid = bus.value.decode().lower()
    res["gpu_pci"] = busid
    try:
        res["gpu_numa_node"] = int(open(f"/sys/bus/pci/devices/{busid}/numa_node").read())
    except OSError as e:
        res["gpu_numa_node"] = f"unreadable: {e}"
    st = open("/proc/self/status").read().splitlines()
    res["status"] = {l.split(":")[0]: l.split(":", 1)[1].strip() for l in st
                     if l.startswith(("Cpus_allowed_list", "Mems_allowed_list"))}
    allowed = os.sched_getaffinity(0)
    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        n = int(d.rsplit("node", 1)[1])
        cpus = cpulist(open(d + "/cpulist").read()) & allowed
        if cpus:
            nodes[n] = sorted(cpus)
    res["nodes_with_allowed_cpus"] = {n: [c[0], c[-1], len(c)] for n, c in nodes.items()}

    dev = ctypes.c_void_p()
    ck(hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(GIB)), "hipMalloc")
    ck(hip.hipMemset(dev, 1, ctypes.c_size_t(GIB)), "memset")
    runs = []
    for n, cpus in list(nodes.items()) + [("unpinned", sorted(allowed))]:
        os.sched_setaffinity(0, cpus)
        r = {"node": n}
        h = ctypes.c_void_p()
        ck(hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(GIB), ctypes.c_uint(0)), "hostmalloc")
        r["hostmalloc_pages"] = nodes_of(h.value, GIB)
        r["hostmalloc_d2h_GBps"] = timed_copy(h.value, dev.value, GIB, 2)
        r["hostmalloc_h2d_GBps"] = timed_copy(dev.value, h.value, GIB, 1)
        ck(hip.hipHostFree(h), "hostfree")
        buf = np.empty(GIB, np.uint8)
        buf.fill(3)
        p = buf.ctypes.data
        r["numpy_pages"] = nodes_of(p, GIB)
        r["pageable_d2h_GBps"] = timed_copy(p, dev.value, GIB, 2, reps=2)
        ck(hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(GIB), ctypes.c_uint(0)), "register")
        r["registered_d2h_GBps"] = timed_copy(p, dev.value, GIB, 2)
        r["registered_h2d_GBps"] = timed_copy(dev.value, p, GIB, 1)
        ck(hip.hipHostUnregister(ctypes.c_void_p(p)), "unregister")
        del buf
        runs.append(r)
        print(json.dumps(r), flush=True)
    res["runs"] = runs
    hip.hipFree(dev)
    line = json.dumps(res)
    print(line)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
