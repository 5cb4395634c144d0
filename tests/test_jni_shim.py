"""The Java binding (jni/): the JNI-independent shim that jni/rsketch_jni.c
calls, and the C caller that drives it like the JVM would.

CPU: the shim's argument checks and status -> exception mapping (no device
access), and that the JNI glue / Java natives / shim declarations agree.
GPU: tests/c/shim_caller.c replays the reference's JUnit cases and a 200k
batch through the shim (built by `make -C jni`, run as a subprocess)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "jni")


class Buf(ctypes.Structure):
    _fields_ = [("addr", ctypes.c_void_p), ("cap", ctypes.c_int64)]


class Keys(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("n", ctypes.c_uint64),
                ("fixed_len", ctypes.c_uint32), ("location", ctypes.c_uint32)]


@pytest.fixture(scope="module")
def shim():
    path = os.path.join(JNI, "bin", "librsketch_shim.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", JNI], check=True)
    lib = ctypes.CDLL(path)
    lib.rsk_shim_exception_class.restype = ctypes.c_char_p
    lib.rsk_shim_last_error.restype = ctypes.c_char_p
    lib.rsk_shim_keys.argtypes = [Buf, Buf, ctypes.c_int64, ctypes.POINTER(Keys)]
    return lib


def test_exception_classes(shim):
    cls = {rc: shim.rsk_shim_exception_class(rc) for rc in range(8)}
    assert cls[0] is None
    assert cls[1] == b"java/lang/IllegalArgumentException"  # RedissonBloomFilter.java:175,227
    assert cls[2] == b"java/lang/IllegalStateException"     # "Bloom filter is not initialized!" :217
    assert cls[3] == cls[4] == b"org/redisson/client/RedisException"  # -WRONGTYPE / -INVALIDOBJ
    assert cls[6] == b"java/lang/OutOfMemoryError"
    assert shim.rsk_shim_exception_class(100) == b"org/redisson/client/RedisException"  # config changed
    assert shim.rsk_shim_exception_class(101) == b"org/redisson/client/RedisException"  # -ERR bit offset ...


def test_key_buffer_checks(shim):
    data = (ctypes.c_uint8 * 16)()
    offs = (ctypes.c_int64 * 4)(0, 5, 9, 16)
    k = Keys()
    ok = shim.rsk_shim_keys(Buf(ctypes.addressof(data), 16), Buf(ctypes.addressof(offs), 4), 3, ctypes.byref(k))
    assert ok == 0 and k.n == 3 and k.offsets == ctypes.addressof(offs) and k.location == 0
    bad = [
        (Buf(ctypes.addressof(data), 15), Buf(ctypes.addressof(offs), 4), 3, b"past the keys buffer"),
        (Buf(ctypes.addressof(data), 16), Buf(ctypes.addressof(offs), 3), 3, b"fewer than n+1"),
        (Buf(ctypes.addressof(data), 16), Buf(None, 0), 3, b"direct LongBuffer"),
        (Buf(None, 0), Buf(ctypes.addressof(offs), 4), 3, b"direct ByteBuffer"),
        (Buf(ctypes.addressof(data), 16), Buf(ctypes.addressof(offs), 4), -1, b"negative"),
    ]
    for kb, ob, n, msg in bad:
        assert shim.rsk_shim_keys(kb, ob, n, ctypes.byref(k)) == 1
    dec = (ctypes.c_int64 * 3)(0, 9, 5)
    assert shim.rsk_shim_keys(Buf(ctypes.addressof(data), 16), Buf(ctypes.addressof(dec), 3), 2, ctypes.byref(k)) == 1
    assert shim.rsk_shim_keys(Buf(None, 0), Buf(None, 0), 0, ctypes.byref(k)) == 0  # empty batch


def _java_natives():
    src = open(os.path.join(JNI, "java", "org", "redisson", "gpu", "RSketchNative.java")).read()
    return {m.group(1): len([a for a in m.group(2).split(",") if a.strip()])
            for m in re.finditer(r"static native \S+ (\w+)\(([^)]*)\)", src)}


def test_jni_glue_covers_every_native_method():
    glue = open(os.path.join(JNI, "rsketch_jni.c")).read()
    fns = {m.group(1): len([a for a in m.group(2).split(",") if a.strip()]) - 2  # minus JNIEnv*, jclass
           for m in re.finditer(r"JNI_FN\(\w+, (\w+)\)\(([^)]*)\)", glue)}
    natives = _java_natives()
    assert natives and set(natives) == set(fns)
    for name, nargs in natives.items():
        assert fns[name] == nargs, name
    hdr = open(os.path.join(JNI, "rsketch_shim.h")).read()
    impl = open(os.path.join(JNI, "rsketch_shim.c")).read()
    for fn in re.findall(r"\b(rsk_shim_\w+)\(", hdr):
        assert re.search(r"\b%s\([^;]*\{" % fn, impl, re.S), fn


def test_java_sources_use_completions_not_raw_promises():
    """Async natives take a Completion (promise + the event loop its listeners
    run on); RSketchNative.complete only hands off to that executor."""
    src = open(os.path.join(JNI, "java", "org", "redisson", "gpu", "RSketchNative.java")).read()
    for m in re.finditer(r"static native void (\w+Async)\(([^)]*)\)", src):
        assert "Completion<" in m.group(2), m.group(1)
    body = src[src.index("static void complete("):]
    body = body[: body.index("\n    }\n")]
    assert "executor.execute" in body and "trySuccess" not in body
    glue = open(os.path.join(JNI, "rsketch_jni.c")).read()
    done = glue[glue.index("static void jni_done("):]
    done = done[: done.index("\n}\n")]
    assert "FindClass" not in done  # resolved once in JNI_OnLoad
    assert "g_complete" in glue and "JNI_OnLoad" in glue


@pytest.mark.gpu
def test_jni_glue_on_gpu():
    """jni/rsketch_jni.c compiled against tests/c/jni_mock/jni.h and driven by a
    fake JVM (tests/c/jni_caller.c): completions, parking, re-entrancy."""
    exe = os.path.join(JNI, "bin", "jni_caller")
    assert os.path.exists(exe), "build it first: make -C jni"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "jni_caller ok" in r.stdout


@pytest.mark.gpu
def test_shim_caller_on_gpu():
    exe = os.path.join(JNI, "bin", "shim_caller")
    assert os.path.exists(exe), "build it first: make -C jni"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "shim_caller ok" in r.stdout
