"""ASan/UBSan run of the CPU-side C code.

`make -C oracle asan` builds the oracle (oracle/rsk_oracle.c) and the host
exchange-plan code of librsketch (redisson_amd/csrc/rsk_plan.hip, plain C++)
with -fsanitize=address,undefined -fno-sanitize-recover=all.  The oracle pins
and the plan tests then run in a child interpreter with the ASan runtime
preloaded; any memory error or undefined behaviour aborts it.  (GPU code
cannot be sanitized on this pool; the HIP host code is covered on the GPU
box by the same tests without instrumentation.)"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_and_plans_under_asan_ubsan():
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("gcc ASan runtime not available")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ)
    env.update({
        "LD_PRELOAD": asan,
        "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
        "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
        "RSK_SANITIZE": "1",
        "RSK_ORACLE_LIB": os.path.join(ROOT, "oracle", "_asan", "librsk_oracle.so"),
        "RSK_PLAN_LIB": os.path.join(ROOT, "oracle", "_asan", "librsk_plan.so"),
        "OMP_NUM_THREADS": "4",
    })
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_oracle_pins.py", "tests/test_plan.py", "tests/test_codec.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
