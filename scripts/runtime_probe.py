"""Diagnostic: does librsketch work when torch is imported before/after it?"""
import subprocess
import sys

CASES = {
    "lib_then_torch": "from redisson_amd import _lib; _lib.load(); import torch; import torch.distributed;",
    "torch_then_lib": "import torch; import torch.distributed; from redisson_amd import _lib; _lib.load();",
}
BODY = """
import numpy as np
from redisson_amd import Redisson
c = Redisson.create()
h = c.getHyperLogLog('x'); h.addAll(list(range(1000))); print('count', h.count())
"""
for name, pre in CASES.items():
    r = subprocess.run([sys.executable, "-c", pre + BODY], capture_output=True, text=True, timeout=300)
    print(name, "rc", r.returncode, r.stdout.strip()[-200:], r.stderr.strip()[-400:])
