import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Load librsketch (system ROCm HIP/HSA) before any test module imports torch,
# so the process never maps a second, torch-bundled HSA runtime first.
# (Not under the sanitizer run, tests/test_sanitizers.py: it loads only the
# ASan/UBSan builds of the oracle and of the host plan code.)
if os.path.exists(os.path.join(ROOT, "redisson_amd", "librsketch.so")) and not os.environ.get("RSK_SANITIZE"):
    from redisson_amd import _lib as _rsk_lib

    _rsk_lib.load()
    if os.path.exists(_rsk_lib.DIAG_PATH):
        _rsk_lib.diag()  # the support library too, before torch (see bench.py)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU and the built librsketch.so")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def engine():
    from redisson_amd import Engine

    return Engine.get(0)


@pytest.fixture()
def route(engine):
    """Route overrides of the shared engine (rsk_diag_set_route, from the
    support library): route(bloom_stream=1, sa_parts=13) or route("reply=1,sa_tiny=1");
    every route is automatic again after the test."""

    def set_(spec=None, **kw):
        if spec:
            for kv in filter(None, spec.split(",")):
                k, v = kv.split("=")
                kw[k] = int(v)
        for k, v in kw.items():
            engine.set_route(k, v)

    yield set_
    engine.set_route("reset", 0)


@pytest.fixture()
def client():
    from redisson_amd import Redisson

    c = Redisson.create()
    yield c
    c.shutdown()
