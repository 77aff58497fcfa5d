import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import dllm  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native HIP library")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


# below Linux's ephemeral range (32768-60999): a port checked free there can be taken by an outgoing connection (a
# gloo / RCCL socket of an earlier test) before the rendezvous binds it (EADDRINUSE seen on the GPU box, round 5)
_PORT = [10000 + (os.getpid() % 200) * 100]


def _bindable(port: int) -> bool:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        try:
            s.bind(("127.0.0.1", port))
            return True
        except OSError:
            return False


@pytest.fixture
def free_port():
    """A rendezvous port whose next 9 ports are free too (tests use free_port + k for follow-up runs); every
    test gets its own block of 10, so no test reuses a port another one left in TIME_WAIT."""
    while True:
        _PORT[0] += 10
        if all(_bindable(_PORT[0] + k) for k in range(10)):
            return _PORT[0]

