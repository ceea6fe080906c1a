import glob
import os
import uuid

import pytest


# Tests save back to back and assert every save lands: block on a busy
# staging buffer instead of the production default (skip the save, reference
# semantics); test_flash_ckpt_gpu::test_gpu_busy_save_is_skipped covers "skip".
os.environ.setdefault("DWAMD_CKPT_BUSY", "wait")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _isolated_shm(monkeypatch):
    """Every test gets its own shm namespace and cleans it up."""
    prefix = "pt" + uuid.uuid4().hex[:8]
    monkeypatch.setenv("DWAMD_SHM_PREFIX", prefix)
    yield prefix
    for f in glob.glob(f"/dev/shm/dwamd_{prefix}*"):
        try:
            os.remove(f)
        except OSError:
            pass


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
