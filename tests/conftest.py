import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every gateway built by a test checks its request-lifecycle transitions
# (gateway/request_table.py: a transition from a state it may not come from raises)
os.environ.setdefault("LLMQ_LIFECYCLE_DEBUG", "1")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def hipops():
    import torch  # noqa: F401
    from llm_message_queue_amd import _native
    return _native.require_hipops()


@pytest.fixture(autouse=True)
def _fresh_metrics():
    from llm_message_queue_amd.utils.metrics import reset_default_metrics
    reset_default_metrics()
    yield
