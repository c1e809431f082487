import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    config.addinivalue_line("markers", "reference: needs /root/reference (container only)")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    has_ref = os.path.isdir(os.environ.get("WAB_REFERENCE", "/root/reference"))
    gpu = None
    for item in items:
        if "reference" in item.keywords and not has_ref:
            item.add_marker(pytest.mark.skip(reason="reference not mounted"))
        if "gpu" in item.keywords:
            if gpu is None:
                gpu = _has_gpu()
            if not gpu:
                item.add_marker(pytest.mark.skip(reason="no HIP device in this container"))
