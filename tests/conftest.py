import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_collection_modifyitems(config, items):
    """Every test runs under a time limit even when the runner passes no
    --timeout: a GPU test without its own mark gets 60 s (the slowest
    unmarked one takes ~5 s on an MI355X), a CPU test 120 s."""
    import pytest
    for item in items:
        if item.get_closest_marker("timeout") is None:
            item.add_marker(pytest.mark.timeout(60 if item.get_closest_marker("gpu") else 120))
