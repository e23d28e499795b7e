import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("bpp-phyl_amd", "oracle"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU; runs on the GPU box")
    config.addinivalue_line("markers", "slow: larger sizes")


@pytest.fixture(scope="session")
def root_dir():
    return ROOT


def set_tune(monkeypatch, key, value):
    """Set one of libplk's tuning knobs: they all live in PLK_TUNE="KEY=value,..."
    (csrc/plk.hip tune_get)."""
    cur = [kv for kv in os.environ.get("PLK_TUNE", "").split(",") if "=" in kv and kv.split("=", 1)[0] != key]
    cur.append(f"{key}={value}")
    monkeypatch.setenv("PLK_TUNE", ",".join(cur))


def clear_tune(monkeypatch, key):
    cur = [kv for kv in os.environ.get("PLK_TUNE", "").split(",") if "=" in kv and kv.split("=", 1)[0] != key]
    monkeypatch.setenv("PLK_TUNE", ",".join(cur))
