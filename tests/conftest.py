import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The tree-specialised kernels are compiled by hiprtc at their first use (a 256-taxon protein
# tree: ~45 s).  The tests share one disk cache inside the repository (`.jit_cache`,
# git-ignored; filled by a GPU run of the suite and travelling with the tree): an entry is
# used only when its stored source equals the generated one and its code object's hash
# checks out, otherwise it is recompiled (csrc/plk.hip jit_compile).  An explicit
# PLK_JIT_CACHE (a directory, or 0 for none) wins.
os.environ.setdefault("PLK_JIT_CACHE", os.path.join(ROOT, ".jit_cache"))
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


def run_make(*args):
    """`make *args` under an exclusive lock: pytest-xdist workers share the build trees, and a
    worker's make once rewrote a binary another worker was executing (ETXTBSY).  After the
    first build the others find nothing to do."""
    import fcntl
    import subprocess
    import tempfile
    with open(os.path.join(tempfile.gettempdir(), "plk_tests_make.lock"), "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        subprocess.run(["make", *args], check=True)


def set_tune(monkeypatch, key, value):
    """Set one of libplk's tuning knobs: they all live in PLK_TUNE="KEY=value,..."
    (csrc/plk.hip tune_get)."""
    cur = [kv for kv in os.environ.get("PLK_TUNE", "").split(",") if "=" in kv and kv.split("=", 1)[0] != key]
    cur.append(f"{key}={value}")
    monkeypatch.setenv("PLK_TUNE", ",".join(cur))


def clear_tune(monkeypatch, key):
    cur = [kv for kv in os.environ.get("PLK_TUNE", "").split(",") if "=" in kv and kv.split("=", 1)[0] != key]
    monkeypatch.setenv("PLK_TUNE", ",".join(cur))
