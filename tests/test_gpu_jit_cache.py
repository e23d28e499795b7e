"""The on-disk cache of the hiprtc-compiled tree kernels (PLK_JIT_CACHE).

A second process evaluating the same tree loads the cached code object instead of
compiling (PLK_JIT_LOG reports which), gets the same lnL bitwise, and an entry whose stored
source differs from the generated one is never used (it is recompiled and replaced).
"""
import glob
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path.insert(0, %r)
import workload
wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=4096)
ev = workload.Evaluator(wl, 0, 0, 4096, extra_flags=__import__("plk").PLK_FLAG_LNL_ONLY)
lnl, _, _ = ev.step()
print(json.dumps({"lnl": lnl, "path": ev.eng.kernel_path()}))
""" % os.path.join(ROOT, "bpp-phyl_amd")


def _run(cache_dir):
    env = dict(os.environ, PLK_JIT_CACHE=str(cache_dir), PLK_JIT_LOG="1")
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_disk_cache_hit_and_stale_entry(tmp_path):
    out1, err1 = _run(tmp_path)
    assert out1["path"] == "jit_tree4"
    assert "jit compiled" in err1 and "cache hit" not in err1
    cos = glob.glob(str(tmp_path / "*.co"))
    assert len(cos) == 1 and os.path.exists(cos[0][:-3] + ".hip")
    out2, err2 = _run(tmp_path)
    assert "cache hit" in err2 and "jit compiled" not in err2
    assert out2["lnl"] == out1["lnl"]
    # a stored source that differs from the generated one: the entry is not used
    src = cos[0][:-3] + ".hip"
    with open(src, "a") as f:
        f.write("\n// edited\n")
    out3, err3 = _run(tmp_path)
    assert "jit compiled" in err3 and "cache hit" not in err3
    assert out3["lnl"] == out1["lnl"]


def test_damaged_cache_entry_is_recompiled(tmp_path):
    """A truncated code object whose stored source still matches (e.g. a full disk while the
    .co was written): its size / hash no longer match the entry's .sum, so it is never
    loaded (the HIP runtime's ELF reader aborts on it); the kernel is recompiled and the
    entry overwritten, with the same lnL."""
    out1, _ = _run(tmp_path)
    co = glob.glob(str(tmp_path / "*.co"))[0]
    size = os.path.getsize(co)
    with open(co, "r+b") as f:
        f.truncate(size // 3)
    out2, err2 = _run(tmp_path)
    assert "jit compiled" in err2 and "cache hit" not in err2, err2[-1500:]
    assert out2["lnl"] == out1["lnl"]
    assert os.path.getsize(co) == size
    out3, err3 = _run(tmp_path)
    assert "cache hit" in err3 and "jit compiled" not in err3
    assert out3["lnl"] == out1["lnl"]
