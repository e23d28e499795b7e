"""bench.py's launch handling (CPU, no GPU call): --gpus N is honoured under any launcher or
refused -- WORLD_SIZE must equal --gpus under torch.distributed.run; without a launcher N > 1
is one process over N devices (plk_create_multi), or --devices; never a silent 1-GPU line."""
import argparse
import importlib.util
import os
import subprocess
import sys

import pytest

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(_REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def _args(gpus=1, devices=None):
    return argparse.Namespace(gpus=gpus, devices=devices)


@pytest.fixture
def bench(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    return _bench()


def test_single_default(bench):
    assert bench.launch_layout(_args()) == {"kind": "single", "world": 1, "devices": None}


def test_world_size_must_match_gpus(bench, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit) as e:
        bench.launch_layout(_args(gpus=8))
    assert e.value.code == 2
    assert bench.launch_layout(_args(gpus=4)) == {"kind": "ranks", "world": 4, "devices": None}
    with pytest.raises(SystemExit):
        bench.launch_layout(_args(gpus=4, devices="0,1,2,3"))


def test_more_gpus_than_visible_is_refused(bench, monkeypatch):
    monkeypatch.setattr(bench.plk, "device_count", lambda: 1)
    with pytest.raises(SystemExit) as e:
        bench.launch_layout(_args(gpus=2))
    assert e.value.code == 2
    monkeypatch.setattr(bench.plk, "device_count", lambda: 8)
    assert bench.launch_layout(_args(gpus=8)) == {"kind": "multi", "world": 1, "devices": list(range(8))}


def test_explicit_devices(bench):
    assert bench.launch_layout(_args(gpus=2, devices="0,0")) == {"kind": "multi", "world": 1, "devices": [0, 0]}
    with pytest.raises(SystemExit):
        bench.launch_layout(_args(gpus=2, devices="0"))
    lay = bench.launch_layout(_args(gpus=2, devices="0,0"))
    assert bench.parallelism(lay, _args(gpus=2)) == "multi-device x2"


def test_single_gpu_explicit_device(bench):
    """--gpus 1 --devices K: one process on device K, not device 0."""
    lay = bench.launch_layout(_args(gpus=1, devices="3"))
    assert lay == {"kind": "single", "world": 1, "devices": [3]}
    assert bench.single_device(lay) == 3
    assert bench.single_device(bench.launch_layout(_args())) == 0
    with pytest.raises(SystemExit):
        bench.launch_layout(_args(gpus=1, devices="0,1"))


def test_cli_exits_nonzero_without_gpus(tmp_path):
    """`python bench.py --gpus 2` with no launcher on a box with fewer GPUs: exit status 2 and a
    message, before any GPU work (this container has none)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(_REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr
    assert r.stdout == ""
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(_REPO, "bench.py"), "--gpus", "8", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 8" in r.stderr, r.stderr[-2000:]
