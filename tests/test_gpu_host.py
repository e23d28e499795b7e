"""GPU test of the C++ Bio++ API mirror: the drop-in test program
(tests/cpp/test_likelihood_gpu.cpp) runs the reference's test_likelihood /
test_likelihood_clock calls on the MI355X and checks their goldens."""
import os
import subprocess

import pytest

import plk

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "bpp-phyl_amd", "host")


def test_cpp_drop_in_goldens():
    assert plk.device_count() > 0, "no GPU visible"
    subprocess.run(["make", "-s", "-j8", "-C", HOST], check=True)
    r = subprocess.run([os.path.join(HOST, "bin", "test_likelihood_gpu")], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout


def test_cpp_drop_in_nh():
    """tests/cpp/test_likelihood_nh_gpu.cpp: the reference's test_likelihood_nh.cpp calls
    (simulated alignments, per-branch theta recovered within 0.2 for both root
    parametrisations), per-theta evaluations recomputing one eigen-system, and the
    BrLenRoot / RootPosition derivatives against central differences."""
    assert plk.device_count() > 0, "no GPU visible"
    subprocess.run(["make", "-s", "-j8", "-C", HOST], check=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    r = subprocess.run([os.path.join(HOST, "bin", "test_likelihood_nh_gpu")], capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout
