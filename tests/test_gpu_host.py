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
