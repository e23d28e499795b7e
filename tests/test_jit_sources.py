"""The tree-specialised kernels are generated as HIP source at run time and compiled with
hiprtc on the device (plk_jit.hpp, plk_jitm.hpp).  These CPU tests emit the source of
both generators for a small two-fragment program (tests/jit/jit_emit.cpp: stored and
unstored cherries, a tip, a loaded fragment root, the root reduction) in the shapes the
library uses -- one class per wave and every class in the wave, with and without
rescaling; jit_treeM for 20 and 4 states -- and cross-compile each for gfx950 with hipcc,
so that a generator change that breaks the emitted code fails here, not on the GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)

pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")


@pytest.fixture(scope="module")
def emitter(tmp_path_factory):
    d = tmp_path_factory.mktemp("jit_emit")
    exe = str(d / "jit_emit")
    subprocess.run([HIPCC, "-std=c++17", "-O1", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "bpp-phyl_amd", "csrc"),
                    "-I" + os.path.join(ROOT, "include"), "-o", exe, os.path.join(ROOT, "tests", "jit", "jit_emit.cpp")],
                   check=True, capture_output=True, timeout=600)
    return exe, d


@pytest.mark.parametrize("args", [
    ("tree4", "4", "0"), ("tree4", "4", "1", "0", "1"), ("tree4", "1", "1"), ("tree4q", "4", "0"), ("tree4q", "2", "0"),
    ("treeM", "4", "1", "20"), ("treeM", "1", "0", "20"), ("treeM", "4", "0", "4"),
    ("treeM_deep", "4", "1", "20", "5")])
def test_emitted_kernel_compiles_for_gfx950(emitter, args):
    _compile_emitted(emitter, args, None)


# direct codes (two 16-byte words per pattern): one class per workgroup, every class in the wave
@pytest.mark.parametrize("args", [("tree4q", "4", "0"), ("tree4", "4", "1", "0", "1")])
def test_emitted_direct_codes_kernel_compiles_for_gfx950(emitter, args):
    _compile_emitted(emitter, args, "2")


def _compile_emitted(emitter, args, dc):
    exe, d = emitter
    env = dict(os.environ, **({"JIT_EMIT_DC": dc} if dc else {}))
    src = subprocess.run([exe, *args], check=True, capture_output=True, timeout=60, env=env).stdout.decode()
    if dc:
        assert "#define DC_ 1\n#define DCW_ 2" in src
    name = "plk_jit_treeM" if args[0].startswith("treeM") else "plk_jit_tree4c" if args[0] == "tree4q" else "plk_jit_tree4"
    if args[0] == "tree4q":
        assert "kQuadD[] = {{0, 0, 0, 0, 0, 0, 0, 0},{0,1,2,3,8,9,10," in src   # the quad unit's record
    assert f"void {name}(" in src
    path = d / ("k_" + "_".join(args) + ("_dc" if dc else "") + ".hip")
    # hiprtc includes the HIP device runtime implicitly; hipcc needs the header
    path.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-c", "-o",
                        str(path) + ".o", str(path)], capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-4000:]
