"""CPU tests of the C-ABI boundary: libplk.so builds for gfx950, loads without a GPU,
and exports every entry point include/plk.h declares.  No compute calls."""
import os
import re
import subprocess

import pytest

import plk
from conftest import run_make

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "plk.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(plk_[a-z_0-9]+)\s*\(", hdr)))


def _ensure_built():
    if not os.path.exists(plk.LIB_PATH):
        run_make("-s", "-C", os.path.join(ROOT, "bpp-phyl_amd"))


def test_header_symbols_listed_in_binding():
    assert sorted(plk.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    _ensure_built()
    out = subprocess.run(["nm", "-D", "--defined-only", plk.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (plk_[a-z_0-9]+)$", out, flags=re.M))
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version():
    _ensure_built()
    lib = plk.load()
    assert lib.plk_abi_version() == 2
    assert lib.plk_block_size() == 4096


def test_library_built_from_these_sources():
    """The loaded libplk.so carries the hash of the sources beside it (Makefile recipe), so
    a stale binary cannot pass for HEAD's code -- here and, through the gpu twin in
    tests/test_gpu_configs.py, on the GPU box that receives the prebuilt library."""
    _ensure_built()
    assert plk.build_id() == plk.source_hash()


def test_code_object_is_gfx950():
    _ensure_built()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", plk.LIB_PATH], capture_output=True,
                         text=True)
    # the fat binary embeds an amdgcn code object; check via the bundle entry name
    blob = open(plk.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_no_cpu_fallback_without_gpu():
    """plk_create must fail loudly (PLK_ERR_DEVICE) when no gfx950 device is usable."""
    _ensure_built()
    if plk.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(plk.PlkError) as ei:
        plk.Engine(0, 4, 4, 100, 4, 2)
    assert ei.value.code == -2
