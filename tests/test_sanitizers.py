"""ASan + UBSan builds (race detection / sanitizers) of the host code: the Bio++
mirror's sources with its CPU test program (`make -C bpp-phyl_amd/host asan`) and the oracle
with its driver (`make -C oracle asan`, oracle/sanitize_check.cpp).  Any sanitizer finding --
heap or stack overflow, use after free, leak, undefined behaviour -- aborts the program
(-fno-sanitize-recover=all, LeakSanitizer on); the runs must be clean and give the same
results as the ordinary builds.  Host code only: GPU sanitizers are not available."""
import json
import os
import subprocess
from conftest import run_make

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "bpp-phyl_amd", "host")
ORACLE = os.path.join(ROOT, "oracle")
_SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(exe, tmp_path):
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=_SAN_ENV)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_oracle_asan_ubsan_clean(tmp_path):
    run_make("-s", "-C", ORACLE, "asan")
    out = _run(os.path.join(ORACLE, "_san", "oracle_check"), tmp_path)
    assert out.strip().endswith("PASSED"), out


def test_host_mirror_asan_ubsan_clean(tmp_path):
    run_make("-s", "-C", os.path.join(ROOT, "bpp-phyl_amd"))
    run_make("-s", "-j8", "-C", HOST, "asan", "bin/test_host_cpu")
    san = [json.loads(x) for x in _run(os.path.join(HOST, "san", "test_host_cpu"), tmp_path).splitlines() if x.strip()]
    ref = subprocess.run([os.path.join(HOST, "bin", "test_host_cpu")], check=True, capture_output=True,
                         text=True, timeout=300).stdout
    ref = [json.loads(x) for x in ref.splitlines() if x.strip()]
    assert [r["kind"] for r in san] == [r["kind"] for r in ref]
    # same computations, -O0 vs -O2: the records agree to rounding
    for a, b in zip(san, ref):
        if a["kind"] in ("model", "gamma"):
            for k, v in a.items():
                if isinstance(v, list) and v and isinstance(v[0], float):
                    assert max(abs(x - y) for x, y in zip(v, b[k])) <= 1e-9 * max(1.0, max(abs(y) for y in b[k])), k
