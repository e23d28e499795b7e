#!/bin/bash
# whole -m gpu suite (repository JIT cache), smoke(), default line
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -1; [ $rc -eq 0 ] || { tail -40 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));s=d.get('strong',{});print('default', round(d['ms_per_step'],5), round(d['roofline']['frac'],3), 'strong', s.get('ms_per_step'))"
