#!/bin/bash
# round 6: the shader clock during the driver's exact bench window (--steps 20 --warmup 5),
# from per-workgroup clock stamps (PLK_DEBUG_CLOCK build of the same traversal program)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6clk
mkdir -p $O
export TMPDIR=/tmp
(rocm-smi --showclocks > $O/smi_clocks_before.txt 2>&1 || true)
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --clock-json $O/clk_20_5_a.json > $O/line_clk_20_5_a.json 2> $O/err_a.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/line_plain_20_5_b.json 2> $O/err_b.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --clock-json $O/clk_20_5_c.json --no-cpu-baseline > $O/line_clk_20_5_c.json 2> $O/err_c.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 50 --clock-json $O/clk_200_50_d.json --no-cpu-baseline > $O/line_clk_200_50_d.json 2> $O/err_d.log
rc=$?
(rocm-smi --showclocks > $O/smi_clocks_after.txt 2>&1 || true)
for f in $O/line_*.json; do echo "== $f"; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['traversal_ms'])"; done
exit $rc
