#!/bin/bash
# pmat64m_kernel: parity tests, then cfg4 under the kernel trace for each (P64R, P64NB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5p64ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "pmat64 or treeM_cherry or pmatrix_kernel or random_topologies or codon or s64" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export TMPDIR=/tmp
cd /tmp
for v in "P64RX=0" "P64RX=4,P64NB=4" "P64RX=2,P64NB=4" "P64RX=4,P64NB=2" "P64RX=2,P64NB=2" "P64RX=1,P64NB=4" "P64RX=0" "P64RX=4,P64NB=4"; do
  tag=$(echo $v | tr ',=' '__')
  PLK_TUNE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
    python3 $R/bench.py --config yn98_codon_50k_128 --no-cpu-baseline --no-strong --steps 20 --warmup 3 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  s=$(find $O/$tag -name "run_kernel_stats.csv" | head -1)
  echo "$v $(python3 -c "import json;d=json.load(open('$O/$tag.json'));print(d['ms_per_step'])") $(grep -h pmat64 $s | cut -d, -f1-4)"
done
