#!/bin/bash
# round 6: cherry tables with the row loads issued before the P^T staging -- parity, then the
# cfg4 / cfg3 kernel statistics
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD; O=gpurun_out/${TAG:-r6ctab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "cherry_tables or yn98 or lg08" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in yn98_codon_50k_128 lg08_g4_protein_200k_256; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/t_$c -o k -- \
    python3 $R/bench.py --no-cpu-baseline --no-strong --config $c > $R/$O/line_$c.json 2> $R/$O/err_$c.log ) || exit 1
  f=$(find $O/t_$c -name "*kernel_stats.csv" | head -1); cp $f $O/${c}_kernel_stats.csv; rm -rf $O/t_$c
  grep -E "cherry_table|treeM|pmat" $O/${c}_kernel_stats.csv | cut -d, -f1-4
done
