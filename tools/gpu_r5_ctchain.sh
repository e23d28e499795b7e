#!/bin/bash
# cherry_table_kernel: row-list entry loaded together with the P^T staging (in-tree build) vs
# the previous order (ab/libplk_ctold.so): parity tests, then cfg4 / cfg3 under the kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ctchain
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "cherry or jit_treeM or random_topologies or subtree_patterns_any or pmat64" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export TMPDIR=/tmp
cd /tmp
for cfg in yn98_codon_50k_128 lg08_g4_protein_200k_256; do
  st=200; [ $cfg = lg08_g4_protein_200k_256 ] && st=40
  for lib in ab/libplk_ctold.so bpp-phyl_amd/libplk.so ab/libplk_ctold.so bpp-phyl_amd/libplk.so; do
    tag=$(basename $lib .so)_${cfg:0:4}_$RANDOM
    PLK_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 $R/bench.py --config $cfg --no-cpu-baseline --no-strong --steps $st --warmup 20 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
    s=$(find $O/$tag -name "run_kernel_stats.csv" | head -1)
    python3 - $s "$lib $cfg" $O/$tag.json <<'PY'
import csv,sys,json
d=json.load(open(sys.argv[3]))
for r in csv.DictReader(open(sys.argv[1])):
    if 'cherry_table' in r['Name']:
        print(sys.argv[2], r['Name'][:32], r['Calls'], round(float(r['AverageNs'])/1000,2), round(float(r['MinNs'])/1000,2), 'step', round(d['ms_per_step'],4))
PY
    rm -rf $O/$tag
  done
done
