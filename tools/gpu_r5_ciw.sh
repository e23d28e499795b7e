#!/bin/bash
# cfg5 tiers with every class in the wave (default) vs one class per wave (PLK_TUNE JIT_CIW=0):
# per-tier launch durations from the kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ciw
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "JIT_CIW=1" "JIT_CIW=0" "JIT_CIW=0,JIT_DM=6" "JIT_CIW=0,JIT_G=2" ; do
  tag=$(echo $v | tr ',=' '__')
  PLK_TUNE=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
    python3 $R/bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong --steps 50 --warmup 10 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  t=$(find $O/$tag -name "*kernel_trace.csv" | head -1)
  python3 - $t "$v" $O/$tag.json <<'PY'
import csv,sys,json
d=json.load(open(sys.argv[3]))
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'jit_tree4' in r['Kernel_Name']]
dur=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000 for r in rows]
a=dur[-100::2]; b=dur[-99::2]
import statistics as st
print(sys.argv[2], 'step', round(d['ms_per_step'],4), 'launches', len(dur), 'tierA med', round(st.median(a),1), 'tierB med', round(st.median(b),1), 'grid', rows[-1].get('Grid_Size', rows[-1].get('Grid_Size_X','?')), rows[-2].get('Grid_Size', '?'), 'wg', rows[-1].get('Workgroup_Size','?'), 'vgpr', rows[-1].get('VGPR_Count', rows[-1].get('Arch_VGPR_Count','?')), 'lds', rows[-1].get('LDS_Block_Size', rows[-1].get('Lds_Size','?')))
PY
  rm -rf $O/$tag
done
