#!/bin/bash
# compressed 20/64-state tests + mirror, cfg3 jit_treeM register-depth sweep, SQ counters
set -o pipefail
bash tools/gpu_tests.sh t5 -k "subtree or cpp_drop_in" || exit 1
O=gpurun_out/r2b; mkdir -p $O
for spec in "dm4:PLK_JITM_DM=4" "dm5:PLK_JITM_DM=5" "dm6:PLK_JITM_DM=6"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --config lg08_g4_protein_200k_256 --steps 10 --warmup 2 --no-cpu-baseline > $O/cfg3_$name.json 2> $O/cfg3_$name.err || { tail -5 $O/cfg3_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_$name.json')); r=d['roofline']; print('$name', d['kernel_path'], '%.4e' % d['value'], 'trav_ms %.3f' % r['traversal_ms'], 'frac %.3f' % r['frac'], 'exec %.3f' % r['executed']['frac'])"
done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
( cd /tmp && PLK_JITM_DM=4 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $R/$O/sq -o run -- python3 $R/bench.py --config lg08_g4_protein_200k_256 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/$O/sq.err ) || { tail -5 $O/sq.err; exit 1; }
( cd /tmp && PLK_JITM_DM=4 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/sq2 -o run -- python3 $R/bench.py --config lg08_g4_protein_200k_256 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/$O/sq2.err ) || { tail -5 $O/sq2.err; echo "sq2 failed (continuing)"; }
echo done
