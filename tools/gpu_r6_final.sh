#!/bin/bash
# Round-6 measurement session: the driver's exact bench command (twice), the same under the
# kernel trace, per-configuration lines, PMC passes per configuration, the clock probe.
#   tools/gpu_r6_final.sh <out-subdir>
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd); O=gpurun_out/${1:-r6final}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default_$i.json 2> $O/bench_default_$i.err || { tail -5 $O/bench_default_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_default_$i.json').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['value'], d['roofline']['frac'], d['strong']['ms_per_step'])"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/deftrace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/$O/bench_default_under_rocprof.json 2> $R/$O/rocprof.err ) || { tail -5 $O/rocprof.err; exit 1; }
cp $(find $O/deftrace -name "*kernel_stats.csv" | head -1) $O/default_kernel_stats.csv && rm -rf $O/deftrace
for c in "cfg3 --config lg08_g4_protein_200k_256 --cpu-runs 3" "cfg4 --config yn98_codon_50k_128 --cpu-runs 3" \
         "cfg5 --config nh_gtr_g4_dna_2M_512 --cpu-runs 3" "cfg5s --scaling strong --no-cpu-baseline"; do
  set -- $c; t=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/line_$t.json 2> $O/line_$t.err || { tail -5 $O/line_$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/line_$t.json').read().strip().splitlines()[-1]); print('$t', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --clock-json $O/clock_20_5.json --no-cpu-baseline --no-strong > $O/line_clock.json 2> $O/clock.err || exit 1
p() { tag=$1; cfg=$2; steps=$3
  bash tools/gpu_prof.sh $tag $cfg lnl $steps > /dev/null || exit 1
  python tools/traffic_from_pmc.py $tag $cfg lnl ../$O/pmc > /dev/null || exit 1
  rm -rf gpurun_out/prof/$tag; echo "$tag profiled"; }
p r6f_cfg2_lnl gtr_g4_dna_1M_64 20
p r6f_cfg5_lnl nh_gtr_g4_dna_2M_512 20
p r6f_cfg4_lnl yn98_codon_50k_128 20
p r6f_cfg3_lnl lg08_g4_protein_200k_256 10
echo done
