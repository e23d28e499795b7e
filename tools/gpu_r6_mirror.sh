#!/bin/bash
# round 6: the Bio++ mirror's cfg2 line (setParameters + getValue through the API, unscaled
# first) twice, and once under the kernel trace (which kernels the mirror's evaluations run)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD; O=gpurun_out/${TAG:-r6mirror}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 bpp-phyl_amd/host/bin/bench_mirror cfg2 1000000 20 5 > $O/mirror_cfg2_20_5_$i.json || exit $?
  cat $O/mirror_cfg2_20_5_$i.json
done
timeout -k 10 300 bpp-phyl_amd/host/bin/bench_mirror cfg2 > $O/mirror_cfg2_200_50.json || exit $?
cat $O/mirror_cfg2_200_50.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o m -- \
  $R/bpp-phyl_amd/host/bin/bench_mirror cfg2 1000000 20 5 > $R/$O/mirror_cfg2_rocprof.json ) || exit 1
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp $f $O/mirror_cfg2_kernel_stats.csv && rm -rf $O/trace
cut -d, -f1-4 $O/mirror_cfg2_kernel_stats.csv | head -8
