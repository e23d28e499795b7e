#!/bin/bash
# Row f4 session: DR parity tests, the C++ drop-in test, DR-vs-path measurements.
#   tools/gpu_dr.sh <tag>
set -o pipefail
O=gpurun_out/${1:-dr}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dr.py -x -v --timeout 120 --timeout-method thread > $O/pytest_dr.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_dr.log; exit 1; }
tail -2 $O/pytest_dr.log
timeout -k 10 120 bpp-phyl_amd/host/bin/test_likelihood_gpu > $O/cpp.log 2>&1 || { echo "cpp test failed"; tail -40 $O/cpp.log; exit 1; }
grep -E "DR|PASS|FAIL" $O/cpp.log
timeout -k 10 200 python tools/bench_dr.py --config gtr_g4_dna_1M_64 > $O/dr_cfg2.json 2> $O/dr_cfg2.err || { tail -5 $O/dr_cfg2.err; exit 1; }
cat $O/dr_cfg2.json
timeout -k 10 200 python tools/bench_dr.py --config lg08_g4_protein_200k_256 --path-branches 32 > $O/dr_cfg3.json 2> $O/dr_cfg3.err || { tail -5 $O/dr_cfg3.err; exit 1; }
cat $O/dr_cfg3.json
timeout -k 10 200 python tools/bench_dr.py --config yn98_codon_50k_128 --path-branches 32 > $O/dr_cfg4.json 2> $O/dr_cfg4.err || { tail -5 $O/dr_cfg4.err; exit 1; }
cat $O/dr_cfg4.json
