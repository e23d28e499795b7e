#!/bin/bash
# Tail / grid-size sweep of the headline kernel: tools/gpu_tail.sh <tag> [bench args]
set -o pipefail
TAG=${1:-tail}; shift
O=gpurun_out/$TAG; mkdir -p $O
run() { # run <name> <env...> -- <bench args>
  local name=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --config gtr_g4_dna_1M_64 --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); p=d['config']['n_patterns'] if 'n_patterns' in d['config'] else 0; k=d['kernel_ms_per_step']['partials']; print('$name', d['value'], 'kernel_ms %.4f' % k, 'part/s %.4e' % d['partials_only_updates_per_s'])"
}
run p983k X=1 -- --patterns 983040 "$@" || exit 1
run p1M X=1 -- "$@" || exit 1
run p1081k X=1 -- --patterns 1081344 "$@" || exit 1
run w512 PLK_JIT_WGS=512 -- "$@" || exit 1
run w640 PLK_JIT_WGS=640 -- "$@" || exit 1
run w1024 PLK_JIT_WGS=1024 -- "$@" || exit 1
run w7813 PLK_JIT_WGS=7813 -- "$@" || exit 1
