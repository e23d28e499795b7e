#!/bin/bash
# Round-2 A/B experiments, one case per run directory of profiles/r02/ab_runs.md
# (gpurun_out/r2<letter>/).  Each is a bench sweep over environment switches
# (tools/gpu_sweep_env.sh), sometimes behind a focused parity run (tools/gpu_tests.sh).
#   tools/ab_r02.sh <letter>        e.g. /usr/local/graft/bin/gpurun -- 'bash tools/ab_r02.sh p'
# The defaults these experiments chose are in csrc/plk.hip next to each switch.
set -o pipefail
C2=gtr_g4_dna_1M_64; C3=lg08_g4_protein_200k_256; C4=yn98_codon_50k_128; C5=nh_gtr_g4_dna_2M_512
S="bash tools/gpu_sweep_env.sh"
T="bash tools/gpu_tests.sh"
case "$1" in
  a)  # jit_treeM (20 states) first sweep; 1-GPU rehearsals of the N>1 bench
      $T r2a -k "multi or comm or sharded" || exit 1
      $S r2a $C3 "cfg3_base:" "cfg3_dm2:PLK_JITM_DM=2" "cfg3_dm4:PLK_JITM_DM=4" "cfg3_l2:PLK_JITM_L=2" \
        "cfg3_minw1:PLK_JITM_MINW=1" "cfg3_treeM:PLK_JITM=0" || exit 1
      O=gpurun_out/r2a
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo > $O/rehearse_gloo2.json 2> $O/rehearse_gloo2.err || exit 1
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29512 bench.py --gpus 1 --steps 10 --warmup 2 --force-dist --no-cpu-baseline > $O/rehearse_nccl1.json 2> $O/rehearse_nccl1.err || exit 1 ;;
  b)  $S r2b $C3 "cfg3_dm4:PLK_JITM_DM=4" "cfg3_dm5:PLK_JITM_DM=5" "cfg3_dm6:PLK_JITM_DM=6" ;;
  c)  # matrix-core kernels for 4 / 20 / 64 states against the defaults
      $S r2c $C3 "cfg3_staged4:PLK_JITM_DM=4" "cfg3_direct4:PLK_JITM_DM=4,PLK_JITM_DIRECT=1" "cfg3_direct3:PLK_JITM_DM=3,PLK_JITM_DIRECT=1" || exit 1
      $S r2c $C4 "cfg4_treeM:" "cfg4_jitm:PLK_JITM64=1" "cfg4_jitm_direct:PLK_JITM64=1,PLK_JITM_DIRECT=1" "cfg4_jitm_dm2:PLK_JITM64=1,PLK_JITM_DM=2" || exit 1
      $S r2c $C2 "cfg2_jit4:" "cfg2_mfma8:PLK_S4_JITM=1" "cfg2_mfma8d:PLK_S4_JITM=1,PLK_JITM_DIRECT=1" "cfg2_mfma12:PLK_S4_JITM=1,PLK_JITM_DM=12" || exit 1
      $S r2c $C5 "cfg5_jit4:" "cfg5_mfma8:PLK_S4_JITM=1" "cfg5_mfma8d:PLK_S4_JITM=1,PLK_JITM_DIRECT=1" ;;
  d)  $S r2d $C3 "dm4:PLK_JITM_DM=4" "dm4h:PLK_JITM_DM=4,PLK_JITM_HOIST=1" "dm4p2:PLK_JITM_DM=4,PLK_JITM_PD=2" \
        "dm3p2:PLK_JITM_DM=3,PLK_JITM_PD=2" "dm3p2h:PLK_JITM_DM=3,PLK_JITM_PD=2,PLK_JITM_HOIST=1" \
        "dm3h:PLK_JITM_DM=3,PLK_JITM_HOIST=1" "dm4l2:PLK_JITM_DM=4,PLK_JITM_L=2" ;;
  e)  # generated 4-state kernels kept for ISA reading (llvm-objdump -d gpurun_out/r2e/dump*/plk_jit_0.co)
      mkdir -p gpurun_out/r2e/dump2 gpurun_out/r2e/dump5
      PLK_JIT_DUMP=gpurun_out/r2e/dump2 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2e/cfg2.json || exit 1
      PLK_JIT_DUMP=gpurun_out/r2e/dump5 timeout -k 10 200 python bench.py --config $C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2e/cfg5.json ;;
  f)  # high-word rescale decision
      $T r2f -k "jit or scaling or rescale or fixture" quick || exit 1
      $S r2f $C5 "base:" "dm4:PLK_JIT_CIW_DM=4" "dm6:PLK_JIT_CIW_DM=6" "l2:PLK_JIT_L=2" "g1:PLK_JIT_G=1" "g4:PLK_JIT_G=4" \
        "minw3:PLK_JIT_MINW=3" "ciw0:PLK_JIT_CIW=0" || exit 1
      $S r2f3 $C3 "base:" && $S r2f2 $C2 "base:" ;;
  g)  $S r2g $C5 "base:" "g4:PLK_JIT_G=4" "g4l2:PLK_JIT_G=4,PLK_JIT_L=2" "g6:PLK_JIT_G=6" "g8:PLK_JIT_G=8" \
        "g8l2:PLK_JIT_G=8,PLK_JIT_L=2" "g4dm4:PLK_JIT_G=4,PLK_JIT_CIW_DM=4" "g4dm6:PLK_JIT_G=4,PLK_JIT_CIW_DM=6" "g4w3:PLK_JIT_G=4,PLK_JIT_MINW=3" ;;
  h)  $S r2h $C5 "g4dm6:PLK_JIT_G=4,PLK_JIT_CIW_DM=6" "g4dm7:PLK_JIT_G=4,PLK_JIT_CIW_DM=7" "g4dm8:PLK_JIT_G=4,PLK_JIT_CIW_DM=8" \
        "g3dm6:PLK_JIT_G=3,PLK_JIT_CIW_DM=6" "g8dm6:PLK_JIT_G=8,PLK_JIT_CIW_DM=6" "g8dm7:PLK_JIT_G=8,PLK_JIT_CIW_DM=7" \
        "g4dm6l2:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_L=2" "g4dm6p32:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_PAIR_KB=32" \
        "g4dm6p96:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_PAIR_KB=96" "g4dm6t96:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_TAB_KB=96" ;;
  i)  # counters of the round's kernels (digest: tools/stalls_digest.py gpurun_out/stalls/<cfg>)
      $S r2i $C5 "cfg5:" || exit 1
      bash tools/gpu_stalls.sh cfg5 $C5 && bash tools/gpu_stalls.sh cfg2 $C2 && bash tools/gpu_stalls.sh cfg3 $C3 ;;
  k)  # cost of the P(t) scalar loads: every internal branch reads node 0's P (wrong results, timing only)
      $S r2k5 $C5 "base:" "samep:PLK_DEBUG_SAMEP=1" && $S r2k2 $C2 "base:" "samep:PLK_DEBUG_SAMEP=1" ;;
  l)  $T r2l -k "jit_tree4 or nonhomogeneous or scaling or bench_mode" quick || exit 1
      $S r2l $C5 "ppipe:" "noppipe:PLK_JIT_PPIPE=0" "ppipe_dm5:PLK_JIT_CIW_DM=5" "ppipe_g8:PLK_JIT_G=8" && $S r2l2 $C2 "base:" ;;
  m)  $T r2m -k "jit_tree4 or nonhomogeneous or scaling or bench_mode" quick || exit 1
      $S r2m $C5 "stream:" "nopipe:PLK_JIT_PPIPE=0" "g8:PLK_JIT_G=8" "dm5:PLK_JIT_CIW_DM=5" "dm7:PLK_JIT_CIW_DM=7" ;;
  n)  $S r2n $C5 "base:" "samep:PLK_DEBUG_SAMEP=1" "g3:PLK_JIT_G=3" "g5:PLK_JIT_G=5" "g6:PLK_JIT_G=6" \
        "pair32:PLK_JIT_PAIR_KB=48" "w2:PLK_JIT_MINW=2" ;;
  o)  $S r2o $C5 "split:" "nosplit:PLK_JIT_SPLIT_Y=0" "split_g8:PLK_JIT_G=8" "split_dm7:PLK_JIT_CIW_DM=7" "split_dm5:PLK_JIT_CIW_DM=5" || exit 1
      $S r2o2 $C2 "split:" "nosplit:PLK_JIT_SPLIT_Y=0" || exit 1
      $T r2o -k "jit_tree4 or nonhomogeneous or bench_mode" quick ;;
  p)  $S r2p $C5 "g8:PLK_JIT_G=8" "g6:PLK_JIT_G=6" "g7:PLK_JIT_G=7" "g8dm5:PLK_JIT_G=8,PLK_JIT_CIW_DM=5" \
        "g8l2:PLK_JIT_G=8,PLK_JIT_L=2" "g8t64:PLK_JIT_G=8,PLK_JIT_TAB_KB=64" "g8p96:PLK_JIT_G=8,PLK_JIT_PAIR_KB=96" || exit 1
      $S r2p2 $C2 "g2:PLK_JIT_G=2" "g4:PLK_JIT_G=4" "l4:PLK_JIT_L=4" "dm8:PLK_JIT_DM=8" ;;
  q)  # the generated 20-state kernel kept for ISA reading
      mkdir -p gpurun_out/r2q/dump3
      PLK_JIT_DUMP=gpurun_out/r2q/dump3 timeout -k 10 200 python bench.py --config $C3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2q/cfg3.json ;;
  r)  $S r2r $C3 "base:" "youter:PLK_JITM_YOUTER=1" "youter_dm3:PLK_JITM_YOUTER=1,PLK_JITM_DM=3" "youter_w1:PLK_JITM_YOUTER=1,PLK_JITM_MINW=1" || exit 1
      PLK_JITM_YOUTER=1 $T r2r_y -k "jit_treeM_vs_oracle" quick ;;
  s)  $S r2s $C3 "nopad:" "pad:PLK_JITM_PADSTAGE=1" "nopad2:" "pad2:PLK_JITM_PADSTAGE=1" ;;
  t)  # launch anatomy of the 4-state kernel: whole / return after table staging / return at once
      $S r2t $C2 "base:" "stage:PLK_DEBUG_STAGE_ONLY=1" "empty:PLK_DEBUG_STAGE_ONLY=2" || exit 1
      $S r2t5 $C5 "base:" "stage:PLK_DEBUG_STAGE_ONLY=1" "empty:PLK_DEBUG_STAGE_ONLY=2" ;;
  u)  # cost of the in-handle RCCL exchange: plain 1-GPU run, 1 RCCL rank, 2 gloo ranks on one GPU
      O=gpurun_out/r2u; mkdir -p $O
      timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/plain.json || exit 1
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29512 bench.py --gpus 1 --steps 40 --warmup 3 --force-dist --no-cpu-baseline > $O/nccl1.json || exit 1
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --dist-backend gloo > $O/gloo2.json || exit 1
      $T r2u -k "comm or multi" quick ;;
  v)  $S r2v4 $C4 "base:" "rows64:PLK_CHERRY_ROWS=64" "rows128:PLK_CHERRY_ROWS=128" "rows512:PLK_CHERRY_ROWS=512" \
        "g2:PLK_TREEM_G=2" "g1:PLK_TREEM_G=1" "dm2:PLK_TREEM_DM=2" || exit 1
      $S r2v3 $C3 "base:" "rows64:PLK_CHERRY_ROWS=64" "rows128:PLK_CHERRY_ROWS=128" ;;
  w)  $S r2w $C2 "base:" "pw2:PLK_JIT_PW=2" "pw2g1:PLK_JIT_PW=2,PLK_JIT_G=1" "pw2g2:PLK_JIT_PW=2,PLK_JIT_G=2" \
        "l2:PLK_JIT_L=2" "l5:PLK_JIT_L=5" "dm6:PLK_JIT_DM=6" "pair0:PLK_JIT_PAIR_KB=0" ;;
  y)  $S r2y $C3 "base:" "dm3w3:PLK_JITM_DM=3,PLK_JITM_MINW=3" "dm2w3:PLK_JITM_DM=2,PLK_JITM_MINW=3" \
        "dm2w4:PLK_JITM_DM=2,PLK_JITM_MINW=4" "dm3w3l2:PLK_JITM_DM=3,PLK_JITM_MINW=3,PLK_JITM_L=2" "dm4w3:PLK_JITM_DM=4,PLK_JITM_MINW=3" ;;
  x)  # jit_treeM MFMA-pipe and LDS counters (tools/stalls_digest.py gpurun_out/stalls/cfg3m plk_jit_treeM)
      R=$(pwd); O=$R/gpurun_out/stalls/cfg3m; mkdir -p $O
      ( export TMPDIR=/tmp; cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d $O/a -o run -- python3 $R/bench.py --config $C3 --no-cpu-baseline --steps 2 --warmup 1 > /dev/null ) ;;
  z)  # cfg3 register pressure: the same tree and model with 1 / 2 / 4 rate classes (fp64 fraction per class count)
      O=gpurun_out/r2z; mkdir -p $O
      for spec in "c1:1:" "c2:2:" "c2w3:2:PLK_JITM_MINW=3" "c2dm5:2:PLK_JITM_DM=5" "c4:4:"; do
        IFS=: read name cls envs <<< "$spec"
        env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --config $C3 --classes $cls --steps 10 --warmup 2 \
          --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
        python -c "import json; d=json.load(open('$O/$name.json')); r=d['roofline']; print('$name', d['kernel_path'], 'ms %.4f' % r['traversal_ms'], 'frac %.3f' % r['frac'], 'exec %.3f' % r['executed']['frac'])"
      done ;;
  hyb)  # 20 states: hybrid 16x16x4 + 4x4x4 contraction vs all-4x4x4
      PLK_JITM_HYB=1 $T r2hyb -k "jit_treeM or bench_mode" quick || exit 1
      $S r2hyb $C3 "hyb:PLK_JITM_HYB=1" "nohyb:" "hyb_dm3:PLK_JITM_HYB=1,PLK_JITM_DM=3" "hyb_dm5:PLK_JITM_HYB=1,PLK_JITM_DM=5" \
        "hyb_l2:PLK_JITM_HYB=1,PLK_JITM_L=2" ;;
  pyov)  # Python-side evaluate overhead (cached ctypes pointers): step time of the default bench lines
      $T r2pyov -k "multi or bench_mode or comm or evaluate" quick || exit 1
      for c in $C2 $C5; do timeout -k 10 200 python bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/r2pyov_$c.json || exit 1
        python -c "import json; d=json.load(open('gpurun_out/r2pyov_$c.json')); print('$c', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel %.4f' % d['kernel_ms_per_step']['partials'])"; done ;;
  hiptrace)  # host-side timeline of the evaluation loop (HIP API + kernels)
      R=$(pwd); O=$R/gpurun_out/r2hiptrace; mkdir -p $O
      ( export TMPDIR=/tmp; cd /tmp && timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O -o run -- \
        python3 $R/bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-events > $O/bench.json ) ;;
  jmdbg)  # jit_treeM timing anatomy: without the per-contraction barrier / P(t) loads (wrong results)
      $S r2jmdbg $C3 "base:" "nobar:PLK_DEBUG_JITM=1" "noload:PLK_DEBUG_JITM=2" "neither:PLK_DEBUG_JITM=3" \
        "onea:PLK_DEBUG_JITM=4" "onea_neither:PLK_DEBUG_JITM=7" ;;
  g64)  # treeM<64>: 128-pattern workgroups (P^T staging shared by 8 waves)
      PLK_TREEM_G64=8 $T r2g64 -k "yn98 or 64 or bench_mode" quick || exit 1
      $S r2g64 $C4 "g4:" "g8:PLK_TREEM_G64=8" "g4b:" "g8b:PLK_TREEM_G64=8" ;;
  jitcache)  # hiprtc compile time per config and the on-disk code-object cache (second process hits it)
      export PLK_JIT_LOG=1 PLK_JIT_CACHE=$(pwd)/gpurun_out/r2jitcache/cache
      for c in $C2 $C3 $C5; do
        timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r2jitcache_$c.1.err || exit 1
        timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/r2jitcache_$c.2.err || exit 1
        grep "\[plk\]" gpurun_out/r2jitcache_$c.1.err gpurun_out/r2jitcache_$c.2.err
      done
      $T r2jitcache -k "multi or jit_tree4_bitwise" quick ;;
  occ5)  # cfg5: three waves per SIMD via lower fragment height (classes-in-wave register levels)
      $S r2occ5 $C5 "base:" "dm3w3:PLK_JIT_CIW_DM=3,PLK_JIT_MINW=3,PLK_JIT_L=1" "dm4w3:PLK_JIT_CIW_DM=4,PLK_JIT_MINW=3,PLK_JIT_L=1" \
        "dm3:PLK_JIT_CIW_DM=3,PLK_JIT_L=1" "dm4l1:PLK_JIT_CIW_DM=4,PLK_JIT_L=1" "dm5w3:PLK_JIT_CIW_DM=5,PLK_JIT_MINW=3,PLK_JIT_L=1" ;;
  hyb64)  # 64 states: per-tree kernel on 16x16x4 (PLK_JITM64=1 PLK_JITM_HYB=1) vs treeM<64> and jitm64 on 4x4x4
      PLK_JITM64=1 PLK_JITM_HYB=1 $T r2hyb64 -k "jit_treeM_64 or bench_mode" quick || exit 1
      $S r2hyb64 $C4 "treeM:" "jitm64:PLK_JITM64=1" "jitm64hyb:PLK_JITM64=1,PLK_JITM_HYB=1" \
        "jitm64hyb_dm2:PLK_JITM64=1,PLK_JITM_HYB=1,PLK_JITM_DM=2" "jitm64hyb_w1:PLK_JITM64=1,PLK_JITM_HYB=1,PLK_JITM_MINW=1" ;;
  *)  echo "usage: tools/ab_r02.sh <a..y>"; exit 2 ;;
esac
