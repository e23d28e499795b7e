#!/bin/bash
# One-process eight-shard rehearsal of the multi-device handle on the one GPU of the box
# (bench.py --gpus 8 --devices 0,...,0): host fan-out timestamps (plk_get_fanout) with the
# runtime's default four hardware queues, and with eight (one per shard's stream, as eight
# devices would have).
set -o pipefail
O=gpurun_out/${1:-r5f}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --no-cpu-baseline --steps 20 > $O/dev8_q$q.json 2> $O/dev8_q$q.err || exit $?
done
python - <<PY
import json
for q in (4, 8):
    r = json.load(open(f"$O/dev8_q{q}.json"))
    for name, x in (("weak 8 x 1M", r), ("strong 2M / 8", r["strong"])):
        f = x["fanout"]
        print(f"queues {q} {name}: ms/step {x['ms_per_step']:.4f}; traversal launched (us) " +
              " ".join("%.1f" % v for v in f["traversal_launched_us"]) +
              f"; spread mean {f['launch_spread_mean_us']:.1f} max {f['launch_spread_max_us']:.1f}")
PY
