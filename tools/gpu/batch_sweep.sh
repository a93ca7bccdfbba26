#!/bin/bash
# Config B at the smaller batches a multi-rank -b 66 run shrinks to (bench.py's fit_batch: 2,048 chunks per
# step at N = 4 and 1,024 at N = 8 for 100 + 5 steps), against the N = 1 auto batch of 4,096, on one GPU.
# Usage: bash tools/gpu/batch_sweep.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-batch_sweep}
mkdir -p $O
for r in 1 2; do
  for c in 4096 2048 1024; do
    echo "[$(date +%T)] round $r chunks $c"
    timeout -k 10 180 python3 -u bench.py --steps $((81920 / c)) --warmup 5 --chunks $c --no-cpu-baseline > $O/c${c}_$r.json 2> $O/c${c}_$r.err || exit 1
  done
done
for f in $O/c*.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['frac'], r['shader_mhz_avg'])"; done
