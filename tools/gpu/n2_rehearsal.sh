#!/bin/bash
# Multi-rank rehearsal on the one-GPU box (round 5): bare `bench.py --gpus 2` must refuse two ranks on one physical
# GPU (exit non-zero, no line); with --share-gpus it runs and the line says physical_gpus 1, gpus_shared true.
set -o pipefail
O=gpurun_out/${1:-n2}; mkdir -p $O
if timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/refused.json 2> $O/refused.err; then
  echo "ERROR: two ranks on one GPU were not refused"; exit 1
fi
echo "refused as expected: $(grep -m1 'physical GPU' $O/refused.err)"
timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --share-gpus > $O/shared.json 2> $O/shared.err || { tail -5 $O/shared.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/shared.json')); c=d['config']; print(d['n_gpus'], d['value'], c['physical_gpus'], c['gpus_shared'], c['launcher'])"
