#!/bin/bash
# Round 6: the multi-rank bench path on the one-GPU box with this round's bench.py (rank spawn, per-rank library
# record, rank-0 grace): bare --gpus 2 must refuse two ranks on one physical GPU; --share-gpus runs the rehearsal.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06l}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 > $O/n2_refused.json 2> $O/n2_refused.err; echo "bare --gpus 2 rc=$?"
tail -2 $O/n2_refused.err
timeout -k 10 400 python3 bench.py --gpus 2 --share-gpus --steps 5 --warmup 2 > $O/n2_shared.json 2> $O/n2_shared.err || { tail -20 $O/n2_shared.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/n2_shared.json')); c=d['config']; print(d['value'], d['n_gpus'], c['physical_gpus'], c['gpus_shared'], c['launcher'], c['lib_sha16'], d['roofline'].get('traffic'))"
