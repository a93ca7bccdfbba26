#!/bin/bash
# Round 6: config C's PMC record (k = 4: traffic and VALU of one 16,384-chunk launch, the bench's auto batch at k = 4),
# then config C's line with it attached.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06k}; O=gpurun_out/$T; mkdir -p $O
K=4 PMC_JOBS=16384 PARTS=pmc bash tools/gpu/round_profile.sh $T/prof_k4 || exit 1
cp gpurun_out/$T/prof_k4/pmc_latest.json profiles/pmc_latest_k4.json
timeout -k 10 400 python3 bench.py --k 4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_k4.json 2> $O/bench_k4.err || { tail -20 $O/bench_k4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k4.json')); r=d['roofline']; print('k4', d['value'], r['frac'], r.get('traffic'), r.get('traffic_note'), r['executed'].get('valu_busy_pct'))"
