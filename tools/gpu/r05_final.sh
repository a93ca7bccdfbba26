#!/bin/bash
# Round-5 evidence on the final tree (one gpurun call): GPU suite, the round profile (trace + PMC + address),
# configs C and D with board power.  Usage: bash tools/gpu/r05_final.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05f}
O=gpurun_out/$TAG
mkdir -p $O/cfg
echo "[$(date +%T)] pytest gpu"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu/round_profile.sh $TAG/prof 20 || exit 1
echo "[$(date +%T)] config C"
timeout -k 10 300 python3 bench.py --k 4 --steps 10 --warmup 3 --no-cpu-baseline > $O/cfg/bench_k4.json 2> $O/cfg/bench_k4.err || exit 1
echo "[$(date +%T)] config D"
timeout -k 10 300 python3 bench.py --workload p130 --steps 20 --warmup 3 --no-cpu-baseline > $O/cfg/bench_p130.json 2> $O/cfg/bench_p130.err || exit 1
for f in $O/cfg/*.json; do python3 -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], r.get('frac'), r.get('shader_mhz_avg'), (r.get('power') or {}).get('power_w_avg'))"; done
echo "[$(date +%T)] done"
