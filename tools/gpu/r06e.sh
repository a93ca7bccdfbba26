#!/bin/bash
# Round 6: static power against die temperature (tools/microbench/hot_idle_run.py), and the k = 4 stage-1 fold size
# on the half-stream product with more rounds (16 / 32 / 64 MiB).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06e}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step hot_idle
timeout -k 10 300 python3 tools/microbench/hot_idle_run.py 8 40 > $O/hot_idle.json 2> $O/hot_idle.err || { tail -5 $O/hot_idle.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/hot_idle.json'))
for k in ('cold_sleep','heater_2s_bins','hot_sleep'): print(k, [(b['t'], b['power_w'], b['hotspot_c']) for b in d[k]])"
step "fold k=4"
K=4 JOBS=16384 GATE=1 PIPE=6 ROUNDS=5 POWER=1 STAGE1=default,25,26 timeout -k 10 700 python3 -u tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/fold_k4.txt 2>&1 || { tail -20 $O/fold_k4.txt; exit 1; }
tail -7 $O/fold_k4.txt
step done
