#!/bin/bash
# Round-6 end check on the final tree: the GPU suite, smoke() and the driver's bench command (with its CPU baseline),
# then config E with -e (short, its roofline from the -e PMC count).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06_end}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; p=r['power']; print(d['value'], r['frac'], r['executed']['frac'], r['shader_mhz_avg'], r.get('traffic'), r.get('traffic_note'), p.get('power_w_from_energy'), d['cpu_baseline']['value'], d['config']['lib_sha16'])"
step bench_address_e
timeout -k 10 400 python3 bench.py --workload address --endo --chunks 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_address_e.json 2> $O/bench_address_e.err || { tail -5 $O/bench_address_e.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_address_e.json')); r=d['roofline']; print(d['value'], r.get('frac'), r.get('shader_mhz_avg'))"
step done
