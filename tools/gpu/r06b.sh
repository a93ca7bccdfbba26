#!/bin/bash
# Round 6, second GPU call: the GPU suite on the tree with the half prefix stream as the product and -m address -e,
# smoke(), the bench lines of configs B (with its CPU baseline), C, D, E and E with -e, then the round's trace and PMC
# evidence for the new product kernel (tools/gpu/round_profile.sh trace + pmc -> pmc_latest.json).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06b}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() { local name=$1; shift; step $name; timeout -k 10 400 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }; \
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r.get('frac'), r.get('shader_mhz_avg'), (r.get('power') or {}).get('power_w_avg'), (d.get('cpu_baseline') or {}).get('value'), d['config'].get('lib_sha16'))" $O/$name.json; }
run bench --gpus 1 --steps 20 --warmup 5
run bench_k4 --k 4 --steps 10 --warmup 3 --no-cpu-baseline
run bench_p130 --workload p130 --steps 10 --warmup 3 --no-cpu-baseline
run bench_address --workload address --steps 3 --warmup 1 --cpu-seconds 10 --cpu-windows 1
run bench_address_e --workload address --endo --steps 2 --warmup 1 --cpu-seconds 10 --cpu-windows 1
PARTS="trace pmc" bash tools/gpu/round_profile.sh $T/prof 20 || exit 1
step done
