#!/bin/bash
# Bench lines of the other BASELINE configs and of the check configurations (run under gpurun from the repo
# root), each step under its own time limit; the first failure ends the script.
#   config C (--k 4), config D (--workload p130), and config B without the level-0 gate with the second/third
#   check on the host, on the GPU and in auto mode, plus the gated scan with the GPU check.
# Usage: bash tools/gpu/configs.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-configs}
mkdir -p $O
run() { local name=$1; shift; echo "[$(date +%T)] $name"; timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }; }
run bench_k4 --k 4 --steps 10 --warmup 3 --no-cpu-baseline
run bench_p130 --workload p130 --steps 10 --warmup 3 --no-cpu-baseline
for m in host gpu auto; do run nogate_$m --steps 10 --warmup 2 --no-cpu-baseline --no-gate --check $m; done
run gate_gpu --steps 10 --warmup 2 --no-cpu-baseline --check gpu
for f in $O/*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[1], d['value'], d['ms_per_step'], c.get('candidates'), c.get('device_checked'), c.get('device_check_s'), d['roofline'].get('kernel_busy_ms_per_step'), d['roofline'].get('shader_mhz_avg'))" $f
done
