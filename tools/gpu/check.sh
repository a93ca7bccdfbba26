#!/bin/bash
# GPU-box round check (run under gpurun from the repo root): smoke(), the GPU test suite, the driver's N=1 bench
# command, and `bench.py --gpus 2` run bare (bench.py starts its two ranks itself; both share the one GPU).
# Usage: bash tools/gpu/check.sh <tag> [pytest -k expression]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
K=${2:+-k "$2"}
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 20 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
cat $O/bench_n2.json
