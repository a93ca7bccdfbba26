#!/bin/bash
# GPU-box profiling recipe for the round's evidence (run under gpurun from the repo root):
#   bench line, rocprofv3 kernel-trace stats, and the two HBM PMC passes (separate runs).
# Usage: bash tools/profile_bench.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="--steps 5 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 600 python3 bench.py $* > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $B > $OUT/trace.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py $B > $OUT/fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py $B > $OUT/write.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU OccupancyPercent -d $OUT/valu -o valu --output-format csv -- python3 bench.py $B > $OUT/valu.log 2>&1
rc=$?
cat $OUT/bench.json
echo "rc=$rc"
exit $rc
