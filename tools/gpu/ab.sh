#!/bin/bash
# Same-process A/B of libkhbsgs builds on the bench's launch (JOBS chunks, default 4096; real gate), interleaved rounds
# (tools/perf_variants.py, one engine open at a time).  Usage: bash tools/gpu/ab.sh <tag> [lib.so ...]
# Env: ROUNDS (5), TIMING_ONLY (variants whose candidates are not compared).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ab}; shift
O=gpurun_out/$TAG
mkdir -p $O
JOBS=${JOBS:-4096} GATE=1 ROUNDS=${ROUNDS:-5} timeout -k 10 600 python3 -u tools/perf_variants.py "$@" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -${TAILN:-4} $O/ab.txt
