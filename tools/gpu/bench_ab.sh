#!/bin/bash
# Whole-bench A/B of an alternative library pair (KHB_LIB_DIR=<dir with libkhbsgs.so + libkhhost.so>, built by
# LIBDIR=1 tools/build_variant.sh <name> ...) against the in-tree product: the driver's bench command, alternating,
# ROUNDS times each, no CPU baseline.  The alternative's lines carry "variant": <name> (bench.py --variant).
# Usage: bash tools/gpu/bench_ab.sh <tag> <alt lib dir> [steps] [extra bench.py args...]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; ALT=$2; STEPS=${3:-20}; shift 3; EXTRA="$*"
NAME=$(basename $ALT | sed 's/^lib_//')
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in product alt; do
    if [ $v = alt ]; then export KHB_LIB_DIR=$ALT; VARG="--variant $NAME"; else unset KHB_LIB_DIR; VARG=""; fi
    timeout -k 10 300 python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline $EXTRA $VARG > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/${v}_$r.json')); r=d['roofline']; p=r.get('power',{}); print('$v $r', d['value'], r['shader_mhz_avg'], p.get('power_w_avg'), p.get('ppt_residency_frac'), p.get('joules_per_1e9_giant_steps'), d['config']['lib_sha16'])"
  done
done
