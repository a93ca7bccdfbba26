#!/bin/bash
# KHB_HALF_STREAM A/B: the product vs the half prefix stream, two launches in flight, real gate,
# board power per configuration.  Build first: tools/build_variant.sh half -DKHB_HALF_STREAM=1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-half_ab}; mkdir -p $O
JOBS=4096 GATE=1 PIPE=6 ROUNDS=${ROUNDS:-7} POWER=1 timeout -k 10 900 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_half.so > $O/half_ab.txt 2>&1 || { tail -20 $O/half_ab.txt; exit 1; }
tail -3 $O/half_ab.txt
