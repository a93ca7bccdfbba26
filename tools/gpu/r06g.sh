#!/bin/bash
# Round 6: the zero-memory build of the current product (half prefix stream folded into the caches + the all-zero
# gate) against the product, two launches in flight, board power per configuration: the compute-only energy per
# giant step and the memory side in situ.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06g}; O=gpurun_out/$T; mkdir -p $O
JOBS=4096 GATE=1 GATE_ZERO=13 PIPE=6 ROUNDS=3 POWER=1 timeout -k 10 600 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so keyhuntm1cpu_amd/lib_scr1half/libkhbsgs_scr1half.so > $O/zero_mem.txt 2>&1 || { tail -20 $O/zero_mem.txt; exit 1; }
tail -14 $O/zero_mem.txt
