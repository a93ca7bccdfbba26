#!/bin/bash
# The prefix stream's cost, re-priced (round 5): product (non-temporal stream), plain-load/store stream, the stream
# folded to 2 entries per group with non-temporal (scr2) and plain (scr2plain: L2-resident) accesses, and the half
# stream; real gate, two launches in flight, board power.  Build: tools/experiments/calib_build.sh
# plainscr|scr|half ... and the scr2plain pair (plainscr_patch + scr_patch), see DESIGN.md §5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-stream_ab}; mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 PIPE=6 ROUNDS=${ROUNDS:-5} POWER=1 TIMING_ONLY=scr2plain timeout -k 10 1100 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so $V/libkhbsgs_plainscr.so $V/libkhbsgs_scr2.so $V/libkhbsgs_scr2plain.so \
  $V/libkhbsgs_half.so > $O/stream_ab.txt 2>&1 || { tail -20 $O/stream_ab.txt; exit 1; }
tail -5 $O/stream_ab.txt
