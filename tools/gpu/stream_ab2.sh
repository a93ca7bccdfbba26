#!/bin/bash
# The prefix stream's cost, bounded from below (round 5): the product against the stream folded to 2 entries (134 MB
# per slot) and to 1 entry per group (67 MB per slot, MALL-resident), plain accesses; timing only.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-stream_ab2}; mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 PIPE=6 ROUNDS=${ROUNDS:-5} POWER=1 TIMING_ONLY=scr2plain,scr1plain timeout -k 10 1100 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so $V/libkhbsgs_scr2plain.so $V/libkhbsgs_scr1plain.so $V/libkhbsgs_half.so > $O/stream_ab2.txt 2>&1 || { tail -20 $O/stream_ab2.txt; exit 1; }
grep -v amdgpu $O/stream_ab2.txt | tail -8
