#!/bin/bash
# Stage-1 fold size at k=1 on the final tree (round 5): the default 2 MiB against 1 MiB and 4 MiB, two launches in
# flight, board power.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-fold_ab}; mkdir -p $O
JOBS=4096 GATE=1 STAGE1=default,20,22 PIPE=6 ROUNDS=${ROUNDS:-5} POWER=1 timeout -k 10 900 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/fold_ab.txt 2>&1 || { tail -20 $O/fold_ab.txt; exit 1; }
grep -v amdgpu $O/fold_ab.txt | tail -6
