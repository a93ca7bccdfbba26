#!/bin/bash
# early_patch.py A/B (round 5): the product vs the first x's fold load issued before the second x is computed.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-early_ab}; mkdir -p $O
JOBS=4096 GATE=1 PIPE=6 ROUNDS=${ROUNDS:-5} POWER=1 timeout -k 10 900 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_early.so > $O/early_ab.txt 2>&1 || { tail -20 $O/early_ab.txt; exit 1; }
grep -v amdgpu $O/early_ab.txt | tail -4
