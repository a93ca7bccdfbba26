#!/bin/bash
# The zero-memory timing build: the product and the cache-resident prefix stream (scr1plain),
# each with the real gate and with the all-zero 1 KiB gate, two launches in flight, board power per configuration.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-zero_mem_ab}; mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 GATE_ZERO=13 PIPE=6 ROUNDS=${ROUNDS:-3} POWER=1 TIMING_ONLY=scr1plain timeout -k 10 900 python3 -u tools/perf_variants.py \
  keyhuntm1cpu_amd/lib/libkhbsgs.so $V/libkhbsgs_scr1plain.so > $O/zero_mem_ab.txt 2>&1 || { tail -20 $O/zero_mem_ab.txt; exit 1; }
grep -v amdgpu $O/zero_mem_ab.txt | tail -8
