#!/bin/bash
# Round 6: instruction- and scalar-cache behaviour of the product walk (its pair loop is 38 KB of code; the SQC's
# instruction cache is shared by a CU pair), one PMC pass each over a bench-sized launch (tools/perf_variants.py).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06f}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
step icache
JOBS=4096 GATE=1 ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_icache -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_icache.log 2>&1 || { tail -5 $O/pmc_icache.log; exit 1; }
step dcache
JOBS=4096 GATE=1 ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/pmc_dcache -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_dcache.log 2>&1 || { tail -5 $O/pmc_dcache.log; exit 1; }
step done
