#!/bin/bash
# Round 6: the L2-resident scratch (spill) pattern's energy, and the stage-1 fold size re-tuned on the half-stream
# product at k = 1 (2 vs 4 MiB) and k = 4 (8 / 16 / 32 MiB), two launches in flight, board power per configuration.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06d}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step energy
timeout -k 10 200 python3 tools/microbench/valu_energy_run.py 4 sleep scratch_l2 scratch lds mad64 sleep > $O/valu_energy.jsonl 2> $O/valu_energy.err || { tail -5 $O/valu_energy.err; exit 1; }
cat $O/valu_energy.jsonl
step "fold k=1"
JOBS=4096 GATE=1 PIPE=6 ROUNDS=4 POWER=1 STAGE1=default,22 timeout -k 10 400 python3 -u tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/fold_k1.txt 2>&1 || { tail -20 $O/fold_k1.txt; exit 1; }
tail -4 $O/fold_k1.txt
step "fold k=4"
K=4 JOBS=16384 GATE=1 PIPE=6 ROUNDS=3 POWER=1 STAGE1=default,23,25 timeout -k 10 500 python3 -u tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/fold_k4.txt 2>&1 || { tail -20 $O/fold_k4.txt; exit 1; }
tail -5 $O/fold_k4.txt
step done
