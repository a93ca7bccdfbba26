#!/bin/bash
# Round 6, third GPU call: the four-context tests, the counter list, the energy of the SALU / SMEM / LDS / scratch
# classes (tools/microbench/valu_energy.hip), the -e address kernels' occupancy A/B (4 / 3 / 2 waves per SIMD) and one
# PMC pass of the product's non-VALU instruction classes over a bench-sized launch.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06c}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest multidev
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multidev.py -x -v --timeout 300 --timeout-method thread > $O/pytest_multidev.log 2>&1 || { tail -30 $O/pytest_multidev.log; exit 1; }
tail -1 $O/pytest_multidev.log
step counters
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list failed"
step energy
timeout -k 10 300 python3 tools/microbench/valu_energy_run.py 4 sleep salu smem lds scratch add_u32 mad64 sleep > $O/valu_energy.jsonl 2> $O/valu_energy.err || { tail -5 $O/valu_energy.err; exit 1; }
cat $O/valu_energy.jsonl
for r in 1 2; do
  for v in product ew3 ew2; do
    step "address -e $v $r"
    if [ $v = product ]; then unset KHB_LIB_DIR; VARG=""; else export KHB_LIB_DIR=keyhuntm1cpu_amd/lib_$v; VARG="--variant $v"; fi
    timeout -k 10 300 python3 bench.py --workload address --endo --chunks 2 --steps 1 --warmup 1 --no-cpu-baseline $VARG > $O/endo_${v}_$r.json 2> $O/endo_${v}_$r.err || { tail -5 $O/endo_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/endo_${v}_$r.json')); print('$v', d['value'], d['roofline']['shader_mhz_avg'])"
  done
done
unset KHB_LIB_DIR
step pmc classes
JOBS=4096 GATE=1 ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT -d $O/pmc_classes -o pmc --output-format csv -- python3 tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/pmc_classes.log 2>&1 || { tail -5 $O/pmc_classes.log; exit 1; }
step done
