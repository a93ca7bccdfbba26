#!/bin/bash
# The round's roofline evidence (run under gpurun from the repo root), one command per step, each under its
# own time limit, chained so that the first failure ends the script:
#   1. the driver's bench command under `rocprofv3 --kernel-trace --stats` (trace.json = the line printed
#      under the profiler) and tools/trace_union.py over its trace (device-busy union vs the line);
#   2. the HBM PMC passes behind profiles/pmc_latest.json (real gate vs the all-zero 1 KiB gate over the
#      bench's auto 4096-chunk launch, so bench.py's roofline.traffic applies to its default line;
#      FETCH_SIZE / WRITE_SIZE in passes of their own) and the SQ pass;
#   3. config E: bench.py --workload address, and SQ_INSTS_VALU of one 8-chunk launch of the product
#      library and of the hash-less addrwalk build (the x/y walk term of the floor, tools/addr_floor.py).
# Usage: bash tools/gpu/round_profile.sh <tag> [steps]     Env: PARTS (default "trace pmc address"), PMC_JOBS
# (chunks per PMC launch, default 4096 = the bench's auto batch at 4 waves/SIMD), K (default 1; K=4 PMC_JOBS=16384
# PARTS=pmc gives config C's record, profiles/pmc_latest_k4.json).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
STEPS=${2:-20}
O=gpurun_out/$TAG
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
W=keyhuntm1cpu_amd/lib/variants/libkhbsgs_addrwalk.so
J=${PMC_JOBS:-4096}
export K=${K:-1}          # the geometry's k (perf_variants reads K; K=4 with PMC_JOBS=16384 is config C's launch)
PARTS=${PARTS:-trace pmc address}
step() { echo "[$(date +%T)] $*"; }
has() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }

if has trace; then
step trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- \
  python3 bench.py --gpus 1 --steps $STEPS --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || exit 1
KT=$(find $O/trace -name "*kernel_trace.csv" | sort | tail -1)
python3 tools/trace_union.py "$KT" --kernel k_giant_scan --steps $STEPS --bench $O/trace_bench.json > $O/trace_union.json || exit 1
cat $O/trace_union.json
fi

if has pmc; then
for g in 0 13; do
  step pmc fetch gate_zero=$g
  JOBS=$J GATE=1 GATE_ZERO=$g ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum -d $O/pmc_fetch_$g -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_fetch_$g.log 2>&1 || exit 1
done
step pmc write
JOBS=$J GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum -d $O/pmc_write_0 -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_write_0.log 2>&1 || exit 1
step pmc sq
JOBS=$J GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_sq.log 2>&1 || exit 1
step pmc sq2
JOBS=$J GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq2 -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_sq2.log 2>&1 || exit 1
for d in $O/pmc_fetch_0 $O/pmc_fetch_13 $O/pmc_write_0 $O/pmc_sq $O/pmc_sq2; do   # pmc_summary reads <dir>/pmc_counter_collection.csv
  f=$(find $d -name "*counter_collection.csv" | sort | tail -1)
  [ "$f" = "$d/pmc_counter_collection.csv" ] || cp "$f" $d/pmc_counter_collection.csv
done
python3 tools/pmc_summary.py $O $J $O/pmc_latest.json $K > /dev/null || exit 1
fi

if has address; then
step address bench
timeout -k 10 300 python3 bench.py --workload address --steps 3 --warmup 1 --cpu-seconds 20 > $O/bench_address.json 2> $O/bench_address.err || exit 1
cat $O/bench_address.json
if [ -f $W ]; then
  for lib in $L $W; do
    n=$(basename $lib .so)
    step pmc address $n
    timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/addr_$n -o pmc --output-format csv -- python3 tools/addr_floor.py $lib > $O/addr_$n.json 2> $O/addr_$n.err || exit 1
    cat $O/addr_$n.json
  done
fi
fi
step done
