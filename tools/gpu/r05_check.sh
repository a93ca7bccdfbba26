#!/bin/bash
# Round-5 check on one GPU box (run from the repo root under gpurun), one step per command, each under its own
# time limit, chained so that the first failure ends the script:
#   power   amdsmi's raw view (fields, energy counter, power cap) before any HIP work
#   tests   the GPU suite
#   bench   the driver's bench command (power sampled over the timed region)
#   trace   the bench under rocprofv3 --kernel-trace --stats (copy / fill kernels gone?)
#   sq      one SQ pass over one bench-sized launch: VALU instructions, VALU cycles, dual-issue cycles
# Usage: bash tools/gpu/r05_check.sh <tag>     Env: PARTS (default "power tests bench trace sq")
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05}
O=gpurun_out/$TAG
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
PARTS=${PARTS:-power tests bench trace sq}
step() { echo "[$(date +%T)] $*"; }
has() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }

if has power; then
step power probe
timeout -k 10 60 python3 tools/gpu/power_probe.py > $O/power_probe.json 2> $O/power_probe.err || exit 1
fi
if has tests; then
step pytest gpu
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
fi
if has bench; then
step bench
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 20 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
fi
if has trace; then
step trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-power > $O/trace_bench.json 2> $O/trace.err || exit 1
KT=$(find $O/trace -name "*kernel_trace.csv" | sort | tail -1)
python3 tools/trace_union.py "$KT" --kernel k_giant_scan --steps 10 --bench $O/trace_bench.json > $O/trace_union.json || exit 1
cat $(find $O/trace -name "*kernel_stats.csv" | sort | tail -1)
fi
if has sq; then
step pmc sq
JOBS=4096 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq2 -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_sq2.log 2>&1 || exit 1
fi
step done
