# Derived utilisation counters for the product scan kernel (VALUBusy, occupancy, TA data stalls).
# Usage (GPU box): JOBS=512 GATE=1 ROUNDS=1 bash tools/gpu/pmc_busy.sh <tag>
export TMPDIR=/tmp
TAG=${1:-busy}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
timeout -s KILL 300 rocprofv3 --pmc VALUBusy OccupancyPercent SQ_INSTS_VALU -d $OUT/a -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $OUT/a.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc MemUnitStalled SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d $OUT/b -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $OUT/b.log 2>&1
echo rc=$?
