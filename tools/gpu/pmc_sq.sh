# SQ instruction/wait counters for the product scan kernel (one perf_variants launch set).
# Usage (GPU box): bash tools/gpu/pmc_sq.sh <tag>
export TMPDIR=/tmp
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/a -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $OUT/a.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES -d $OUT/b -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $OUT/b.log 2>&1
echo rc=$?
