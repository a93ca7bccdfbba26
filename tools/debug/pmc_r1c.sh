export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
rocprofv3 -L > gpurun_out/r1c_counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/pmcA -o pmc --output-format csv -- python3 tools/perf_variants.py $L > gpurun_out/pmcA.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum -d gpurun_out/pmcB -o pmc --output-format csv -- python3 tools/perf_variants.py $L > gpurun_out/pmcB.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmcC -o pmc --output-format csv -- python3 tools/perf_variants.py $L > gpurun_out/pmcC.log 2>&1
echo rc=$?
