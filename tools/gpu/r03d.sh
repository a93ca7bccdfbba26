# Round 3: SQ counters of the product (8 x 32) and F9 walks, one perf_variants launch set each
# (JOBS=2048 chunks, gate on), to attribute the F9 walk's lower issue rate.
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
rocprofv3 -L > $O/avail.txt 2>&1 || true
V=keyhuntm1cpu_amd/lib/variants
for n in prod f9; do
  lib=keyhuntm1cpu_amd/lib/libkhbsgs.so; [ $n = f9 ] && lib=$V/libkhbsgs_f9lds4.so
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $O/$n-a -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-a.log 2>&1 || exit 1
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d $O/$n-b -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-b.log 2>&1 || exit 1
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc VALUBusy VALUUtilization GRBM_GUI_ACTIVE -d $O/$n-c -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-c.log 2>&1 || exit 1
done
echo done
