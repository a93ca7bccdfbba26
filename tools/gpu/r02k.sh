# PMC of the F9 walk (product) vs the 8 x 32 walk (f9w0): VALU issue, LDS / SALU / VMEM instruction counts, waits.
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
V=keyhuntm1cpu_amd/lib/variants/libkhbsgs_f9w0.so
for n in f9 w32; do
  lib=$L; [ $n = w32 ] && lib=$V
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $O/$n-a -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-a.log 2>&1 || exit 1
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $O/$n-b -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-b.log 2>&1 || exit 1
done
echo done
