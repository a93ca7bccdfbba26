# A/B: F9 walk (product lib) vs the 8 x 32 walk (variant f9w0): timing + VALU / stall counters.
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
V=keyhuntm1cpu_amd/lib/variants/libkhbsgs_f9w0.so
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 300 python3 tools/perf_variants.py $L $V > $O/ab.txt 2>&1 || exit 1
for n in f9 w32; do
  lib=$L; [ $n = w32 ] && lib=$V
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU OccupancyPercent -d $O/$n-a -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-a.log 2>&1 || exit 1
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM -d $O/$n-b -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n-b.log 2>&1 || exit 1
done
echo done
