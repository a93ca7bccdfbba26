# Round 3: instruction fetch and VALU-mix counters of the product and F9 walks.
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
for n in prod f9; do
  lib=keyhuntm1cpu_amd/lib/libkhbsgs.so; [ $n = f9 ] && lib=$V/libkhbsgs_f9lds3.so
  JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_WAVE_CYCLES -d $O/$n -o pmc --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n.log 2>&1 || exit 1
done
echo done
