# Round 3 final tree: config E and C lines, and the PMC passes behind profiles/pmc_latest.json
# (tools/pmc_summary.py): real vs all-zero gate, FETCH_SIZE + EA read requests, WRITE_SIZE + EA write
# requests, SQ instruction counters, over 3072-chunk launches (the bench step).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 300 python bench.py --workload address --steps 3 --warmup 1 --cpu-seconds 20 > $O/bench_address.json 2> $O/bench_address.err || exit 1
timeout -k 10 300 python bench.py --k 4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_k4.json 2> $O/bench_k4.err || exit 1
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
for g in 0 13; do
  JOBS=3072 GATE=1 GATE_ZERO=$g ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum -d $O/pmc_fetch_$g -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_fetch_$g.log 2>&1 || exit 1
done
JOBS=3072 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum -d $O/pmc_write_0 -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_write_0.log 2>&1 || exit 1
JOBS=3072 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_sq.log 2>&1 || exit 1
cat $O/bench_address.json $O/bench_k4.json
