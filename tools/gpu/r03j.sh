# Round 3 final-tree evidence: full GPU suite, config B bench line + kernel trace (trace_union), config E
# bench line, and the gate attribution (verdict r2 item 4): the product with its 2^28-bit gate vs an
# all-zero 2^13-bit gate (same instructions, every gate load an L1 hit), timed and under PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 20 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
python3 tools/trace_union.py $O/trace/trace_kernel_trace.csv --steps 20 --bench $O/trace_bench.json > $O/trace_union.json || exit 1
timeout -k 10 300 python bench.py --workload address --steps 3 --warmup 1 --cpu-seconds 20 > $O/bench_address.json 2> $O/bench_address.err || exit 1
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
JOBS=4096 GATE=1 GATE_ZERO=13 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $L > $O/gate_ab.txt 2>&1 || exit 1
for g in 0 13; do
  JOBS=2048 GATE=1 GATE_ZERO=$g ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $O/pmc_tcc_$g -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_tcc_$g.log 2>&1 || exit 1
  JOBS=2048 GATE=1 GATE_ZERO=$g ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $O/pmc_sq_$g -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/pmc_sq_$g.log 2>&1 || exit 1
done
echo done
