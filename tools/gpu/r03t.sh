# Round 3, 3 waves/SIMD product: full GPU suite, config B bench line + kernel trace (trace_union).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 20 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
python3 tools/trace_union.py $O/trace/trace_kernel_trace.csv --steps 20 --bench $O/trace_bench.json > $O/trace_union.json || exit 1
cat $O/bench.json $O/trace_union.json
