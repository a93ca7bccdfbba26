# Round 3 final tree (3 waves/SIMD, alignbit squaring): full GPU suite, smoke(), config B bench line +
# kernel trace (trace_union), config D line, and a 2-rank rehearsal of the N > 1 path on one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 20 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
python3 tools/trace_union.py $O/trace/trace_kernel_trace.csv --steps 20 --bench $O/trace_bench.json > $O/trace_union.json || exit 1
timeout -k 10 300 python bench.py --workload p130 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_p130.json 2> $O/bench_p130.err || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > $O/n2.json 2> $O/n2.err || exit 1
cat $O/bench.json $O/trace_union.json
