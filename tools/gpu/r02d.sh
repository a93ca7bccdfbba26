# Round 2: full GPU suite on the two-slot build, then the tail-overlap A/B (queue depth 1 vs 2).
set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log
grep -q "passed" $O/pytest.log || exit 1
KHB_QUEUE_DEPTH=1 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_q1.json 2> $O/bench_q1.err && \
KHB_QUEUE_DEPTH=2 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_q2.json 2> $O/bench_q2.err
