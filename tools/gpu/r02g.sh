# Round 2: the F9 (9 x 29-bit) product walk: microbench, full GPU suite, bench (queue depth 2).
set -o pipefail
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 120 tools/microbench/fe29bench > $O/fe29bench.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
