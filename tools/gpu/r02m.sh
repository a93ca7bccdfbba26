# Product back on the 8 x 32 walk; F9 library parity; full GPU suite; bench.
set -o pipefail
O=gpurun_out/r02m
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
