set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u -m pytest tests/test_gpu_address.py -k unsolved -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r02c/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/r02c/bench_p66.json 2> gpurun_out/r02c/bench_p66.err && \
timeout -k 10 300 python bench.py --workload p130 --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/r02c/bench_p130.json 2> gpurun_out/r02c/bench_p130.err
