# -m address with v_bitop3 / v_alignbit hashing: parity tests + config E bench.
set -o pipefail
O=gpurun_out/r02t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_address.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python tools/bench_address.py --search 2 > $O/addr_both.json 2> $O/addr_both.err && \
timeout -k 10 300 python tools/bench_address.py --search 1 > $O/addr_compress.json 2> $O/addr_compress.err
