# Gate bit test with 64-bit shifts (product) vs word select + 32-bit shift (gs0).
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
JOBS=4096 GATE=1 ROUNDS=5 timeout -k 10 500 python3 tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_gs0.so > $O/ab.txt 2>&1 && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_search.py tests/test_gpu_p130.py tests/test_gpu_scan.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
