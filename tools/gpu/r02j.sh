# F9 walk with the centre in LDS (no spills in the walk) vs the 8 x 32 walk; then the GPU suite.
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $L keyhuntm1cpu_amd/lib/variants/libkhbsgs_f9w0.so > $O/ab.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
