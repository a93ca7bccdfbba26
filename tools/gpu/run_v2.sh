export TMPDIR=/tmp
mkdir -p gpurun_out/v2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v2/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=keyhuntm1cpu_amd/lib
JOBS=512 GATE=1 ROUNDS=5 timeout -k 10 400 python -u tools/perf_variants.py $L/variants/libkhbsgs_base.so $L/libkhbsgs.so $L/variants/libkhbsgs_q1.so $L/variants/libkhbsgs_q2.so $L/variants/libkhbsgs_q3.so $L/variants/libkhbsgs_b8.so > gpurun_out/v2/perf.txt 2>&1
echo "perf rc=$?"
tail -8 gpurun_out/v2/perf.txt
tail -3 gpurun_out/v2/pytest.log
