# GPU A/B: GPU tests on the product library, then tools/perf_variants.py over the product and the
# variants named on the command line (keyhuntm1cpu_amd/lib/variants/libkhbsgs_<name>.so).
# Usage: bash tools/gpu/run_ab.sh <tag> <variant>...
export TMPDIR=/tmp
TAG=${1:-ab}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=keyhuntm1cpu_amd/lib
libs="$L/libkhbsgs.so"
for v in "$@"; do libs="$libs $L/variants/libkhbsgs_$v.so"; done
JOBS=${JOBS:-512} GATE=1 ROUNDS=${ROUNDS:-5} timeout -k 10 400 python -u tools/perf_variants.py $libs > gpurun_out/$TAG/perf.txt 2>&1
prc=$?
cat gpurun_out/$TAG/perf.txt | grep median
exit $(( rc > prc ? rc : prc ))
