# GPU tests, then A/B of the product library against variants at k=1 and k=4 (JOBS filled per k).
# Usage: bash tools/gpu/run_ab2.sh <tag> <variant>...
export TMPDIR=/tmp
TAG=${1:-ab}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
L=keyhuntm1cpu_amd/lib
libs="$L/libkhbsgs.so"
for v in "$@"; do libs="$libs $L/variants/libkhbsgs_$v.so"; done
K=1 JOBS=512 GATE=1 ROUNDS=5 timeout -k 10 400 python -u tools/perf_variants.py $libs > gpurun_out/$TAG/perf_k1.txt 2>&1 || exit $?
K=4 JOBS=2048 GATE=1 ROUNDS=5 timeout -k 10 400 python -u tools/perf_variants.py $libs > gpurun_out/$TAG/perf_k4.txt 2>&1 || exit $?
grep median gpurun_out/$TAG/perf_k1.txt gpurun_out/$TAG/perf_k4.txt
