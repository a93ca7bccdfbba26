# GPU A/B timing only (no tests): tools/perf_variants.py over the product library and variants.
# Usage: JOBS=.. ROUNDS=.. bash tools/gpu/run_perf.sh <tag> <variant>...
export TMPDIR=/tmp
TAG=${1:-perf}; shift
mkdir -p gpurun_out/$TAG
L=keyhuntm1cpu_amd/lib
libs="$L/libkhbsgs.so"
for v in "$@"; do libs="$libs $L/variants/libkhbsgs_$v.so"; done
JOBS=${JOBS:-512} GATE=1 ROUNDS=${ROUNDS:-5} timeout -k 10 500 python -u tools/perf_variants.py $libs > gpurun_out/$TAG/perf.txt 2>&1
prc=$?
grep median gpurun_out/$TAG/perf.txt
exit $prc
