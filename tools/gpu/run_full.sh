# GPU-box round check: GPU tests, smoke, then bench + rocprof stats + HBM PMC passes (tools/profile_bench.sh).
# Usage (under gpurun, from the repo root): bash tools/gpu/run_full.sh <tag> [bench args...]
export TMPDIR=/tmp
TAG=${1:-full}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
bash tools/profile_bench.sh ${TAG}prof "$@"
