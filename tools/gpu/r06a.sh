#!/bin/bash
# Round 6, first GPU call: the GPU suite on the ABI-7 tree (stage-0 filter on by default at k = 4; bloom-bit
# fixture), smoke(), then two whole-bench A/Bs: the half prefix stream (config B) and the stage-0 filter (config C).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06a}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
ROUNDS=3 bash tools/gpu/bench_ab.sh ${1:-r06a}/half keyhuntm1cpu_amd/lib_half 20 || exit 1
ROUNDS=3 bash tools/gpu/bench_ab.sh ${1:-r06a}/gate0 keyhuntm1cpu_amd/lib_nogate0 20 --k 4 || exit 1
