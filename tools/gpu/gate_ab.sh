#!/bin/bash
# Gate-test change: the gate's GPU parity tests, then the same-process A/B of the product library against
# lib/variants/libkhbsgs_base.so (the previous build), two launches in flight.  Usage: bash tools/gpu/gate_ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-gate_ab}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scan.py tests/test_gpu_search.py tests/test_golden_vectors.py tests/test_gpu_p130.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gate.log 2>&1 || { tail -30 $O/pytest_gate.log; exit 1; }
tail -3 $O/pytest_gate.log
PIPE=6 ROUNDS=${ROUNDS:-7} TAILN=6 bash tools/gpu/ab.sh $TAG keyhuntm1cpu_amd/lib/libkhbsgs.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_base.so
