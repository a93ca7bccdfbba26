#!/bin/bash
# Round 6: 3 vs 4 waves per SIMD on the half-stream product (whole bench, 3 + 3 alternating).
set -o pipefail
export TMPDIR=/tmp
ROUNDS=3 bash tools/gpu/bench_ab.sh ${1:-r06i}/w3 keyhuntm1cpu_amd/lib_w3 20 || exit 1
