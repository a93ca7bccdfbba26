#!/bin/bash
# Round 6: whole-bench A/Bs on the half-stream product: the prefix stream with plain (cached) accesses, and 16 groups per
# work item (two inversions per 16 groups), 3 + 3 alternating runs each.
set -o pipefail
export TMPDIR=/tmp
ROUNDS=3 bash tools/gpu/bench_ab.sh ${1:-r06j}/plainhalf keyhuntm1cpu_amd/lib_plainhalf 20 || exit 1
ROUNDS=3 bash tools/gpu/bench_ab.sh ${1:-r06j}/b16 keyhuntm1cpu_amd/lib_b16 10 || exit 1
