#!/bin/bash
# the v_fma_f64 field product, verified against Python big ints, then timed against fm_mul
# under board-power sampling.  Build first (here): make -C tools/microbench f64mul
set -o pipefail
O=gpurun_out/${1:-f64}
mkdir -p $O
timeout -k 10 60 tools/microbench/f64mul verify 65536 $O/f64mul_verify.bin > $O/verify.log 2>&1 || exit 1
python3 tools/microbench/f64mul_check.py $O/f64mul_verify.bin | tee $O/verify_check.json || exit 1
timeout -k 10 120 python3 tools/microbench/f64mul_run.py 5 | tee $O/f64mul_time.jsonl || exit 1
