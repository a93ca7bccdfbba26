#!/bin/bash
# Energy per instruction class / memory pattern under board-power sampling (tools/microbench/valu_energy.hip).
# Build first (here): make -C tools/microbench valu_energy
set -o pipefail
O=gpurun_out/${1:-energy}; mkdir -p $O
timeout -k 10 300 python3 tools/microbench/valu_energy_run.py 4 | tee $O/valu_energy.jsonl || exit 1
