#!/bin/bash
# khb_stats.event_ms (ABI 6) on the GPU: the suite, then the trace pass of round_profile.sh, whose
# trace_union.json compares rocprofv3's per-launch duration with the bench line's kernel_event_ms_avg.
set -o pipefail
O=gpurun_out/${1:-r05p}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
PARTS=trace bash tools/gpu/round_profile.sh ${1:-r05p}/prof 20
