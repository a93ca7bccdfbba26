# Round-2 evidence: config B bench + kernel trace + HBM and VALU PMC passes (tools/profile_bench.sh),
# then config E (-l both): kernel trace and the VALU pass of the address kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02w
bash tools/profile_bench.sh r02w && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/addr_trace -o trace --output-format csv -- python3 tools/bench_address.py --search 2 --chunks 8 > $O/addr_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU OccupancyPercent -d $O/addr_valu -o valu --output-format csv -- python3 tools/bench_address.py --search 2 --chunks 8 > $O/addr_valu.log 2>&1
