# Config E bench lines under rocprofv3 kernel trace (same command: the JSON's kernel_ms_avg and the
# trace's average duration of k_giant_scan<4>/<3> come from one run).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02za
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/both -o trace --output-format csv -- python3 tools/bench_address.py --search 2 > $O/both.json 2> $O/both.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/compress -o trace --output-format csv -- python3 tools/bench_address.py --search 1 > $O/compress.json 2> $O/compress.err
