# Round 3: shader clock of the product (8 x 32) and F9 walks under the same 4096-chunk launches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 600 python3 tools/perf_variants.py $L $V/libkhbsgs_f9lds3.so > $O/ab.txt 2>&1
cat $O/ab.txt | tail -3
