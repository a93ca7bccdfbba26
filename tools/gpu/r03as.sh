# Round 3: workgroup size of the scan kernels (64 / 192 / 256 threads) at 3 waves/SIMD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03as
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=3072 GATE=1 ROUNDS=4 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_cur.so $V/libkhbsgs_blk64.so $V/libkhbsgs_blk192.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
