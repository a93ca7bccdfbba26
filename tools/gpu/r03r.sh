# Round 3: 3 waves/SIMD (168 VGPRs) with and without the paired reduction, vs the 4-wave product.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_w3.so $V/libkhbsgs_w3pair.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
