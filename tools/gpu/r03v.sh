# Round 3: the carry-hazard pads' cost at 3 waves/SIMD (timing-only build without them).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=3072 GATE=1 ROUNDS=4 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base3.so $V/libkhbsgs_w3nonop.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
