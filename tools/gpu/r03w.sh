# Round 3: the 9 x 29-bit walk at 3 waves/SIMD (registers to spare), centre words in registers or LDS.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=3072 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base3.so $V/libkhbsgs_f9w3reg.so $V/libkhbsgs_f9w3lds.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
