# Round 3: A/B of the 9 x 29 walk (new column schedule) against the 8 x 32 product, one process,
# 4096-chunk launches (2^34 giant steps, the bench's batch), with the level-0 gate.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 600 python3 tools/perf_variants.py $L $V/libkhbsgs_f9lds4.so $V/libkhbsgs_f9reg3.so > $O/ab.txt 2>&1
echo "rc=$?" >> $O/ab.txt
cat $O/ab.txt
