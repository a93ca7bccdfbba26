# Round 3: occupancy 4 / 3 / 2 waves per SIMD, and at 3 the gate tested one walk step after its loads
# (pending x pair in registers; candidates must equal the product's).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_w3.so $V/libkhbsgs_w3defer.so > $O/ab1.txt 2>&1 &&
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_w2.so $V/libkhbsgs_w3defer.so > $O/ab2.txt 2>&1
grep -h median $O/ab1.txt $O/ab2.txt
