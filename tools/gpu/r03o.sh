# Round 3: timing-only removal of existing work from the field ops (results wrong by design):
# rmfold = the product's 15-add column fold as xors, rmt = fm_reduce's 9-add T chain as xors,
# rmp = the reduction's 8 977*H mads as full-rate ops.  Marginal value of removing H-class ops.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 300 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_rmfold.so $V/libkhbsgs_rmt.so > $O/ab1.txt 2>&1 &&
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 300 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_rmp.so $V/libkhbsgs_p0.so > $O/ab2.txt 2>&1
grep -h median $O/ab1.txt $O/ab2.txt
