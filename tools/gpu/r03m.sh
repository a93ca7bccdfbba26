# Round 3: issue-cost calibration inside the product walk: +20 v_mov / 4x5 independent v_mad per field
# multiply, each against its barrier-only control (same code, no padding).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_bar1.so $V/libkhbsgs_mov20.so > $O/ab_mov.txt 2>&1 &&
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_bar2.so $V/libkhbsgs_mad20i.so > $O/ab_mad.txt 2>&1
tail -3 $O/ab_mov.txt $O/ab_mad.txt
