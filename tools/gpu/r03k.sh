# Round 3: gate size A/B after the attribution (r03j): the product's 2^28-bit gate vs OR-folds to
# 4 / 2 MiB (L2-sized; more x pass to the level-1 check) vs the all-zero L1-resident reference.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
JOBS=4096 GATE=1 GATE_LOG2S=25,24 GATE_ZERO=13 ROUNDS=3 timeout -k 10 500 python3 tools/perf_variants.py $L > $O/gate_sizes.txt 2>&1
cat $O/gate_sizes.txt | tail -5
