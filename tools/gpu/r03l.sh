# Round 3: deferred gate test (test one walk step after the load) vs the round's base, + zero-gate ceiling.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 GATE_ZERO=13 ROUNDS=3 timeout -k 10 600 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_defer.so > $O/ab.txt 2>&1
cat $O/ab.txt | tail -5
