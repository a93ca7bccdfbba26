# Round 3: the prefix-scratch stream's cost (scr1: scratch folded to 2 entries per group, timing only),
# with the real gate and with the all-zero 1 KiB gate.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 GATE_ZERO=13 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so $V/libkhbsgs_scr1.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
