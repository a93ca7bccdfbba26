set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 GATE_ZERO=13 PIPE=6 ROUNDS=3 POWER=1 timeout -k 10 900 python3 -u tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so $V/libkhbsgs_scr2.so $V/libkhbsgs_half.so > $O/mem_ab.txt 2>&1 || { tail -20 $O/mem_ab.txt; exit 1; }
tail -8 $O/mem_ab.txt
