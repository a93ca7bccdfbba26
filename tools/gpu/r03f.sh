# Round 3: F9 walk A/B (p - C.x in registers, C.y in LDS) vs both in LDS vs the 8 x 32 product, plus the
# PMC VALU count of the register variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 600 python3 tools/perf_variants.py $L $V/libkhbsgs_f9lds3.so $V/libkhbsgs_f9lds2.so > $O/ab.txt 2>&1 || exit 1
JOBS=2048 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES VALUBusy -d $O/lds2 -o pmc --output-format csv -- python3 tools/perf_variants.py $V/libkhbsgs_f9lds2.so > $O/lds2.log 2>&1
cat $O/ab.txt | tail -4
