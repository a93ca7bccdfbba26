# Round 3: marginal issue cost of each instruction class inside the product walk: 20 padding
# instructions of one kind after every field multiply (4 independent chains), each process
# against the barrier-only control p0 (same code, zero padding).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
run() { JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 300 python3 tools/perf_variants.py $V/libkhbsgs_p0.so $V/libkhbsgs_$1.so $V/libkhbsgs_$2.so > $O/ab_$1_$2.txt 2>&1; }
run mov addu && run addco addc && run madv mads && run mullo add3 && run nop base
grep -h "median" $O/ab_*.txt
