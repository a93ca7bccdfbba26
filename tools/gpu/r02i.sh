# A/B: F9 walk at 4 waves/SIMD (product, spills) vs 3 waves/SIMD vs the 8 x 32 walk.
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 400 python3 tools/perf_variants.py $L keyhuntm1cpu_amd/lib/variants/libkhbsgs_w3.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_f9w0.so > $O/ab.txt 2>&1
