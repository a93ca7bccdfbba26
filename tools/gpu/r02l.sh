# F9 walk: centre LDS loads volatile (product) vs plain loop-variant (cnv0) vs the 8 x 32 walk.
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
JOBS=4096 GATE=1 ROUNDS=3 timeout -k 10 500 python3 tools/perf_variants.py keyhuntm1cpu_amd/lib/libkhbsgs.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_cnv0.so keyhuntm1cpu_amd/lib/variants/libkhbsgs_f9w0.so > $O/ab.txt 2>&1
