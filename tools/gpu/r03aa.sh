# Round 3: reduction with per-word 64-bit sums (v_lshl_add_u64) and one carry chain (fm_reduce_w):
# field-op / fused-op / dump / candidate parity, then A/B against the previous product.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan.py tests/test_gpu_search.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc = 0 ] || exit $rc
V=keyhuntm1cpu_amd/lib/variants
JOBS=3072 GATE=1 ROUNDS=4 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_cur.so $V/libkhbsgs_red.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
