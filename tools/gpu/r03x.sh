# Round 3: squaring with the cross sum doubled by v_alignbit and one carry chain (fe_asm.hpp
# fm_sqr512x): field-op / dump / candidate parity, then A/B against the 3-wave product before it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc = 0 ] || exit $rc
V=keyhuntm1cpu_amd/lib/variants
JOBS=3072 GATE=1 ROUNDS=4 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base3.so $V/libkhbsgs_sq1.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
