# Round 3: paired-high-word reduction (fe_asm.hpp fm_reduce_pair): field-op / dump / candidate parity,
# then A/B against the round's base build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc = 0 ] || exit $rc
V=keyhuntm1cpu_amd/lib/variants
JOBS=4096 GATE=1 ROUNDS=4 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_base.so keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
