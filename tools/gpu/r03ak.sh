# Round 3: one inversion per work item (the next item's centre x-differences ride in this item's
# inversion): GPU parity suite, then A/B against the two-inversion build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ak
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc = 0 ] || exit $rc
V=keyhuntm1cpu_amd/lib/variants
JOBS=3072 GATE=1 ROUNDS=4 timeout -k 10 400 python3 tools/perf_variants.py $V/libkhbsgs_cur.so $V/libkhbsgs_pipe.so > $O/ab.txt 2>&1
grep -h median $O/ab.txt
