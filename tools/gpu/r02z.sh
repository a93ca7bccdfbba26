# Round-2 closing check: full GPU suite + smoke on the final tree.
set -o pipefail
O=gpurun_out/r02z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/pytest.log; cat $O/smoke.log
exit $rc
