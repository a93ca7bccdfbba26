#!/bin/bash
# Round 6: the GPU suite on the tree with the 32 MiB k=4 fold default, config C's line, and the executed VALU per key of
# the -e address kernel (-l both -e, two chunks) and of the plain one, for the -e line's roofline.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06h}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench_k4
timeout -k 10 400 python3 bench.py --k 4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_k4.json 2> $O/bench_k4.err || { tail -20 $O/bench_k4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k4.json')); print('k4', d['value'], d['roofline']['shader_mhz_avg'])"
for s in 6 2; do
  step "pmc address search=$s"
  SEARCH=$s CHUNKS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/addr_s$s -o pmc --output-format csv -- python3 tools/addr_floor.py keyhuntm1cpu_amd/lib/libkhbsgs.so > $O/addr_s$s.json 2> $O/addr_s$s.err || { tail -5 $O/addr_s$s.err; exit 1; }
  cat $O/addr_s$s.json
done
step done
