#!/bin/bash
# Round-end check on the final tree: the GPU suite, smoke() and the driver's bench command.
set -o pipefail
O=gpurun_out/${1:-r05_end}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; p=r['power']; print(d['value'], r['frac'], r['shader_mhz_avg'], p.get('power_w_from_energy'), p.get('ppt_residency_frac'), d['cpu_baseline']['value'], d['cpu_baseline']['spread_pct'])"
