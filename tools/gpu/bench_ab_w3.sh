#!/bin/bash
# Same-box bench A/B of the 4-wave product library against a 3-wave build (profiles/r04s): two interleaved
# rounds of bench.py, the 3-wave library picked up by libkhhost through LD_LIBRARY_PATH (RUNPATH $ORIGIN
# yields to it; maps.txt records which libkhbsgs.so was loaded).  Build the 3-wave library first:
#   bash tools/build_variant.sh w3tmp -DKHB_WAVES_PER_SIMD=3 && mkdir -p keyhuntm1cpu_amd/lib/variants/w3 &&
#   mv keyhuntm1cpu_amd/lib/variants/libkhbsgs_w3tmp.so keyhuntm1cpu_amd/lib/variants/w3/libkhbsgs.so
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
W3=keyhuntm1cpu_amd/lib/variants/w3
LD_LIBRARY_PATH=$W3 timeout -k 10 120 python3 -c "
import torch
from keyhuntm1cpu_amd import khhost
khhost.lib()
print([l.split()[-1] for l in open('/proc/self/maps') if 'libkhbsgs' in l][:1])" > $O/maps.txt 2>&1 || exit 1
cat $O/maps.txt
for r in 1 2; do
  echo "[$(date +%T)] round $r"
  timeout -k 10 180 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/w4_$r.json 2> $O/w4_$r.err || exit 1
  LD_LIBRARY_PATH=$W3 timeout -k 10 180 python3 -u bench.py --steps 40 --warmup 5 --chunks 3072 --no-cpu-baseline > $O/w3c3072_$r.json 2> $O/w3c3072_$r.err || exit 1
  LD_LIBRARY_PATH=$W3 timeout -k 10 180 python3 -u bench.py --steps 30 --warmup 5 --chunks 4096 --no-cpu-baseline > $O/w3c4096_$r.json 2> $O/w3c4096_$r.err || exit 1
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); c=d['config']
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('shader_mhz_avg'))"; done
