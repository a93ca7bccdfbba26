# Round 3: one inversion per item vs two, through the product session (two slots in flight, the
# bench's 3072-chunk steps): bench lines alternating the two libraries.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
for r in 1 2; do
  for v in pipe cur; do
    cp $V/libkhbsgs_$v.so $L
    timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${v}_$r.json').read().strip().split(chr(10))[-1]); print('$v', $r, d['value'], d['ms_per_step'], d['roofline']['shader_mhz_avg'])"
  done
done
cp $V/libkhbsgs_pipe.so $L
