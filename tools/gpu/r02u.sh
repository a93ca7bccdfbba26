# -m address A/B after the bitop3 hashing: occupancy 4 / 2 and the shared 02/03 schedule (ap = pair).
set -o pipefail
O=gpurun_out/r02u
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
for v in aw2 ap4 ap2; do
  for s in 2 1; do
    LD_LIBRARY_PATH=$V/$v timeout -k 10 300 python tools/bench_address.py --search $s > $O/s${s}_$v.json 2> $O/s${s}_$v.err || exit 1
  done
done
timeout -k 10 300 python tools/bench_address.py --search 2 > $O/s2_base.json 2> $O/s2_base.err && \
timeout -k 10 300 python tools/bench_address.py --search 1 > $O/s1_base.json 2> $O/s1_base.err
