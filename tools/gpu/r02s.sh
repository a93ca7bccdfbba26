# -m address occupancy A/B: 4 (spilling), 3, 2 (no spills) waves per SIMD for the hash kernels.
set -o pipefail
O=gpurun_out/r02s
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
for w in 2 3; do
  LD_LIBRARY_PATH=$V/aw$w timeout -k 10 300 python tools/bench_address.py --search 2 > $O/both_aw$w.json 2> $O/both_aw$w.err || exit 1
  LD_LIBRARY_PATH=$V/aw$w timeout -k 10 300 python tools/bench_address.py --search 1 > $O/compress_aw$w.json 2> $O/compress_aw$w.err || exit 1
done
timeout -k 10 300 python tools/bench_address.py --search 2 > $O/both_aw4.json 2> $O/both_aw4.err
