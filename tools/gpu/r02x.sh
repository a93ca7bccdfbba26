# A/B: kScanG with x1's gate load issued before x2 is computed (KHB_GATE_EARLY=1) vs the product.
set -o pipefail
O=gpurun_out/r02x
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/base$r.json 2> $O/base$r.err || exit 1
  LD_LIBRARY_PATH=$V/ge1 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/early$r.json 2> $O/early$r.err || exit 1
done
