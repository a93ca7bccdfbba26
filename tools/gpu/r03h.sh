# Round 3: stochastic PC sampling (stall reasons per instruction) of the product and F9 walks.
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
V=keyhuntm1cpu_amd/lib/variants
for n in prod f9; do
  lib=keyhuntm1cpu_amd/lib/libkhbsgs.so; [ $n = f9 ] && lib=$V/libkhbsgs_f9lds3.so
  JOBS=1024 GATE=1 ROUNDS=1 timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d $O/$n -o pcs --output-format csv -- python3 tools/perf_variants.py $lib > $O/$n.log 2>&1
  echo "$n rc=$?"
  ls -la $O/$n | head
done
