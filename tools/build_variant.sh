#!/bin/bash
# Build one A/B variant of libkhbsgs.so (lib/variants/libkhbsgs_<name>.so) with extra -D flags, its four
# translation units compiled in parallel.  Usage: tools/build_variant.sh <name> [-DKEY=VAL ...]
set -e
NAME=$1; shift
OUT=keyhuntm1cpu_amd/lib/variants
OBJ=build/variants/$NAME
mkdir -p $OUT $OBJ
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value $*"
pids=()
for s in khbsgs k_bsgs k_addr k_baby k_check; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $OBJ/$s.o keyhuntm1cpu_amd/csrc/$s.hip & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc $FLAGS -shared -o $OUT/libkhbsgs_$NAME.so $OBJ/*.o
echo "built $OUT/libkhbsgs_$NAME.so ($*)"
