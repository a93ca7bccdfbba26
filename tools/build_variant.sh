#!/bin/bash
# Build one A/B variant of libkhbsgs.so (lib/variants/libkhbsgs_<name>.so) with extra -D flags, its translation
# units compiled in parallel.  The build names itself in khb_build_info (variant=<name>, defines=<flags>), so a
# bench line taken on it says so (bench.py refuses it without --variant).
# Usage: tools/build_variant.sh <name> [-DKEY=VAL ...]
#   LIBDIR=1 also writes keyhuntm1cpu_amd/lib_<name>/ (this libkhbsgs.so + a copy of the in-tree libkhhost.so,
#   which finds it through its $ORIGIN rpath) for a whole-bench A/B: KHB_LIB_DIR=... bench.py --variant <name>.
set -e
NAME=$1; shift
OUT=keyhuntm1cpu_amd/lib/variants
OBJ=build/variants/$NAME
mkdir -p $OUT $OBJ
DEFS=$(echo "$*" | tr ' ' ',')
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value $* -DKHB_VARIANT=\"$NAME\" -DKHB_BUILD_DEFINES=\"$DEFS\""
pids=()
for s in khbsgs k_bsgs k_addr k_addr_e k_baby k_check; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $OBJ/$s.o keyhuntm1cpu_amd/csrc/$s.hip & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc $FLAGS -shared -o $OUT/libkhbsgs_$NAME.so $OBJ/*.o
echo "built $OUT/libkhbsgs_$NAME.so ($*)"
if [ -n "$LIBDIR" ]; then
  D=keyhuntm1cpu_amd/lib_$NAME
  mkdir -p $D
  cp $OUT/libkhbsgs_$NAME.so $D/libkhbsgs.so
  cp keyhuntm1cpu_amd/lib/libkhhost.so $D/libkhhost.so
  echo "wrote $D (KHB_LIB_DIR=$D python bench.py --variant $NAME)"
fi
