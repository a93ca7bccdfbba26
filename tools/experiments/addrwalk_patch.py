# Count-only patch for tools/experiments/calib_build.sh: the -m address kernels with
# the hashing removed, so PMC SQ_INSTS_VALU of this build is the x/y walk alone (results wrong by design).
# x and y stay live through a test that never fires, so the walk is not eliminated.
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = """    if constexpr (MODE == kAddrC || MODE == kAddrB) {
#pragma unroll 1
      for (uint32_t pre = 2; pre <= 3; ++pre) {"""
b = """    if ((x.v[0] ^ x.v[5] ^ y.v[0] ^ y.v[3]) == 0x9e3779b9u && x.v[7] == 0x7f4a7c15u) emit(0);
    if constexpr (false) {
#pragma unroll 1
      for (uint32_t pre = 2; pre <= 3; ++pre) {"""
assert a in s
s = s.replace(a, b)
a = """    if constexpr (MODE == kAddrU || MODE == kAddrB) {
      hash160_uncompressed(h, x, y);"""
b = """    if constexpr (false) {
      hash160_uncompressed(h, x, y);"""
assert a in s
s = s.replace(a, b)
open(p, 'w').write(s)
