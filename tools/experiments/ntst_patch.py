# Timing-only patch for tools/experiments/calib_build.sh: the prefix-scratch STORES non-temporal, the loads
# plain (round 1 measured both non-temporal slower; this isolates the stores, which are read back ~512 walk
# steps later from HBM anyway and otherwise pass through L2 / the Infinity Cache beside the gate).
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) { *p = v; }"
b = """__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) {
  v4u* q = reinterpret_cast<v4u*>(p);
  __builtin_nontemporal_store(v4u{v.v[0], v.v[1], v.v[2], v.v[3]}, q);
  __builtin_nontemporal_store(v4u{v.v[4], v.v[5], v.v[6], v.v[7]}, q + 1);
}"""
assert a in s
s = s.replace(a, b)
open(p, 'w').write(s)
