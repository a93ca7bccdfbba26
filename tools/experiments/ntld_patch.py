# Timing-only patch for tools/experiments/calib_build.sh: the prefix-scratch LOADS non-temporal (KHB_NT_ST=1
# also makes the stores non-temporal).  With a stage-1 gate fold in L2 the stream's read-back is what
# competes with the fold for L2.
import os
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "__device__ __forceinline__ Fe scr_ld(const Fe* p) { return *p; }"
b = """__device__ __forceinline__ Fe scr_ld(const Fe* p) {
  const v4u* q = reinterpret_cast<const v4u*>(p);
  const v4u lo = __builtin_nontemporal_load(q), hi = __builtin_nontemporal_load(q + 1);
  return Fe{{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w}};
}"""
assert a in s
s = s.replace(a, b)
if os.environ.get("KHB_NT_ST") == "1":
    a = "__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) { *p = v; }"
    b = """__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) {
  v4u* q = reinterpret_cast<v4u*>(p);
  __builtin_nontemporal_store(v4u{v.v[0], v.v[1], v.v[2], v.v[3]}, q);
  __builtin_nontemporal_store(v4u{v.v[4], v.v[5], v.v[6], v.v[7]}, q + 1);
}"""
    assert a in s
    s = s.replace(a, b)
open(p, 'w').write(s)
