# Timing-only patch for tools/experiments/calib_build.sh: the prefix-scratch stream with plain loads and stores
# (the product's are non-temporal since round 4, scan_kernels.hpp scr_st / scr_ld).
import re
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
pat = re.compile(r"__device__ __forceinline__ void scr_st\(Fe\* p, const Fe& v\) \{.*?\n\}\n"
                 r"__device__ __forceinline__ Fe scr_ld\(const Fe\* p\) \{.*?\n\}\n", re.S)
assert pat.search(s)
s = pat.sub("__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) { *p = v; }\n"
            "__device__ __forceinline__ Fe scr_ld(const Fe* p) { return *p; }\n", s, count=1)
open(p, 'w').write(s)
