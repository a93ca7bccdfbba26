# Patch for tools/experiments/calib_build.sh: KHB_BLOCK=n threads per workgroup of the scan kernels
# (default 256 = 4 waves; the lane count stays a multiple of it).
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "constexpr uint32_t kBlock = 256;"
assert a in s
s = s.replace(a, "constexpr uint32_t kBlock = KHB_BLOCK;")
open(p, 'w').write(s)
