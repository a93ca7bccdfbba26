# Timing-only patch for tools/experiments/calib_build.sh: KHB_SCR_MASK=m folds the prefix-scratch
# index of the forward pass and the walk to (i & m), so the 16 B + 16 B per giant step of prefix
# traffic stays in a few entries per group (MALL/L2-resident) instead of streaming through HBM.
# Results are wrong by design (the walk reads the wrong prefixes).
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "pre = scr_ld(scr + (size_t)(i >= 2 ? i - 2 : 0) * S);"
b = "pre = scr_ld(scr + (size_t)((i >= 2 ? i - 2 : 0) & KHB_SCR_MASK) * S);"
assert a in s; s = s.replace(a, b)
a = "scr_st(sg + i * S, a);"
b = "scr_st(sg + (i & KHB_SCR_MASK) * S, a);"
assert a in s; s = s.replace(a, b)
open(p, 'w').write(s)
