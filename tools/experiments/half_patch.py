# Timing-only patch for tools/experiments/calib_build.sh: the half prefix stream (tools/experiments/half_stream.hpp).
# The forward pass stores only the odd prefixes; walk_group_g_half rebuilds the even ones (one extra product per two
# walk steps).  Exact: perf_variants compares its candidates with the product's.
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "// One reference group centred on C, walked on its own"
assert a in s
s = s.replace(a, '#include "../../tools/experiments/half_stream.hpp"\n\n' + a, 1)
a = "    scr_st(sg, a);\n"
assert a in s
s = s.replace(a, "    if (!is_gated(MODE)) scr_st(sg, a);\n", 1)
a = "      scr_st(sg + i * S, a);\n"
assert a in s
s = s.replace(a, "      if (!is_gated(MODE) || (i & 1u)) scr_st(sg + i * S, a);\n", 1)
a = "    if constexpr (is_gated(MODE))\n      walk_group_g<"
assert a in s
s = s.replace(a, "    if constexpr (is_gated(MODE))\n      walk_group_g_half<", 1)
open(p, 'w').write(s)
