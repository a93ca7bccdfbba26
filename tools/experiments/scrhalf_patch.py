# Timing-only patch for tools/experiments/calib_build.sh (round 6): the half prefix stream (the product) with plain
# loads and stores (plainscr_patch.py) folded to (i & KHB_SCR_MASK) entries per group, so that it stays in the caches:
# with the all-zero gate of tools/perf_variants.py (GATE_ZERO=13) this is the zero-memory build of the current product,
# the compute-only energy per giant step of VERDICT r5 item 5.  Results are wrong by design (the walk reads the wrong
# prefixes); perf_variants skips their parity check (TIMING_ONLY).
import os
import runpy
here = os.path.dirname(os.path.abspath(__file__))
runpy.run_path(os.path.join(here, "plainscr_patch.py"))
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "if (i > 2) pre = scr_ld(scr + (size_t)(i - 3) * S);"
assert a in s
s = s.replace(a, "if (i > 2) pre = scr_ld(scr + (size_t)((i - 3) & KHB_SCR_MASK) * S);")
a = "Fe pre = scr_ld(scr + (size_t)(kHalf - 3) * S);          // P_509"
assert a in s
s = s.replace(a, "Fe pre = scr_ld(scr + (size_t)((kHalf - 3) & KHB_SCR_MASK) * S);")
a = "if (!(kHalfStream && is_gated(MODE)) || (i & 1u)) scr_st(sg + i * S, a);"
assert a in s
s = s.replace(a, "if (!(kHalfStream && is_gated(MODE)) || (i & 1u)) scr_st(sg + (i & KHB_SCR_MASK) * S, a);")
open(p, 'w').write(s)
