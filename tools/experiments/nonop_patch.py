# Timing-only patch for tools/experiments/calib_build.sh: the carry-hazard pads (KHB_NOP, one
# `s_nop 0` between a VCC write and its carry-in reader) removed from every field-op chain.  The
# results are not guaranteed (the wait state is the ISA's rule); perf_variants skips the parity check.
p = 'keyhuntm1cpu_amd/csrc/device/fe_asm.hpp'
s = open(p).read()
a = '#define KHB_NOP "s_nop 0\\n\\t"'
assert a in s
s = s.replace(a, '#define KHB_NOP ""')
open(p, 'w').write(s)
